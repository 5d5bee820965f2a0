"""svdformer_pointsea_amd -- MI355X-native (gfx950) implementation of the
SVDFormer / PointSea per-batch completion hot path.

Drop-in modules mirroring the reference's operator API:
  svdformer_pointsea_amd.pointnet2_utils  <- pointnet2_ops.pointnet2_utils
  svdformer_pointsea_amd.chamfer3D        <- metrics.CD.chamfer3D.dist_chamfer_3D
  svdformer_pointsea_amd.emd_module       <- metrics.EMD.emd_module
  svdformer_pointsea_amd.model_utils      <- models/model_utils.py hot-path pieces
  svdformer_pointsea_amd.attention        <- self/cross_attention, SDG_Decoder (model_utils.py)
  svdformer_pointsea_amd.render           <- PCViews (model_utils.py), PCViews_Real (mv_utils_zs.py)
  svdformer_pointsea_amd.svdformer        <- models/SVDFormer.py + utils/loss_utils.get_loss
All compute runs in libpcops.so (include/pcops.h); there is no CPU fallback.
"""
from ._lib import LIB_PATH, lib  # noqa: F401

__all__ = ["LIB_PATH", "lib"]
