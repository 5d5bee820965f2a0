"""Hot-path pieces of models/model_utils.py (and models_PointSea/model_utils.py)
re-expressed on libpcops.so.  Names and signatures follow the reference so
its model classes can import them unchanged:

  query_knn(nsample, xyz, new_xyz, include_self=True)   model_utils.py:281-286
  query_knn_point(k, xyz, new_xyz)                      :807-810
  group_local(xyz, k=20, return_idx=False)              :812-826
  index_points(points, idx)                             :828-845
  fps_subsample(pcd, n_points=2048)                     :489-499
  sample_and_group_knn(xyz, points, npoint, k, ...)     :323-356
  self_attention / cross_attention / SDG_Decoder        :542-629
  self_attention_woinp / SDG_Decoder_PointSea           models_PointSea/model_utils.py:463-509
  PCViews                                               :1179-1234
"""
import numpy as np
import torch
from torch import nn

from ._lib import call, lib, ptr, require_float, stream_of
from .pointnet2_utils import furthest_point_sample, gather_operation, grouping_operation


def _knn(q, p, k, pad=0, want_dist=False):
    """K nearest of p for every row of q; q (B,S,C), p (B,N,C) fp32 on the GPU."""
    q = q.float().contiguous()  # distances are evaluated in fp32 (also under autocast)
    p = p.float().contiguous()
    require_float(q, "new_xyz")
    require_float(p, "xyz")
    B, S, C = q.shape
    N = p.shape[1]
    if p.shape[0] != B or p.shape[2] != C:
        raise RuntimeError(f"knn: shape mismatch {tuple(q.shape)} vs {tuple(p.shape)}")
    if k + pad > N:
        raise RuntimeError(f"selected index k out of range (k={k + pad}, N={N})")
    idx = torch.empty(B, S, k, dtype=torch.int32, device=q.device)
    dist = torch.empty(B, S, k, dtype=torch.float32, device=q.device) if want_dist else None
    with torch.cuda.device(q.device):
        call("knn", lib().pcops_knn, ptr(q), ptr(p), B, S, N, C, k, pad, ptr(idx), ptr(dist), stream_of(q))
    return (idx, dist) if want_dist else idx


def query_knn(nsample, xyz, new_xyz, include_self=True):
    """Find k-NN of new_xyz in xyz -> (B,S,nsample) int32 (model_utils.py:281-286)."""
    pad = 0 if include_self else 1
    return _knn(new_xyz, xyz, nsample, pad)


def query_knn_point(k, xyz, new_xyz):
    """(B,S,k) int64 like torch.topk (model_utils.py:807-810)."""
    return _knn(new_xyz, xyz, k).long()


def index_points(points, idx):
    """points (B,N,C), idx (B,S[,K]) -> (B,S[,K],C) (model_utils.py:828-845)."""
    B, N, C = points.shape
    shp = idx.shape
    idx3 = idx.reshape(B, -1, 1).to(torch.int32).contiguous()
    g = grouping_operation(points.transpose(1, 2).contiguous(), idx3)  # (B,C,S*K,1)
    return g.reshape(B, C, *shp[1:]).movedim(1, -1)


def group_local(xyz, k=20, return_idx=False):
    """xyz (B,C,N) -> (B,C,N,k) neighbour features (model_utils.py:812-826)."""
    xyz = xyz.contiguous()
    pts = xyz.transpose(2, 1).contiguous()
    idx32 = _knn(pts, pts, k)
    group_xyz = grouping_operation(xyz, idx32)
    if return_idx:
        return group_xyz, idx32.long()
    return group_xyz


def fps_subsample(pcd, n_points=2048):
    """pcd (B,N,3) -> (B,n_points,3) (model_utils.py:489-499)."""
    new_pcd = gather_operation(pcd.permute(0, 2, 1).contiguous(), furthest_point_sample(pcd.contiguous(), n_points))
    return new_pcd.permute(0, 2, 1).contiguous()


def sample_and_group_knn(xyz, points, npoint, k, use_xyz=True, idx=None):
    """model_utils.py:323-356: FPS -> gather -> kNN -> group (xyz, points)."""
    xyz_flipped = xyz.permute(0, 2, 1).contiguous()
    new_xyz = gather_operation(xyz, furthest_point_sample(xyz_flipped, npoint))
    if idx is None:
        idx = query_knn(k, xyz_flipped, new_xyz.permute(0, 2, 1).contiguous())
    grouped_xyz = grouping_operation(xyz, idx)
    grouped_xyz -= new_xyz.unsqueeze(3).repeat(1, 1, 1, k)
    if points is not None:
        grouped_points = grouping_operation(points, idx)
        new_points = torch.cat([grouped_xyz, grouped_points], 1) if use_xyz else grouped_points
    else:
        new_points = grouped_xyz
    return new_xyz, new_points, idx, grouped_xyz
