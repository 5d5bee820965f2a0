"""Whole-model golden vectors from the REFERENCE's own model code
(models/SVDFormer.py, models_PointSea/PointSea.py), run in the build
container only; only the .npz output is committed.

  models.npz
    svd_keys / svd_shapes     the reference SVDFormer Model(cfg_pcn) state_dict
    ps_keys / ps_shapes       the reference PointSea Model(cfg_55) state_dict
    svd_partial, svd_out{0,1,2}   eval-mode forward on a seeded (2,2048,3) cloud
    ps_partial,  ps_out{0,1,2}    (PCViews depth for SVDFormer, PCViews_Real for PointSea)
  Weights: tests/golden/weights.py fill_state(seed) in sorted-key order, so any
  module tree with the same keys and shapes gets the same values.

The reference's CUDA-only ops are replaced by this repo's CPU restatement of
their .cu files (oracle/pcops_oracle.c: FPS, gather, group, Chamfer), which
is pinned on its own by tests/test_oracle.py.  torchvision (absent) is
stubbed: resnet18 is the reference's own models/resnet.py constructor with
pretrained=False (the ImageNet weights are a remote fetch), torch_scatter's
max as in make_golden.py.  Usage:  python tests/golden/make_golden_models.py
"""
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
from weights import fill_state  # noqa: E402

from oracle import oracle as O  # noqa: E402


def _np(t):
    return t.detach().float().contiguous().numpy()


def _stubs():
    p2 = types.ModuleType("pointnet2_ops")
    p2u = types.ModuleType("pointnet2_ops.pointnet2_utils")
    p2u.furthest_point_sample = lambda xyz, n: torch.from_numpy(O.furthest_point_sample(_np(xyz), int(n)))
    p2u.gather_operation = lambda f, idx: torch.from_numpy(O.gather_operation(_np(f), idx.numpy()))
    p2u.grouping_operation = lambda f, idx: torch.from_numpy(O.grouping_operation(_np(f), idx.int().numpy()))

    def _unavailable(*a, **k):
        raise RuntimeError("not reached by the models")

    p2u.ball_query = p2u.three_nn = p2u.three_interpolate = _unavailable
    p2.pointnet2_utils = p2u
    sys.modules["pointnet2_ops"] = p2
    sys.modules["pointnet2_ops.pointnet2_utils"] = p2u

    cd = types.ModuleType("metrics.CD.chamfer3D.dist_chamfer_3D")

    class chamfer_3DDist(torch.nn.Module):
        def forward(self, a, b):
            d1, d2, i1, i2 = O.chamfer_forward(_np(a), _np(b))
            return torch.from_numpy(d1), torch.from_numpy(d2), torch.from_numpy(i1), torch.from_numpy(i2)

    cd.chamfer_3DDist = chamfer_3DDist
    for name in ["metrics", "metrics.CD", "metrics.CD.chamfer3D"]:
        sys.modules[name] = types.ModuleType(name)
    sys.modules["metrics.CD.chamfer3D.dist_chamfer_3D"] = cd

    ts = types.ModuleType("torch_scatter")
    ts.scatter = lambda src, index, dim=-1, out=None, reduce="sum": out.scatter_reduce_(dim, index, src, "amax",
                                                                                        include_self=True)
    sys.modules["torch_scatter"] = ts

    tv = types.ModuleType("torchvision")
    tvm = types.ModuleType("torchvision.models")
    tvu = types.ModuleType("torchvision.models.utils")
    tvu.load_state_dict_from_url = _unavailable
    tv.models = tvm
    tvm.utils = tvu
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = tvm
    sys.modules["torchvision.models.utils"] = tvu

    class ResNet18_Weights:
        IMAGENET1K_V1 = None

    def resnet18(weights=None, **k):
        from models.resnet import resnet18 as ref_resnet18
        return ref_resnet18(pretrained=False)

    tvm.resnet18, tvm.ResNet18_Weights = resnet18, ResNet18_Weights
    tvm.__all__ = ["resnet18", "ResNet18_Weights"]
    torch.Tensor.cuda = lambda self, *a, **k: self
    torch.nn.Module.cuda = lambda self, *a, **k: self


class _Cfg:
    def __init__(self, **net):
        self.NETWORK = types.SimpleNamespace(**net)
        self.DATASET = types.SimpleNamespace(TEST_DATASET="ShapeNet")


PCN = dict(step1=4, step2=8, merge_points=512, local_points=512, view_distance=0.7, USE_PCSA=True)
S55 = dict(step1=2, step2=4, merge_points=1024, local_points=1024, view_distance=1.5, USE_PCSA=True)
SEED_SVD, SEED_PS = 101, 202


def partial_cloud(seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(2, 2048, 3, generator=g) - 0.5) * 0.9


def main():
    _stubs()
    sys.path.insert(0, REF)
    out = {}
    torch.manual_seed(0)
    from models.model_utils import PCViews
    from models.SVDFormer import Model as SVD
    m = fill_state(SVD(_Cfg(**PCN)), SEED_SVD).eval()
    sd = m.state_dict()
    out["svd_keys"] = np.array(sorted(sd))
    out["svd_shapes"] = np.array([str(tuple(sd[k].shape)) for k in sorted(sd)])
    x = partial_cloud(1)
    with torch.no_grad():
        depth = PCViews(TRANS=-PCN["view_distance"], RESOLUTION=224).get_img(x).unsqueeze(1)
        y = m(x, depth)
    out["svd_partial"] = x.numpy()
    for i, t in enumerate(y):
        out[f"svd_out{i}"] = t.numpy()

    from models_PointSea.mv_utils_zs import PCViews_Real
    from models_PointSea.PointSea import Model as PS
    m = fill_state(PS(_Cfg(**S55)), SEED_PS).eval()
    sd = m.state_dict()
    out["ps_keys"] = np.array(sorted(sd))
    out["ps_shapes"] = np.array([str(tuple(sd[k].shape)) for k in sorted(sd)])
    x = partial_cloud(2)
    with torch.no_grad():
        depth = PCViews_Real(TRANS=-S55["view_distance"]).get_img(x)
        y = m(x, depth)
    out["ps_partial"] = x.numpy()
    for i, t in enumerate(y):
        out[f"ps_out{i}"] = t.numpy()
    np.savez_compressed(os.path.join(HERE, "models.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
