"""CPU execution of the SVDFormer PCN train step for bench.py's cpu_baseline.

TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg, tests/).  The
reference's point ops are CUDA-only (their CPU branches assert, e.g.
pointnet2_ops/_ext-src/src/sampling.cpp:82-84), so "the reference's CPU
path" is its model code driven by CPU versions of those ops.  Here that is
the package's own model (svdformer_pointsea_amd.svdformer, a restatement of
models/SVDFormer.py) with the HIP entry points swapped, for the duration of
a `with cpu_ops():` block, for:

  * the C restatement in oracle/pcops_oracle.c (FPS, gather, group, kNN,
    Chamfer, depth splat) -- single-threaded C, as the checker is;
  * torch CPU math for the attention core and the attention blocks' fused
    LayerNorm / transpose glue (what the reference's torch modules do on CPU).

Everything else (convolutions, LayerNorm, Adam) is torch on CPU threads.
The product package never imports this module; outside the `with` block the
package's HIP path is untouched.
"""
import contextlib

import torch
from torch.autograd import Function

from . import oracle as O


def _np(t):
    return t.detach().float().contiguous().numpy()


class _FPS(Function):
    @staticmethod
    def forward(ctx, xyz, npoint):
        idx = torch.from_numpy(O.furthest_point_sample(_np(xyz), int(npoint)))
        ctx.mark_non_differentiable(idx)
        return idx

    @staticmethod
    def backward(ctx, g):
        return None, None


class _Gather(Function):
    @staticmethod
    def forward(ctx, features, idx):
        ctx.save_for_backward(idx)
        ctx.n = features.shape[2]
        return torch.from_numpy(O.gather_operation(_np(features), idx.numpy()))

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        return torch.from_numpy(O.gather_operation_grad(_np(g), idx.numpy(), ctx.n)), None


class _Group(Function):
    @staticmethod
    def forward(ctx, features, idx):
        ctx.save_for_backward(idx)
        ctx.n = features.shape[2]
        return torch.from_numpy(O.grouping_operation(_np(features), idx.numpy()))

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        return torch.from_numpy(O.grouping_operation_grad(_np(g), idx.numpy(), ctx.n)), None


class _Chamfer(Function):
    @staticmethod
    def forward(ctx, xyz1, xyz2):
        a, b = _np(xyz1), _np(xyz2)
        d1, d2, i1, i2 = O.chamfer_forward(a, b)
        ctx.save_for_backward(xyz1.detach(), xyz2.detach(), torch.from_numpy(i1), torch.from_numpy(i2))
        i1t, i2t = torch.from_numpy(i1), torch.from_numpy(i2)
        ctx.mark_non_differentiable(i1t, i2t)
        return torch.from_numpy(d1), torch.from_numpy(d2), i1t, i2t

    @staticmethod
    def backward(ctx, gd1, gd2, _gi1, _gi2):
        x1, x2, i1, i2 = ctx.saved_tensors
        g1, g2 = O.chamfer_backward(_np(x1), _np(x2), _np(gd1), _np(gd2), i1.numpy(), i2.numpy())
        return torch.from_numpy(g1), torch.from_numpy(g2)


def _knn(q, p, k, pad=0, want_dist=False):
    r = O.knn(_np(q), _np(p), k, pad, return_dist=want_dist)
    if want_dist:
        return torch.from_numpy(r[0]), torch.from_numpy(r[1])
    return torch.from_numpy(r)


class _AttentionCore:
    """softmax(scale q k^T) v, torch CPU math, same (meta, *srcs) calling
    convention as svdformer_pointsea_amd.attention.AttentionCore."""

    @staticmethod
    def apply(meta, *srcs):
        heads, scale, E, bf, qw, kw, vw = meta[:7]   # meta[7] (bias-sum flags): GPU backward only
        q, k, v = (srcs[w[0]][..., w[1]:w[1] + E] for w in (qw, kw, vw))
        if bf:  # (B, L, E) -> (L, B, E)
            q, k, v = (t.transpose(0, 1) for t in (q, k, v))
        Lq, B, _ = q.shape
        Lk = k.shape[0]
        hd = E // heads
        qh = q.reshape(Lq, B * heads, hd).transpose(0, 1)
        kh = k.reshape(Lk, B * heads, hd).transpose(0, 1)
        vh = v.reshape(Lk, B * heads, hd).transpose(0, 1)
        p = torch.softmax(torch.bmm(qh * scale, kh.transpose(1, 2)), dim=-1)
        o = torch.bmm(p, vh).transpose(0, 1).reshape(Lq, B, E)
        return o.transpose(0, 1).contiguous() if bf else o


class _TransposeAdd:
    @staticmethod
    def apply(a, b, out_dtype):
        x = a if b is None else a + b
        return x.transpose(1, 2).contiguous().to(out_dtype)


class _LayerNorm:
    @staticmethod
    def apply(a, b, weight, bias, eps, want16, sum_of=None):  # sum_of: a GPU-only fusion
        x = (a if b is None else a + b).float()
        y = torch.nn.functional.layer_norm(x, (x.shape[-1],), weight, bias, eps)
        return (y, y.to(torch.bfloat16)) if want16 else y


def depth_images(render, points):
    """PCViews.get_img on CPU (oracle splat) -> (B*V, R, R)."""
    return torch.from_numpy(O.points2depth(_np(points), render.rot_mat.numpy(), render.translation.numpy(),
                                           render.resolution, render.resolution))


def real_images(render, points):
    """PCViews_Real.get_img on CPU -> (B*V, 3, 224, 224): the view transform in
    torch (mv_utils_zs.py:166-195), then the oracle's points2grid / grid2image."""
    b = points.shape[0]
    v = render.num_views
    p = torch.repeat_interleave(points.detach().float(), v, dim=0)
    p = torch.matmul(p, render.rot_mat.repeat(b, 1, 1))
    p = torch.matmul(p, render.rot_mat2.repeat(b, 1, 1))
    p = p - render.translation.unsqueeze(1).repeat(b, 1, 1)
    grid = O.points2grid(_np(p))
    return torch.from_numpy(O.grid2image(grid, render.kernel.numpy()))


@contextlib.contextmanager
def cpu_ops():
    """Swap the package's HIP entry points for the CPU versions above."""
    from svdformer_pointsea_amd import attention, chamfer3D, model_utils, pointnet2_utils, pointsea, svdformer

    patches = [
        (pointsea, "furthest_point_sample", _FPS.apply),
        (pointsea, "gather_operation", _Gather.apply),
        (pointnet2_utils, "furthest_point_sample", _FPS.apply),
        (pointnet2_utils, "gather_operation", _Gather.apply),
        (pointnet2_utils, "grouping_operation", _Group.apply),
        (model_utils, "furthest_point_sample", _FPS.apply),
        (model_utils, "gather_operation", _Gather.apply),
        (model_utils, "grouping_operation", _Group.apply),
        (model_utils, "_knn", _knn),
        (svdformer, "furthest_point_sample", _FPS.apply),
        (svdformer, "gather_operation", _Gather.apply),
        (chamfer3D, "chamfer_3DFunction", _Chamfer),
        (attention, "AttentionCore", _AttentionCore),
        (attention, "_TransposeAdd", _TransposeAdd),
        (attention, "_LayerNorm", _LayerNorm),
    ]
    saved = [(m, n, getattr(m, n)) for m, n, _ in patches]
    try:
        for m, n, f in patches:
            setattr(m, n, f)
        yield
    finally:
        for m, n, f in saved:
            setattr(m, n, f)

