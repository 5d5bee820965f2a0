"""Hot-path pieces of models/model_utils.py (and models_PointSea/model_utils.py)
re-expressed on libpcops.so.  Names and signatures follow the reference so
its model classes can import them unchanged:

  query_knn(nsample, xyz, new_xyz, include_self=True)   model_utils.py:281-286
  query_knn_point(k, xyz, new_xyz)                      :807-810
  group_local(xyz, k=20, return_idx=False)              :812-826
  index_points(points, idx)                             :828-845
  fps_subsample(pcd, n_points=2048)                     :489-499
  sample_and_group_knn(xyz, points, npoint, k, ...)     :323-356
  sample_and_group_knn_cl (fused grouping, channels_last) :323-356 + the first conv's layout
  edge_features (EdgeConv's [x_i - x_j, x_i], channels_last) :812-845, 869-877
  self_attention / cross_attention / SDG_Decoder        :542-629
  self_attention_woinp / SDG_Decoder_PointSea           models_PointSea/model_utils.py:463-509
  PCViews                                               :1179-1234
"""
import numpy as np
import os

import torch
from torch import nn

from . import _lib
from ._lib import Workspace, call, lib, ptr, require_float, stream_of
from .pointnet2_utils import furthest_point_sample, furthest_point_sample_counts, gather_operation, grouping_operation


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
        wsb = lib().pcops_knn_workspace_bytes(B, S, N, C, k + pad) if _KNN_SORTED else 0
        # with scratch: C >= 32 by the streamed, candidate-split form (knnC3_kernel + merge),
        # the index-order scan's result bit for bit
        if wsb:
            ws = Workspace.get(q.device, wsb)
            call("knn", lib().pcops_knn_ws, ptr(q), ptr(p), B, S, N, C, k, pad, ptr(idx), ptr(dist), ptr(ws), wsb,
                 stream_of(q))
        else:
            call("knn", lib().pcops_knn, ptr(q), ptr(p), B, S, N, C, k, pad, ptr(idx), ptr(dist), stream_of(q))
    return (idx, dist) if want_dist else idx


_KNN_SORTED = os.environ.get("PCOPS_KNN_SORTED", "1") != "0"   # A/B switch: 0 = pcops_knn (no scratch)


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


def fps_subsample_counts(pcd, counts, n_points=2048):
    """fps_subsample of zero-padded clouds whose valid rows are counts (B,) int32: the FPS sweep
    stops at each cloud's count (pointnet2_utils.furthest_point_sample_counts); the same points
    as fps_subsample of the padded buffer."""
    idx = furthest_point_sample_counts(pcd.contiguous(), counts, n_points)
    new_pcd = gather_operation(pcd.permute(0, 2, 1).contiguous(), idx)
    return new_pcd.permute(0, 2, 1).contiguous()


class _SAGroup(torch.autograd.Function):
    """pcops_sa_group: grouped (xyz - centre, points) rows in channels_last order."""

    @staticmethod
    def forward(ctx, xyz_t, new_xyz_t, points_t, idx, out_dtype):
        B, N, _ = xyz_t.shape
        S, K = idx.shape[1], idx.shape[2]
        C = 0 if points_t is None else points_t.shape[2]
        out = torch.empty(B, S, K, 3 + C, dtype=out_dtype, device=xyz_t.device)
        with torch.cuda.device(xyz_t.device):
            call("sa_group", lib().pcops_sa_group, ptr(xyz_t), ptr(new_xyz_t), ptr(points_t), ptr(idx), B, N, S, K, C,
                 ptr(out), 1 if out_dtype == torch.bfloat16 else 0, stream_of(xyz_t))
        ctx.save_for_backward(idx)
        ctx.dims = (B, N, S, K, C)
        ctx.mark_non_differentiable(idx)
        return out

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        B, N, S, K, C = ctx.dims
        if C == 0 or not ctx.needs_input_grad[2]:
            return None, None, None, None, None
        g = g.contiguous()
        gp = torch.empty(B, N, C, dtype=torch.float32, device=g.device)
        with torch.cuda.device(g.device):
            call("sa_group_grad", lib().pcops_sa_group_grad, ptr(g), 1 if g.dtype == torch.bfloat16 else 0, ptr(idx),
                 B, N, S, K, C, ptr(gp), stream_of(g))
        return None, None, gp, None, None


class SharedFPS:
    """Furthest-point indices of one cloud computed once for two consumers.

    FPS is greedy: the first m indices of an FPS of M >= m points ARE the FPS of m points of the
    same cloud (every round depends only on the rounds before it; the tie rule, sampling_gpu.cu:
    69-173, depends on N, not on M).  The models sample the partial input twice -- the local
    encoder (SVDFormer.py:177, PointSea.py:241, local_points) and the point encoder's first SA
    module (model_utils.py:341, 512) -- so the FPS runs once, for the larger count, on the stream
    that produced it; `take(m)` hands the first m columns to another stream after an event wait
    (graph-capturable: the origin stream waits on a side stream's event)."""

    def __init__(self, idx):
        self.idx = idx
        self.event = self.stream = None
        if idx.is_cuda:
            self.stream = torch.cuda.current_stream(idx.device)
            self.event = torch.cuda.Event()
            self.event.record(self.stream)

    def take(self, m):
        if m > self.idx.shape[1]:
            raise ValueError(f"SharedFPS holds {self.idx.shape[1]} indices, {m} requested")
        if self.event is not None:
            cur = torch.cuda.current_stream(self.idx.device)
            # never on the producing stream itself: stream order suffices there, and under graph
            # capture a side stream waiting on its own event files itself in its own list of
            # parallel capture streams (HIP 7.0) -- the end-of-capture walk never returns (_lib.fork)
            if cur != self.stream:
                _lib.guarded_wait(cur, self.stream, event=self.event)
                self.idx.record_stream(cur)
        return self.idx if m == self.idx.shape[1] else self.idx[:, :m].contiguous()


def sample_and_group_knn_cl(xyz, points_t, npoint, k, out_dtype=torch.float32, fidx=None):
    """sample_and_group_knn (model_utils.py:323-356, use_xyz) in three launches --
    FPS, kNN, and ONE fused grouping (pcops_sa_group) that writes the
    neighbourhood features straight into the channels_last memory the first
    1x1 conv reads.  xyz (B,3,N) without gradient, points_t (B,N,C) token-major
    (or None) -> new_xyz (B,3,S), features (B,3+C,S,K) channels_last, idx."""
    xyz_t = xyz.transpose(1, 2).contiguous()
    fidx = furthest_point_sample(xyz_t, npoint) if fidx is None else fidx.take(npoint)
    new_xyz = gather_operation(xyz.contiguous(), fidx)                 # (B,3,S), the reference's new_xyz
    new_xyz_t = new_xyz.transpose(1, 2).contiguous()
    idx = query_knn(k, xyz_t, new_xyz_t)
    if points_t is not None:
        points_t = points_t.float().contiguous()
    feat = _SAGroup.apply(xyz_t, new_xyz_t, points_t, idx, out_dtype)  # (B,S,K,3+C)
    return new_xyz, feat.permute(0, 3, 1, 2), idx


def sample_and_group_knn(xyz, points, npoint, k, use_xyz=True, idx=None, fidx=None):
    """model_utils.py:323-356: FPS -> gather -> kNN -> group (xyz, points)."""
    xyz_flipped = xyz.permute(0, 2, 1).contiguous()
    new_xyz = gather_operation(xyz, furthest_point_sample(xyz_flipped, npoint) if fidx is None else fidx.take(npoint))
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


class _EdgeGroup(torch.autograd.Function):
    """pcops_edge_group: EdgeConv's (x_i - x_j, x_i) rows in channels_last order."""

    @staticmethod
    def forward(ctx, x_t, idx, out_dtype):
        B, N, C = x_t.shape
        K = idx.shape[2]
        out = torch.empty(B, N, K, 2 * C, dtype=out_dtype, device=x_t.device)
        with torch.cuda.device(x_t.device):
            call("edge_group", lib().pcops_edge_group, ptr(x_t), ptr(idx), B, N, K, C, ptr(out),
                 1 if out_dtype == torch.bfloat16 else 0, stream_of(x_t))
        ctx.save_for_backward(idx)
        ctx.dims = (B, N, K, C)
        return out

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        B, N, K, C = ctx.dims
        if not ctx.needs_input_grad[0]:
            return None, None, None
        g = g.contiguous()
        gx = torch.empty(B, N, C, dtype=torch.float32, device=g.device)
        with torch.cuda.device(g.device):
            call("edge_group_grad", lib().pcops_edge_group_grad, ptr(g), 1 if g.dtype == torch.bfloat16 else 0,
                 ptr(idx), B, N, K, C, ptr(gx), stream_of(g))
        return gx, None, None


def edge_features(x, k, out_dtype=None):
    """EdgeConv's edge features (model_utils.py:869-877): for the k feature-space
    nearest neighbours j of every point i (group_local, :812-826), the rows
    [x_i - x_j, x_i] -> (B, 2C, N, k) in channels_last memory, out_dtype (x's dtype
    by default; bf16 under autocast is what the first 1x1 conv would cast to).
    x (B, C, N).  Two launches: the kNN on the token-major fp32 cloud, then ONE
    pass (pcops_edge_group) that gathers, subtracts, concatenates and writes the
    conv's input layout -- in place of the grouping launch, repeat, subtract, cat
    and channels_last copy."""
    B, C, N = x.shape
    if out_dtype is None:
        out_dtype = x.dtype
    pts = x.float().transpose(1, 2).contiguous()   # (B, N, C) fp32: the kNN's operand and the gather source
    idx = _knn(pts.detach(), pts.detach(), k)
    return _EdgeGroup.apply(pts, idx, out_dtype).permute(0, 3, 1, 2)
