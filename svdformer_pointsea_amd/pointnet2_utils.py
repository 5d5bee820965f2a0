"""Drop-in for `pointnet2_ops.pointnet2_utils` backed by libpcops.so (gfx950).

Same names, signatures, autograd contracts and error behaviour as
pointnet2_ops_lib/pointnet2_ops/pointnet2_utils.py:34-379:
  furthest_point_sample(xyz (B,N,3), npoint) -> (B,npoint) int32   [:34-65]
  gather_operation(features (B,C,N), idx (B,M) int32) -> (B,C,M)    [:68-101]
  three_nn(unknown (B,n,3), known (B,m,3)) -> (dist, idx)           [:104-136]
  three_interpolate(features (B,c,m), idx, weight) -> (B,c,n)       [:139-191]
  grouping_operation(features (B,C,N), idx (B,S,K)) -> (B,C,S,K)    [:194-240]
  ball_query(radius, nsample, xyz, new_xyz) -> (B,M,nsample) int32  [:243-276]
  QueryAndGroup / GroupAll                                          [:279-379]
"""
import torch
import torch.nn as nn
from torch.autograd import Function
from torch.amp import custom_bwd, custom_fwd

from . import _lib
from ._lib import call, lib, ptr, require_float, require_int, stream_of


class FurthestPointSampling(Function):
    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, xyz, npoint):
        require_float(xyz, "points")
        B, N, _ = xyz.shape
        npoint = int(npoint)
        out = torch.empty(B, npoint, dtype=torch.int32, device=xyz.device)
        wsb = lib().pcops_fps_workspace_bytes(B, N)
        ws = _lib.Workspace.get(xyz.device, wsb)
        with torch.cuda.device(xyz.device):
            call("furthest_point_sampling", lib().pcops_furthest_point_sampling, ptr(xyz), B, N, npoint, ptr(out),
                 ptr(ws), wsb, stream_of(xyz))
        ctx.mark_non_differentiable(out)
        return out

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, grad_out):
        return ()


furthest_point_sample = FurthestPointSampling.apply


def furthest_point_sample_counts(xyz, counts, npoint):
    """FPS over zero-padded clouds with known valid row counts (B,) int32: row k >= counts[b]
    of cloud b is absent.  Equals furthest_point_sample on the buffer whose rows >= counts[b]
    are zero (the reference skips |p|^2 <= 1e-3 rows, sampling_gpu.cu:100-101) -- the ragged
    per-sample FPS calls of utils/helpers.py:79-119 -- with the sweep stopping at the count.
    Not differentiable (as furthest_point_sample)."""
    require_float(xyz, "points")
    require_int(counts, "counts")
    B, N, _ = xyz.shape
    if counts.shape != (B,):
        raise RuntimeError(f"counts must have shape ({B},), got {tuple(counts.shape)}")
    npoint = int(npoint)
    out = torch.empty(B, npoint, dtype=torch.int32, device=xyz.device)
    wsb = lib().pcops_fps_workspace_bytes(B, N)
    ws = _lib.Workspace.get(xyz.device, wsb)
    with torch.cuda.device(xyz.device):
        call("furthest_point_sampling_counts", lib().pcops_furthest_point_sampling_counts, ptr(xyz), ptr(counts), B, N,
             npoint, ptr(out), ptr(ws), wsb, stream_of(xyz))
    return out


class GatherOperation(Function):
    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, features, idx):
        require_float(features, "points")
        require_int(idx, "idx")
        B, C, N = features.shape
        M = idx.shape[1]
        out = torch.empty(B, C, M, dtype=torch.float32, device=features.device)
        with torch.cuda.device(features.device):
            call("gather_points", lib().pcops_gather_points, ptr(features), ptr(idx), B, C, N, M, ptr(out),
                 stream_of(features))
        ctx.save_for_backward(idx, features)
        return out

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, grad_out):
        idx, features = ctx.saved_tensors
        B, C, N = features.shape
        M = idx.shape[1]
        grad_out = grad_out.contiguous()
        gp = torch.empty(B, C, N, dtype=torch.float32, device=grad_out.device)
        with torch.cuda.device(grad_out.device):
            call("gather_points_grad", lib().pcops_gather_points_grad, ptr(grad_out), ptr(idx), B, C, N, M, ptr(gp),
                 stream_of(grad_out))
        return gp, None


gather_operation = GatherOperation.apply


class ThreeNN(Function):
    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, unknown, known):
        require_float(unknown, "unknowns")
        require_float(known, "knows")
        B, n, _ = unknown.shape
        m = known.shape[1]
        dist2 = torch.empty(B, n, 3, dtype=torch.float32, device=unknown.device)
        idx = torch.empty(B, n, 3, dtype=torch.int32, device=unknown.device)
        with torch.cuda.device(unknown.device):
            call("three_nn", lib().pcops_three_nn, ptr(unknown), ptr(known), B, n, m, ptr(dist2), ptr(idx),
                 stream_of(unknown))
        dist = torch.sqrt(dist2)
        # the RETURNED dist is the non-differentiable output (pointnet2_utils.py:124-127)
        ctx.mark_non_differentiable(dist, idx)
        return dist, idx

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, grad_dist, grad_idx):
        return ()


three_nn = ThreeNN.apply


class ThreeInterpolate(Function):
    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, features, idx, weight):
        require_float(features, "points")
        require_int(idx, "idx")
        require_float(weight, "weight")
        B, c, m = features.shape
        n = idx.shape[1]
        ctx.save_for_backward(idx, weight, features)
        out = torch.empty(B, c, n, dtype=torch.float32, device=features.device)
        with torch.cuda.device(features.device):
            call("three_interpolate", lib().pcops_three_interpolate, ptr(features), ptr(idx), ptr(weight), B, c, m, n,
                 ptr(out), stream_of(features))
        return out

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, grad_out):
        idx, weight, features = ctx.saved_tensors
        B, c, m = features.shape
        n = idx.shape[1]
        grad_out = grad_out.contiguous()
        gf = torch.empty(B, c, m, dtype=torch.float32, device=grad_out.device)
        with torch.cuda.device(grad_out.device):
            call("three_interpolate_grad", lib().pcops_three_interpolate_grad, ptr(grad_out), ptr(idx), ptr(weight), B,
                 c, n, m, ptr(gf), stream_of(grad_out))
        return gf, torch.zeros_like(idx), torch.zeros_like(weight)


three_interpolate = ThreeInterpolate.apply


class GroupingOperation(Function):
    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, features, idx):
        require_float(features, "points")
        require_int(idx, "idx")
        B, C, N = features.shape
        _, S, K = idx.shape
        out = torch.empty(B, C, S, K, dtype=torch.float32, device=features.device)
        with torch.cuda.device(features.device):
            call("group_points", lib().pcops_group_points, ptr(features), ptr(idx), B, C, N, S, K, ptr(out),
                 stream_of(features))
        ctx.save_for_backward(idx, features)
        return out

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, grad_out):
        idx, features = ctx.saved_tensors
        B, C, N = features.shape
        _, S, K = idx.shape
        grad_out = grad_out.contiguous()
        gf = torch.empty(B, C, N, dtype=torch.float32, device=grad_out.device)
        with torch.cuda.device(grad_out.device):
            call("group_points_grad", lib().pcops_group_points_grad, ptr(grad_out), ptr(idx), B, C, N, S, K, ptr(gf),
                 stream_of(grad_out))
        return gf, torch.zeros_like(idx)


grouping_operation = GroupingOperation.apply


class BallQuery(Function):
    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, radius, nsample, xyz, new_xyz):
        require_float(new_xyz, "new_xyz")
        require_float(xyz, "xyz")
        B, N, _ = xyz.shape
        M = new_xyz.shape[1]
        out = torch.empty(B, M, int(nsample), dtype=torch.int32, device=xyz.device)
        with torch.cuda.device(xyz.device):
            call("ball_query", lib().pcops_ball_query, ptr(new_xyz), ptr(xyz), B, N, M, float(radius), int(nsample),
                 ptr(out), stream_of(xyz))
        ctx.mark_non_differentiable(out)
        return out

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, grad_out):
        return ()


ball_query = BallQuery.apply


class QueryAndGroup(nn.Module):
    """pointnet2_utils.py:279-346 (radius grouping + optional xyz concat)."""

    def __init__(self, radius, nsample, use_xyz=True):
        super().__init__()
        self.radius, self.nsample, self.use_xyz = radius, nsample, use_xyz

    def forward(self, xyz, new_xyz, features=None):
        idx = ball_query(self.radius, self.nsample, xyz, new_xyz)
        xyz_trans = xyz.transpose(1, 2).contiguous()
        grouped_xyz = grouping_operation(xyz_trans, idx)
        grouped_xyz -= new_xyz.transpose(1, 2).unsqueeze(-1)
        if features is not None:
            grouped_features = grouping_operation(features, idx)
            if self.use_xyz:
                return torch.cat([grouped_xyz, grouped_features], dim=1)
            return grouped_features
        assert self.use_xyz, "Cannot have not features and not use xyz as a feature!"
        return grouped_xyz


class GroupAll(nn.Module):
    """pointnet2_utils.py:349-379."""

    def __init__(self, use_xyz=True):
        super().__init__()
        self.use_xyz = use_xyz

    def forward(self, xyz, new_xyz, features=None):
        grouped_xyz = xyz.transpose(1, 2).unsqueeze(2)
        if features is not None:
            grouped_features = features.unsqueeze(2)
            if self.use_xyz:
                return torch.cat([grouped_xyz, grouped_features], dim=1)
            return grouped_features
        return grouped_xyz
