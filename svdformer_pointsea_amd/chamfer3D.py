"""Drop-in for `metrics.CD.chamfer3D.dist_chamfer_3D` backed by libpcops.so.

chamfer_3DDist()(xyz1 (B,N,3), xyz2 (B,M,3)) -> dist1 (B,N), dist2 (B,M)
(squared distances), idx1 (B,N), idx2 (B,M) int32 -- dist_chamfer_3D.py:26-74.
Unlike the reference (dist_chamfer_3D.py:33-43) nothing is allocated on the
host or copied per call: outputs come from torch's caching allocator on the
inputs' device and the kernels run on torch's current stream.
"""
import torch
from torch import nn
from torch.autograd import Function
from torch.amp import custom_bwd, custom_fwd

from ._lib import Workspace, call, lib, ptr, require_float, stream_of


def chamfer_forward_raw(xyz1, xyz2):
    """(dist1, dist2, idx1, idx2) of two fp32 clouds on libpcops, outside autograd."""
    require_float(xyz1, "xyz1")
    require_float(xyz2, "xyz2")
    B, n, _ = xyz1.shape
    m = xyz2.shape[1]
    dev = xyz1.device
    dist1 = torch.empty(B, n, device=dev)
    dist2 = torch.empty(B, m, device=dev)
    idx1 = torch.empty(B, n, dtype=torch.int32, device=dev)
    idx2 = torch.empty(B, m, dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        # large clouds: the spatially culled search (scratch for the sorted clouds and tile boxes)
        wsb = lib().pcops_chamfer_workspace_bytes(B, n, m)
        if wsb:
            ws = Workspace.get(dev, wsb)
            call("chamfer_3D.forward", lib().pcops_chamfer_forward_ws, ptr(xyz1), ptr(xyz2), B, n, m,
                 ptr(dist1), ptr(dist2), ptr(idx1), ptr(idx2), ptr(ws), wsb, stream_of(xyz1))
        else:
            call("chamfer_3D.forward", lib().pcops_chamfer_forward, ptr(xyz1), ptr(xyz2), B, n, m, ptr(dist1),
                 ptr(dist2), ptr(idx1), ptr(idx2), stream_of(xyz1))
    return dist1, dist2, idx1, idx2


class chamfer_3DFunction(Function):
    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, xyz1, xyz2):
        dist1, dist2, idx1, idx2 = chamfer_forward_raw(xyz1, xyz2)
        ctx.save_for_backward(xyz1, xyz2, idx1, idx2)
        ctx.mark_non_differentiable(idx1, idx2)
        return dist1, dist2, idx1, idx2

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, graddist1, graddist2, gradidx1, gradidx2):
        xyz1, xyz2, idx1, idx2 = ctx.saved_tensors
        B, n, _ = xyz1.shape
        m = xyz2.shape[1]
        dev = xyz1.device
        graddist1 = torch.zeros(B, n, device=dev) if graddist1 is None else graddist1.contiguous()
        graddist2 = torch.zeros(B, m, device=dev) if graddist2 is None else graddist2.contiguous()
        g1 = torch.empty(B, n, 3, device=dev)
        g2 = torch.empty(B, m, 3, device=dev)
        with torch.cuda.device(dev):
            call("chamfer_3D.backward", lib().pcops_chamfer_backward, ptr(xyz1), ptr(xyz2), B, n, m, ptr(graddist1),
                 ptr(graddist2), ptr(idx1), ptr(idx2), ptr(g1), ptr(g2), stream_of(xyz1))
        return g1, g2


class chamfer_3DDist(nn.Module):
    def __init__(self):
        super().__init__()

    def forward(self, input1, input2):
        input1 = input1.contiguous()
        input2 = input2.contiguous()
        return chamfer_3DFunction.apply(input1, input2)
