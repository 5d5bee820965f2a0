"""Drop-in for metrics/EMD/emd_module.py (emdFunction / emdModule) on libpcops.

emdModule()(input1 (B,n,3), input2 (B,n,3), eps, iters) -> (dist (B,n) squared
distance to the assigned point, assignment (B,n) int32); backward returns a
gradient for input1 only (emd_module.py:40-88).  The auction is the
deterministic restatement documented in csrc/emd.hip / DESIGN.md.
"""
import torch
from torch import nn
from torch.autograd import Function

from . import _lib
from ._lib import call, lib, ptr, stream_of


class emdFunction(Function):
    @staticmethod
    def forward(ctx, xyz1, xyz2, eps, iters):
        batchsize, n, _ = xyz1.size()
        _, m, _ = xyz2.size()
        assert n == m
        assert xyz1.size()[0] == xyz2.size()[0]
        assert batchsize <= 512
        if n % 1024 != 0:  # emd_cuda.cu:246-249 (the reference prints and returns zeros)
            raise RuntimeError("Input Error! The size of the point clouds should be a multiple of 1024.")
        xyz1 = xyz1.contiguous().float()
        xyz2 = xyz2.contiguous().float()
        _lib.require_float(xyz1, "xyz1")
        _lib.require_float(xyz2, "xyz2")
        return _emd_forward(ctx, xyz1, xyz2, float(eps), int(iters))

    @staticmethod
    def backward(ctx, graddist, gradidx):
        xyz1, xyz2, assignment = ctx.saved_tensors
        graddist = graddist.contiguous().float()
        B, n, _ = xyz1.shape
        g1 = torch.empty_like(xyz1)
        with torch.cuda.device(xyz1.device):
            call("emd_backward", lib().pcops_emd_backward, ptr(xyz1), ptr(xyz2), ptr(graddist), ptr(assignment), B, n,
                 ptr(g1), stream_of(xyz1))
        return g1, torch.zeros_like(xyz2), None, None


def _emd_forward(ctx, xyz1, xyz2, eps, iters):
    B, n, _ = xyz1.shape
    dist = torch.empty(B, n, device=xyz1.device)
    assignment = torch.empty(B, n, dtype=torch.int32, device=xyz1.device)
    wsb = lib().pcops_emd_workspace_bytes(B, n)
    ws = _lib.Workspace.get(xyz1.device, wsb)
    with torch.cuda.device(xyz1.device):
        call("emd_forward", lib().pcops_emd_forward, ptr(xyz1), ptr(xyz2), B, n, eps, iters, ptr(dist),
             ptr(assignment), ptr(ws), wsb, stream_of(xyz1))
    if ctx is not None:
        ctx.save_for_backward(xyz1, xyz2, assignment)
        ctx.mark_non_differentiable(assignment)
    return dist, assignment


def emd_raw(xyz1, xyz2, eps, iters):
    """The auction for any n >= 1 (no n % 1024 restriction), no autograd."""
    return _emd_forward(None, xyz1.contiguous().float(), xyz2.contiguous().float(), float(eps), int(iters))


class emdModule(nn.Module):
    def __init__(self):
        super().__init__()

    def forward(self, input1, input2, eps, iters):
        return emdFunction.apply(input1, input2, eps, iters)
