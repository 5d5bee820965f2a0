"""3x3 / stride 1 / pad 1 / bias-free nn.Conv2d on channels_last bf16 activations
through libpcops (pcops_conv3x3_fwd / _wgrad, csrc/conv.hip) -- and the
single-channel stem conv on the fp32 depth images (pcops_conv3x3_c1_*): the ResNet
BasicBlock convs of SVDFormer's image encoder (models/resnet.py:36-70 via
models/SVDFormer.py:139-146; C = 16 at 224x224 and 32 at 112x112 for the 96
depth images of a PCN batch), where MIOpen's NHWC kernels ran 2.5-6x below
HBM speed.  Other convs (strides, other channel counts, fp32 inputs) stay on
torch's nn.Conv2d.  The module and its state_dict are unchanged.
"""
import os

import torch
from torch import nn

from ._lib import Workspace, call, lib, ptr, stream_of

# PCOPS_CONV3X3=0: torch's nn.Conv2d (MIOpen) for every conv (A/B runs, parity tests)
ENABLED = os.environ.get("PCOPS_CONV3X3", "1") != "0"
_CHANNELS = (16, 32)


def _ohwi(w):
    """(Co, Ci, 3, 3) -> bf16 [co][kh][kw][ci] (a view when w is already channels_last bf16)."""
    return w.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()


class _Conv3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        N, C, H, W = x.shape
        y = torch.empty((N, C, H, W), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        with torch.cuda.device(x.device):
            call("conv3x3_fwd", lib().pcops_conv3x3_fwd, ptr(x), ptr(_ohwi(w)), N, H, W, C, ptr(y), stream_of(x))
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        N, C, H, W = x.shape
        gy = gy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        gx = gw = None
        with torch.cuda.device(x.device):
            if ctx.needs_input_grad[0]:
                # stride-1 input gradient: the same conv of dy with w'[ci][kh][kw][co] = w[co][ci][2-kh][2-kw]
                wt = w.to(torch.bfloat16).flip(2, 3).permute(1, 2, 3, 0).contiguous()
                gx = torch.empty_like(x)
                call("conv3x3_dgrad", lib().pcops_conv3x3_fwd, ptr(gy), ptr(wt), N, H, W, C, ptr(gx), stream_of(x))
            if ctx.needs_input_grad[1]:
                gw = _Conv3x3._wgrad(x, w, gy)
        return gx, gw

    @staticmethod
    def _wgrad(x, w, gy):
        N, C, H, W = x.shape
        gw = torch.empty_like(w)   # w's dtype and memory order (OIHW or channels_last OHWI)
        ohwi = int(w.is_contiguous(memory_format=torch.channels_last) and not w.is_contiguous())
        if not (ohwi or w.is_contiguous()):
            gw = torch.empty(w.shape, dtype=w.dtype, device=w.device)
        nbytes = lib().pcops_conv3x3_wgrad_workspace_bytes(C)
        ws = Workspace.get(x.device, nbytes)
        call("conv3x3_wgrad", lib().pcops_conv3x3_wgrad, ptr(x), ptr(gy), N, H, W, C, ptr(gw),
             0 if w.dtype == torch.float32 else 1, ohwi, ptr(ws), nbytes, stream_of(x))
        return gw


class _Conv3x3Skip(torch.autograd.Function):
    """(conv(x), x) for a ResNet BasicBlock whose input also feeds its identity branch: the two gradients
    x receives (the first conv's input gradient and the identity's) are summed inside the dgrad launch
    (pcops_conv3x3_fwd_res) as autograd's bf16 accumulation would sum them, instead of a separate add
    pass over the block input (models/resnet.py:56-70 `out += identity`)."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.set_materialize_grads(False)
        y = _Conv3x3.forward(ctx, x, w)
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, gy, gskip):
        x, w = ctx.saved_tensors
        N, C, H, W = x.shape
        gx = gw = None
        if gy is None:
            return (None if gskip is None else gskip.to(x.dtype)), None
        gy = gy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        with torch.cuda.device(x.device):
            if ctx.needs_input_grad[0]:
                wt = w.to(torch.bfloat16).flip(2, 3).permute(1, 2, 3, 0).contiguous()
                gx = torch.empty_like(x)
                if gskip is None:
                    call("conv3x3_dgrad", lib().pcops_conv3x3_fwd, ptr(gy), ptr(wt), N, H, W, C, ptr(gx),
                         stream_of(x))
                else:
                    r = gskip.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
                    call("conv3x3_dgrad_res", lib().pcops_conv3x3_fwd_res, ptr(gy), ptr(wt), N, H, W, C, ptr(r),
                         ptr(gx), stream_of(x))
            if ctx.needs_input_grad[1]:
                gw = _Conv3x3._wgrad(x, w, gy)
        return gx, gw


class _Conv3x3C1(torch.autograd.Function):
    """The single-channel stem (nn.Conv2d(1, 16, 3, padding=1, bias=False) on fp32 depth
    images under bf16 autocast): pcops_conv3x3_c1_fwd / _wgrad; the image gets no gradient."""

    @staticmethod
    def forward(ctx, x, w):
        N, _, H, W = x.shape
        y = torch.empty((N, 16, H, W), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        with torch.cuda.device(x.device):
            call("conv3x3_c1_fwd", lib().pcops_conv3x3_c1_fwd, ptr(x), ptr(w.float().contiguous()), N, H, W, ptr(y),
                 stream_of(x))
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        N, _, H, W = x.shape
        gw = None
        if ctx.needs_input_grad[1]:
            gy = gy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            gw = torch.empty_like(w)   # Cin = 1: OIHW and OHWI are the same order
            with torch.cuda.device(x.device):
                nbytes = lib().pcops_conv3x3_c1_wgrad_workspace_bytes()
                ws = Workspace.get(x.device, nbytes)
                call("conv3x3_c1_wgrad", lib().pcops_conv3x3_c1_wgrad, ptr(x), ptr(gy), N, H, W, ptr(gw),
                     0 if w.dtype == torch.float32 else 1, ptr(ws), nbytes, stream_of(x))
        return None, gw


def stem_eligible(x, conv):
    return (ENABLED and isinstance(conv, nn.Conv2d) and x.is_cuda and x.dim() == 4 and x.dtype == torch.float32
            and not x.requires_grad and x.shape[1] == 1 and x.is_contiguous()
            and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
            and conv.in_channels == 1 and conv.out_channels == 16 and conv.kernel_size == (3, 3)
            and conv.stride == (1, 1) and conv.padding == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1
            and conv.bias is None and conv.padding_mode == "zeros"
            and conv.weight.dtype in (torch.float32, torch.bfloat16) and conv.weight.is_contiguous())


def eligible(x, conv):
    if not (ENABLED and isinstance(conv, nn.Conv2d) and x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16):
        return False
    C = x.shape[1]
    return (conv.kernel_size == (3, 3) and conv.stride == (1, 1) and conv.padding == (1, 1)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None and conv.padding_mode == "zeros"
            and C in _CHANNELS and conv.in_channels == C and conv.out_channels == C
            and conv.weight.dtype in (torch.float32, torch.bfloat16)
            and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0)


# PCOPS_CONV_SKIP=0: the BasicBlock's identity gradient added by autograd (A/B runs)
SKIP_FUSED = os.environ.get("PCOPS_CONV_SKIP", "1") != "0"


def conv3x3_skip(x, conv):
    """(conv(x), identity of x) for a BasicBlock without downsample: on libpcops the identity's
    gradient is summed into the conv's input gradient inside the dgrad launch (_Conv3x3Skip)."""
    w = conv.weight
    if SKIP_FUSED and eligible(x, conv) and w.dtype in (torch.float32, torch.bfloat16) and torch.is_grad_enabled():
        return _Conv3x3Skip.apply(x, w)
    return conv3x3(x, conv), x


def conv3x3(x, conv, weight=None):
    """conv(x) for an nn.Conv2d; libpcops when eligible (see module doc), torch otherwise.
    `weight` overrides conv.weight (e.g. a bf16 shadow)."""
    w = conv.weight if weight is None else weight
    if eligible(x, conv) and w.dtype in (torch.float32, torch.bfloat16):
        return _Conv3x3.apply(x, w)
    if stem_eligible(x, conv):
        return _Conv3x3C1.apply(x, w)
    return conv(x)
