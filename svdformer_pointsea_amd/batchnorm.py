"""BatchNorm2d fused with the residual add and activation that follow it in
the reference's encoders, on channels_last activations (pcops_batchnorm_fwd /
_bwd, csrc/batchnorm.hip):

  ResNet BasicBlock   relu(bn1(conv1(x))) ; relu(bn2(conv2(.)) + identity)   models/resnet.py:56-70
  SVFNet stem         relu(bn(conv(depth)))                                   models/SVDFormer.py:139-146
  EdgeConv            leaky_relu(bn(conv1x1(edge)), 0.2)                      models/model_utils.py:855-866
  PointSea ResEncoder torchvision resnet18 stem + BasicBlocks                 models_PointSea/PointSea.py:37-61

The modules stay nn.BatchNorm2d (state_dict, running statistics and
num_batches_tracked as torch keeps them); only their forward is replaced.
torch's MIOpen path runs a BasicBlock's bn2 + add + relu as five full passes
over the activation forward and six backward; here it is two and two.
"""
import os

import torch
from torch import nn

from ._lib import Workspace, call, lib, ptr, stream_of

_DT = {torch.float32: 0, torch.bfloat16: 1}
ACT_NONE, ACT_RELU, ACT_LEAKY = 0, 1, 2
# PCOPS_BN=0: torch's BatchNorm2d + add + activation (A/B runs, parity tests)
ENABLED = os.environ.get("PCOPS_BN", "1") != "0"


def _rows_c(x):
    C = x.shape[1]
    return x.numel() // C, C


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, weight, bias, rmean, rvar, nbt, batch_stats, momentum, eps, act, slope):
        rows, C = _rows_c(x)
        y = torch.empty_like(x)  # channels_last strides preserved
        smean = torch.empty(C, dtype=torch.float32, device=x.device)
        sinv = torch.empty(C, dtype=torch.float32, device=x.device)
        with torch.cuda.device(x.device):
            nbytes = lib().pcops_batchnorm_workspace_bytes(rows, C)
            ws = Workspace.get(x.device, nbytes)
            call("batchnorm_fwd", lib().pcops_batchnorm_fwd, ptr(x), _DT[x.dtype], ptr(res),
                 _DT[res.dtype] if res is not None else 0, rows, C, ptr(weight), ptr(bias), ptr(rmean), ptr(rvar),
                 float(momentum), float(eps), int(batch_stats), act, float(slope), ptr(y), ptr(smean), ptr(sinv),
                 ptr(ws), nbytes, ptr(nbt), stream_of(x))
        ctx.save_for_backward(x, y if act != ACT_NONE else None, weight, smean, sinv)
        ctx.cfg = (batch_stats, act, slope, res is not None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, y, weight, smean, sinv = ctx.saved_tensors
        batch_stats, act, slope, has_res = ctx.cfg
        rows, C = _rows_c(x)
        gy = gy.to(x.dtype).contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if has_res and ctx.needs_input_grad[1] else None
        need_w = weight is not None and ctx.needs_input_grad[2]
        dgamma = torch.empty(C, dtype=torch.float32, device=x.device) if need_w else None
        dbeta = torch.empty(C, dtype=torch.float32, device=x.device) if ctx.needs_input_grad[3] else None
        with torch.cuda.device(x.device):
            nbytes = lib().pcops_batchnorm_workspace_bytes(rows, C)
            ws = Workspace.get(x.device, nbytes)
            call("batchnorm_bwd", lib().pcops_batchnorm_bwd, ptr(gy), ptr(y), ptr(x), _DT[x.dtype], rows, C,
                 ptr(weight), ptr(smean), ptr(sinv), int(batch_stats), act, float(slope), ptr(dx), ptr(dres),
                 ptr(dgamma), ptr(dbeta), ptr(ws), nbytes, stream_of(x))
        return dx, dres, dgamma, dbeta, None, None, None, None, None, None, None, None


def _fusable(x, bn, residual):
    if not (ENABLED and x.is_cuda and x.dim() == 4 and x.dtype in _DT and isinstance(bn, nn.BatchNorm2d)):
        return False
    C = x.shape[1]
    if C % 8 or C > 512 or x.numel() == 0 or not x.is_contiguous(memory_format=torch.channels_last):
        return False
    if bn.weight is None or bn.weight.dtype != torch.float32 or bn.momentum is None:
        return False
    if x.data_ptr() % 16:
        return False
    if residual is not None and (residual.shape != x.shape or residual.dtype not in _DT
                                 or not residual.is_contiguous(memory_format=torch.channels_last)
                                 or residual.data_ptr() % 16):
        return False
    return True


def _activation(out, act, slope):
    if act == ACT_RELU:
        return torch.relu(out)
    if act == ACT_LEAKY:
        return torch.nn.functional.leaky_relu(out, slope)
    return out


def bn_act(x, bn, act=ACT_NONE, slope=0.0, residual=None):
    """act(bn(x) (+ residual)) for an nn.BatchNorm2d `bn`, fused on libpcops when x is a
    channels_last fp32/bf16 CUDA tensor (torch's modules otherwise)."""
    if not _fusable(x, bn, residual):
        out = bn(x)
        if residual is not None:
            out = out + residual
        return _activation(out, act, slope)
    batch_stats = bn.training or bn.running_mean is None
    update = bn.training and bn.running_mean is not None
    rm = bn.running_mean if (update or not batch_stats) else None
    rv = bn.running_var if (update or not batch_stats) else None
    # num_batches_tracked is incremented by the statistics kernel (no extra launch)
    nbt = bn.num_batches_tracked if update else None
    return _BNAct.apply(x, residual, bn.weight, bn.bias, rm, rv, nbt, batch_stats, bn.momentum, bn.eps, act, slope)


def _act_of(m):
    if isinstance(m, nn.ReLU):
        return ACT_RELU, 0.0
    if isinstance(m, nn.LeakyReLU):
        return ACT_LEAKY, float(m.negative_slope)
    return None


def run_sequential(seq, x, conv_fn=None):
    """Run an nn.Sequential, folding each BatchNorm2d and the ReLU / LeakyReLU right
    after it into one bn_act; conv_fn(x, conv) replaces the nn.Conv2d calls when given."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, nn.BatchNorm2d):
            a = _act_of(mods[i + 1]) if i + 1 < len(mods) else None
            if a is not None:
                x = bn_act(x, m, a[0], a[1])
                i += 2
                continue
            x = bn_act(x, m)
        elif conv_fn is not None and isinstance(m, nn.Conv2d):
            x = conv_fn(x, m)
        else:
            x = m(x)
        i += 1
    return x
