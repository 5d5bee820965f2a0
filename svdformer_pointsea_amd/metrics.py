"""Training losses and evaluation metrics of the reference on libpcops:
utils/loss_utils.py:10-155 and metrics/CD/fscore.py:3-16.

  chamfer / chamfer_sqrt / chamfer_single_side(_sqrt)    Chamfer losses
  get_loss / get_loss_PM                                 train_pcn / PointSea losses
  calc_cd                                                CD-L1 (cd_p), CD-L2 (cd_t), F-score
  calc_dcd                                               density-aware Chamfer
  fscore                                                 F-score on squared distances
Names, arguments and return structures are the reference's.  The
nearest-neighbour search is the Chamfer kernel (csrc/chamfer.hip, both
directions in one launch); what follows it are the same reductions, in the
same floating-point order, as the reference's torch expressions.
"""
import os

import torch
from torch.amp import custom_bwd, custom_fwd
from torch.autograd import Function

from . import chamfer3D
from ._lib import call, lib, ptr, stream_of
from .model_utils import fps_subsample

_nn = chamfer3D.chamfer_3DDist()


def _means(p1, p2, root):
    d1, d2, _, _ = _nn(p1, p2)
    if root:
        d1, d2 = torch.sqrt(d1), torch.sqrt(d2)
    return torch.mean(d1), torch.mean(d2)


class _SqrtMeanChamfer(Function):
    """chamfer_sqrt (both=True: (mean(sqrt(d1)) + mean(sqrt(d2))) / 2) and chamfer_single_side_sqrt
    (both=False: mean(sqrt(d1))), loss_utils.py:10-31, as one autograd node.  The forward runs the
    same torch expressions on the Chamfer kernel's distances (same values, bit for bit); the
    backward forms autograd's distance gradient in one launch (pcops_chamfer_sqrt_mean_grad: the
    "/ 2", mean and sqrt backward steps in their order) and hands it to pcops_chamfer_backward,
    instead of ~8 scalar / elementwise launches per loss term."""

    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, p1, p2, both):
        d1, d2, i1, i2 = chamfer3D.chamfer_forward_raw(p1, p2)
        s1 = torch.sqrt(d1)
        m1 = torch.mean(s1)
        s2 = torch.sqrt(d2) if both else None
        out = (m1 + torch.mean(s2)) / 2 if both else m1
        ctx.save_for_backward(p1, p2, i1, i2, s1, s2)
        ctx.both = both
        return out

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, g):
        p1, p2, i1, i2, s1, s2 = ctx.saved_tensors
        B, n, _ = p1.shape
        m = p2.shape[1]
        g = g.contiguous()
        gd1, gd2 = torch.empty_like(s1), torch.empty(B, m, device=p1.device)
        g1, g2 = torch.empty_like(p1), torch.empty_like(p2)
        with torch.cuda.device(p1.device):
            call("chamfer_sqrt_mean_grad", lib().pcops_chamfer_sqrt_mean_grad, ptr(g), 0.5 if ctx.both else 1.0,
                 ptr(s1), B * n, ptr(s2), B * m, ptr(gd1), ptr(gd2), stream_of(p1))
            call("chamfer_3D.backward", lib().pcops_chamfer_backward, ptr(p1), ptr(p2), B, n, m, ptr(gd1), ptr(gd2),
                 ptr(i1), ptr(i2), ptr(g1), ptr(g2), stream_of(p1))
        return (g1 if ctx.needs_input_grad[0] else None), (g2 if ctx.needs_input_grad[1] else None), None


def _fused_loss(p1, p2):
    """The one-node sqrt-mean loss applies (PCOPS_LOSS_FUSED=0 keeps the autograd chain; read per call)."""
    return (os.environ.get("PCOPS_LOSS_FUSED", "1") != "0" and p1.is_cuda and p2.is_cuda and p1.dim() == 3
            and p2.dim() == 3 and p1.shape[0] == p2.shape[0] and p1.shape[-1] == 3 and p2.shape[-1] == 3
            and p1.shape[1] > 0 and p2.shape[1] > 0)


def chamfer(p1, p2):
    m1, m2 = _means(p1, p2, False)
    return m1 + m2


def chamfer_sqrt(p1, p2):
    if _fused_loss(p1, p2):
        return _SqrtMeanChamfer.apply(p1.contiguous(), p2.contiguous(), True)
    m1, m2 = _means(p1, p2, True)
    return (m1 + m2) / 2


def chamfer_single_side(pcd1, pcd2):
    return _means(pcd1, pcd2, False)[0]


def chamfer_single_side_sqrt(pcd1, pcd2):
    if _fused_loss(pcd1, pcd2):
        return _SqrtMeanChamfer.apply(pcd1.contiguous(), pcd2.contiguous(), False)
    return _means(pcd1, pcd2, True)[0]


def gt_pyramid(gt, n1, nc):
    """(gt_c, gt_1): gt FPS-subsampled to n1 points, then that to nc points
    (loss_utils.py:47-48).  It depends on gt only, so a caller may compute it
    ahead of (and beside) the forward pass and hand it to get_loss(gts=...)."""
    gt_1 = fps_subsample(gt, n1)
    return fps_subsample(gt_1, nc), gt_1


def _stage_losses(pcds_pred, gt, CD, gts=None):
    """CD of (coarse, fine1, fine2) against gt FPS-subsampled to each size."""
    Pc, P1, P2 = pcds_pred
    gt_c, gt_1 = gts if gts is not None else gt_pyramid(gt, P1.shape[1], Pc.shape[1])
    return [CD(Pc, gt_c), CD(P1, gt_1), CD(P2, gt)]


def get_loss(pcds_pred, gt, sqrt=True, alpha1=1, alpha2=1, gts=None):
    """loss_utils.py:33-58 -> (cdc + alpha1*cd1 + alpha2*cd2, [cdc, cd1, cd2]).
    `gts` (optional): gt_pyramid(gt, ...) computed earlier by the caller."""
    cdc, cd1, cd2 = _stage_losses(pcds_pred, gt, chamfer_sqrt if sqrt else chamfer, gts)
    return cdc + alpha1 * cd1 + alpha2 * cd2, [cdc, cd1, cd2]


def get_loss_PM(pcds_pred, partial, gt, sqrt=True, gts=None):
    """loss_utils.py:60-82: get_loss + single-sided partial -> fine2 matching."""
    cdc, cd1, cd2 = _stage_losses(pcds_pred, gt, chamfer_sqrt if sqrt else chamfer, gts)
    pm = (chamfer_single_side_sqrt if sqrt else chamfer_single_side)(partial, pcds_pred[2])
    return cdc + cd1 + cd2 + pm, [cdc, cd1, cd2]


def fscore(dist1, dist2, threshold=0.0001):
    """(f1, precision_1, precision_2) per sample; dist1/dist2 are SQUARED."""
    p1 = torch.mean((dist1 < threshold).float(), dim=1)
    p2 = torch.mean((dist2 < threshold).float(), dim=1)
    f1 = 2 * p1 * p2 / (p1 + p2)
    f1[torch.isnan(f1)] = 0
    return f1, p1, p2


def calc_cd(output, gt, calc_f1=False, return_raw=False, normalize=False, separate=False):
    """Per-sample [cd_p (CD-L1), cd_t (CD-L2)] (+ f1) (+ dist1, dist2, idx1, idx2).
    Distances are gt -> output first, as loss_utils.py:98-115; `normalize` is
    accepted and unused there too."""
    dist1, dist2, idx1, idx2 = chamfer3D.chamfer_3DDist()(gt, output)
    l1 = [torch.sqrt(d).mean(1) for d in (dist1, dist2)]
    l2 = [d.mean(1) for d in (dist1, dist2)]
    if separate:
        res = [torch.cat([v.unsqueeze(0) for v in l1]), torch.cat([v.unsqueeze(0) for v in l2])]
    else:
        res = [(l1[0] + l1[1]) / 2, l2[0] + l2[1]]
    if calc_f1:
        res.append(fscore(dist1, dist2)[0])
    if return_raw:
        res.extend([dist1, dist2, idx1, idx2])
    return res


def _density_term(dist, idx, n_targets, alpha, n_lambda, frac):
    """mean_i (1 - exp(-alpha d_i) / (n_hits(idx_i)^lambda + 1e-6) * frac)."""
    hits = torch.zeros(idx.shape[0], n_targets, dtype=idx.dtype, device=idx.device)
    hits.scatter_add_(1, idx.long(), torch.ones_like(idx))
    w = hits.gather(1, idx.long()).float().detach() ** n_lambda
    w = (w + 1e-6) ** (-1) * frac
    return (1 - torch.exp(-dist * alpha) * w).mean(dim=1)


def calc_dcd(x, gt, alpha=1000, n_lambda=1, return_raw=False, non_reg=False):
    """Density-aware Chamfer distance -> [dcd, cd_p, cd_t] (+ raw)."""
    x, gt = x.float(), gt.float()
    n_x, n_gt = x.shape[1], gt.shape[1]
    assert x.shape[0] == gt.shape[0]
    f12, f21 = n_x / n_gt, n_gt / n_x
    if non_reg:
        f12, f21 = max(1, f12), max(1, f21)
    cd_p, cd_t, dist1, dist2, idx1, idx2 = calc_cd(x, gt, return_raw=True)
    # dist1/idx1: every gt point's nearest x; dist2/idx2: every x's nearest gt
    loss = (_density_term(dist1, idx1, n_x, alpha, n_lambda, f21) +
            _density_term(dist2, idx2, n_gt, alpha, n_lambda, f12)) / 2
    res = [loss, cd_p, cd_t]
    if return_raw:
        res.extend([dist1, dist2, idx1, idx2])
    return res
