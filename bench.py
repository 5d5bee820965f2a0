"""Headline benchmark: SVDFormer PCN train-step samples/s on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

One step = one iteration of core/train_pcn.py:101-134 on a synthetic
PCN-shaped batch resident in HBM: depth render of the partial cloud
(PCViews) -> SVDFormer forward (models/SVDFormer.py) -> get_loss (three
sqrt-Chamfers, utils/loss_utils.py:33-58) -> backward -> Adam step.  The
model is randomly initialised (no checkpoints offline), 58.09 M parameters,
B=32 samples per GPU (configs[2] of BASELINE.json: bf16 autocast; point ops
stay fp32 inside).  Every point op and every attention core runs on
libpcops.so (hand-written gfx950 HIP); dense layers are torch (MIOpen /
hipBLASLt).  N>1: one process per GPU, batch-partitioned (weak scaling),
gradients all-reduced over RCCL by DDP -- the only data-path collective.

Rank 0 prints ONE JSON line (the driver's contract, kept under 8 KB: `compact`) with, in addition:
  roofline      -- the dominant libpcops op (the attention core, all passes): algorithmic FLOP per
                   launch / mean launch duration, HIP events on the launch stream;
  cpu_baseline  -- the same train step on the host CPU for a bounded sample
                   (oracle/cpu_path.py: torch CPU + the C restatement of the
                   point ops), rank 0 at N=1 only;
  kernels       -- the 10 largest libpcops call groups: launches / ms per step / frac;
  composite_fps_knn_chamfer -- sum of roofline times / sum of measured times for the FPS + kNN +
                   Chamfer launches on the reference's work model; composite_hw the same
                   on executed work (FPS on the VALU, the culled Chamfer's visited pairs).
The full per-kernel tables of every leg go to profiles/bench_detail_<time>.json (--detail-json)
and to stderr.
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12          # B/s, MI355X_MICROARCH.md (spec)
MFMA_BF16_PEAK = 2.5e15    # FLOP/s dense
MFMA_F32_PEAK = 157.3e12   # FLOP/s (f32 MFMA == f32 vector peak)
VALU_F32_PEAK = 157.3e12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", choices=("svdformer", "pointsea"), default="svdformer",
                    help="svdformer: PCN train step (configs[2]/[3], the headline); pointsea: ShapeNet-55 "
                         "train step with the PCViews_Real renderer (configs[4])")
    ap.add_argument("--batch", type=int, default=None, help="samples per GPU (32 PCN, 16 ShapeNet-55)")
    ap.add_argument("--fp32", action="store_true", help="no bf16 autocast (configs[1] numerics)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fp32-leg", action="store_true",
                    help="skip the configs[1] figure (fp32 forward + loss, B=16) reported beside the bf16 step")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="issue every launch from Python (no HIP graph)")
    ap.add_argument("--timing-steps", type=int, default=2, help="eager steps timed per launch (graph mode)")
    ap.add_argument("--tunableop", choices=("use", "tune", "off"), default="use",
                    help="PyTorch TunableOp for the dense GEMMs: 'use' the committed per-shape hipBLASLt "
                         "selections in tuning/ (if present), 'tune' them during warm-up (rank 0 "
                         "writes the file), or 'off' (library heuristics)")
    ap.add_argument("--overlap", choices=("auto", "off"), default="auto",
                    help="N>1 (or --dist-selftest): 'auto' all-reduces the gradient bucket by bucket from "
                         "backward hooks, inside the captured graph (train.BucketedAllReduce), falling back "
                         "to one all-reduce between the graph replays if capture refuses it; 'off' always "
                         "uses the single all-reduce")
    ap.add_argument("--bucket-mb", type=float, default=25.0, help="gradient bucket size for --overlap auto")
    ap.add_argument("--dist-selftest", action="store_true",
                    help="initialise an RCCL process group even at N=1 (exercises the collective path "
                         "and its graph capture on a one-GPU box)")
    ap.add_argument("--no-input-prefetch", action="store_true",
                    help="ShapeNet-55: crop + FPS the step's own input at its head (A/B of the input prefetch)")
    ap.add_argument("--no-extra-legs", action="store_true",
                    help="skip the fp32 PCN train step and the PointSea ShapeNet-55 train step reported beside "
                         "the headline (N = 1 only)")
    ap.add_argument("--dry-run-launch", action="store_true",
                    help="with --gpus N > 1 outside torch.distributed.run: print the rank launcher's argv and exit")
    ap.add_argument("--pmc-attn-json", default=os.path.join(ROOT, "profiles", "r6_pmc_attn.json"),
                    help="attention MFMA counters (tools/pmc_attn.py) -> attention.pmc_mfma_util")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "r6_pmc_traffic.json"),
                    help="HBM bytes per launch per kernel from rocprofv3 FETCH_SIZE/WRITE_SIZE passes "
                         "(tools/pmc_traffic.py) -> roofline.traffic")
    ap.add_argument("--pmc-json-pointsea", default=os.path.join(ROOT, "profiles", "r6_pmc_traffic_pointsea.json"),
                    help="the same HBM bytes table measured on the PointSea ShapeNet-55 step (its own shapes)")
    ap.add_argument("--pmc-valu-json", default=os.path.join(ROOT, "profiles", "r6_pmc_valu.json"),
                    help="VALU-busy counters per kernel (tools/pmc_valu.py) -> north_star_kernels.*.pmc_valu_busy")
    ap.add_argument("--visited-json", default=os.path.join(ROOT, "profiles", "r6_chamfer_visited.json"),
                    help="pairs the culled Chamfer evaluates per launch shape (tools/chamfer_visited.py) -> hw_frac")
    ap.add_argument("--emd-pairs-json", default=os.path.join(ROOT, "profiles", "r6_emd_pairs.json"),
                    help="auction bid pairs per shape (tools/emd_bench.py --count) -> emd.bid_gpairs_per_s")
    ap.add_argument("--emd-pmc-json", default=os.path.join(ROOT, "profiles", "r6_pmc_emd.json"),
                    help="VALU counters of the EMD kernels (tools/pmc_valu.py) -> emd.bid_pmc_valu_busy")
    ap.add_argument("--detail-json", default=None,
                    help="where the full per-kernel tables go (default profiles/bench_detail_<time>.json)")
    return ap.parse_args()


# ------------------------------------------------------------------ data
def synth_pcn(B, seed, device):
    """PCN-shaped synthetic batch: gt (B,16384,3) on random rotated
    ellipsoid surfaces inside the unit cube; partial (B,2048,3) = the half
    facing a random view, resampled to 2048 with replacement (the PCN
    loader's RandomSamplePoints).  The partial points are a second, independent
    sampling of the same surface (PCN's partials are separate renders, never
    gt's own points): with partial a subset of gt, a partial point that FPS
    keeps in the coarse prediction can land exactly on a gt_c point, and the
    sqrt-Chamfer gradient there is 0 * inf = NaN (it made some training runs
    diverge after a few steps, depending on the trajectory)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    d = torch.randn(B, 16384, 3, generator=g)
    d = d / d.norm(dim=-1, keepdim=True)
    axes = 0.15 + 0.3 * torch.rand(B, 1, 3, generator=g)
    q, _ = torch.linalg.qr(torch.randn(B, 3, 3, generator=g))
    gt = torch.bmm(d * axes, q)
    view = torch.randn(B, 3, generator=g)
    d2 = torch.randn(B, 16384, 3, generator=g)
    d2 = d2 / d2.norm(dim=-1, keepdim=True)
    scan = torch.bmm(d2 * axes, q)
    partial = torch.empty(B, 2048, 3)
    for b in range(B):
        vis = scan[b][(d2[b] @ (view[b] / view[b].norm())) > 0]
        pick = torch.randint(0, vis.shape[0], (2048,), generator=g)
        partial[b] = vis[pick]
    return partial.contiguous().to(device), gt.contiguous().to(device)


def synth_55(B, seed, device, n_gt=8192):
    """ShapeNet-55-shaped synthetic batch: gt (B,8192,3) random rotated
    ellipsoid surfaces normalised like the loader's pc_norm (centroid at 0,
    max radius 1); partial (B,2048,3) = gt minus the points nearest a random
    unit-sphere centre (a quarter to three quarters of them, as
    core/train_55.py:150), randomly resampled to 2048.  The train step
    re-derives its own partial on the device each step with
    data.seprate_point_cloud, as the reference's loop does."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    d = torch.randn(B, n_gt, 3, generator=g)
    d = d / d.norm(dim=-1, keepdim=True)
    axes = 0.3 + 0.7 * torch.rand(B, 1, 3, generator=g)
    q, _ = torch.linalg.qr(torch.randn(B, 3, 3, generator=g))
    gt = torch.bmm(d * axes, q)
    gt = gt - gt.mean(dim=1, keepdim=True)
    gt = gt / gt.norm(dim=-1).amax(dim=1).view(B, 1, 1)
    partial = torch.empty(B, 2048, 3)
    for b in range(B):
        c = torch.randn(1, 3, generator=g)
        c = c / c.norm()
        ncrop = int(torch.randint(n_gt // 4, 3 * n_gt // 4 + 1, (1,), generator=g))
        keep = torch.argsort((gt[b] - c).norm(dim=-1))[ncrop:]
        partial[b] = gt[b][keep[torch.randint(0, keep.numel(), (2048,), generator=g)]]
    return partial.contiguous().to(device), gt.contiguous().to(device)


# ------------------------------------------------------------------ roofline model
# attention calls: B is followed by H, Lq, Lk, D, scale, dtype, 12 strides and 1 (forward) or 3 trailing
# args, so its position counts from the end (the *_colsum entries carry extra pointers before B)
ATTN_ARGS = {"attention forward": 20, "attention bwd dq": 22, "attention bwd dkv": 22, "attention bwd": 22}


def _attn_b(name, a):
    return len(a) - ATTN_ARGS[name]


def kernel_work(name, a):
    """(algorithmic amount, unit, peak, bound) for one libpcops call with int args `a`.

    Per-unit figures are SURVEY.md 8(d)'s, restated in DESIGN.md:
      attention fwd   4*BH*Lq*Lk*D FLOP (QK^T + PV)
      attention dkv   8*BH*Lq*Lk*D FLOP (S recompute, dP, dV, dK)
      attention dq    2*BH*Lq*Lk*D FLOP (dQ only, delta = rowsum(dO*O) fused in; the S/dP recompute in this
                      pass is overhead, not credited -- FA2's 10*BH*Lq*Lk*D
                      total backward count)
      attention bwd   10*BH*Lq*Lk*D FLOP (the one-call backward: delta, dK/dV storing dS, dQ = dS K)
      FPS             16 B per point-iteration, B*N*M of them (HBM model)
      Chamfer fwd     8 FLOP per pair, 2*B*N*M pairs (both directions)
      kNN             (2C+2) FLOP per (query, candidate) pair (distance part)
      glue kernels    bytes that must cross HBM once (each branch states its count)
    """
    if name in ATTN_ARGS:
        i = _attn_b(name, a)  # position of B; then H, Lq, Lk, D, scale, dtype
        BH, Lq, Lk, D, dt = a[i] * a[i + 1], a[i + 2], a[i + 3], a[i + 4], a[i + 6]
        mult = {"attention forward": 4.0, "attention bwd dkv": 8.0, "attention bwd dq": 2.0, "attention bwd": 10.0}[name]
        return mult * BH * Lq * Lk * D, "TFLOP/s", MFMA_BF16_PEAK if dt == 1 else MFMA_F32_PEAK, "mfma"
    if name == "attention bwd delta":
        BH, Lq, D, dt = a[2] * a[3], a[4], a[5], a[6]
        return (2.0 * BH * Lq * D * (4 if dt == 0 else 2) + 4.0 * BH * Lq), "GB/s", HBM_PEAK, "hbm"
    if name == "layernorm_fwd":  # a, adt, b, bdt, gamma, beta, eps, rows, C, y32, y16
        adt, has_b, bdt, rows, C = a[1], a[2] is not None, a[3], a[7], a[8]
        per = (4 if adt == 0 else 2) + ((4 if bdt == 0 else 2) if has_b else 0) + 6
        return float(per) * rows * C, "GB/s", HBM_PEAK, "hbm"
    if name == "layernorm_bwd" and len(a) == 23:
        # pcops_layernorm_bwd_ex: dy, dyt, ld, dy_x, dy16, a, adt, b, bdt, gamma, mean, rstd, rows, C, dx32, dx16, ...
        # read a (+ b), dy (+ dy_x) (+ dy16), write dx32 / dx16 as present
        dyt, has_x, has_16, adt, has_b, bdt, rows, C = a[1], a[3] is not None, a[4] is not None, a[6], \
            a[7] is not None, a[8], a[12], a[13]
        per = ((4 if adt == 0 else 2) + ((4 if bdt == 0 else 2) if has_b else 0) + (4 if dyt == 0 else 2)
               + (2 if has_x else 0) + (2 if has_16 else 0) + (4 if a[14] is not None else 0)
               + (2 if a[15] is not None else 0))
        return float(per) * rows * C, "GB/s", HBM_PEAK, "hbm"
    if name == "layernorm_bwd":
        adt, has_b, bdt, rows, C = a[3], a[4] is not None, a[5], a[9], a[10]
        per = (4 if adt == 0 else 2) + ((4 if bdt == 0 else 2) if has_b else 0) + 6 + 4 + 2
        return float(per) * rows * C, "GB/s", HBM_PEAK, "hbm"
    if name == "furthest_point_sampling":
        B, N, M = a[1], a[2], a[3]
        return 16.0 * B * N * M, "GB/s", HBM_PEAK, "hbm"
    if name == "chamfer_3D.forward":  # over the pairs evaluated: the culled search visits a fraction of them
        B, N, M = a[2], a[3], a[4]
        f = (kernel_table.visited or {}).get(f"{N}x{M}", 1.0)
        return 8.0 * 2 * B * N * M * f, "TFLOP/s", VALU_F32_PEAK, "valu"
    if name == "knn":
        B, S, N, C = a[2], a[3], a[4], a[5]
        return (2.0 * C + 2) * B * S * N, "TFLOP/s", VALU_F32_PEAK, "valu"
    # ---- HBM-bound glue kernels: bytes that must cross HBM once (reads + writes)
    es = lambda code: 2 if code == 1 else 4  # dtype code 0 = fp32, 1 = bf16  # noqa: E731
    if name == "colsum":        # g, gdt, rows, C, out, outdt: read the (rows, C) gradient once
        return float(a[2] * a[3] * es(a[1]) + a[3] * es(a[5])), "GB/s", HBM_PEAK, "hbm"
    if name == "transpose_add":  # a, adt, b, bdt, out, odt, out2, o2dt, B, R, C
        n = a[8] * a[9] * a[10]
        per = es(a[1]) + (es(a[3]) if a[2] else 0) + es(a[5]) + (es(a[7]) if a[6] else 0)
        return float(n * per), "GB/s", HBM_PEAK, "hbm"
    if name == "pcsa_forward":   # x, xdt, gates, gdt, basis, patches, K, C, out: read x, write out
        n = a[5] * a[6] * a[7]
        return float(2 * n * es(a[1]) + a[5] * a[6] * es(a[3])), "GB/s", HBM_PEAK, "hbm"
    if name == "pcsa_backward":  # x, xdt, g, gdt, gates, gatesdt, basis, patches, K, C, dx, dgates
        n = a[7] * a[8] * a[9]
        return float(n * (2 * es(a[1]) + es(a[3])) + 2 * a[7] * a[8] * es(a[5])), "GB/s", HBM_PEAK, "hbm"
    if name == "gather_points":  # features, idx, B, C, N, M: 4 B per index + read value + write out
        B, C, M = a[2], a[3], a[5]
        return float(4 * B * M + 8 * B * C * M), "GB/s", HBM_PEAK, "hbm"
    if name == "gather_points_grad":  # grad_out, idx, B, C, N, M, out: zero out, read grad + idx, scatter-add
        B, C, N, M = a[2], a[3], a[4], a[5]
        return float(4 * B * C * N + 4 * B * M + 8 * B * C * M), "GB/s", HBM_PEAK, "hbm"
    if name == "group_points":   # features, idx, B, C, N, S, K
        B, C, S, K = a[2], a[3], a[5], a[6]
        return float(4 * B * S * K + 8 * B * C * S * K), "GB/s", HBM_PEAK, "hbm"
    if name == "group_points_grad":
        B, C, N, S, K = a[2], a[3], a[4], a[5], a[6]
        return float(4 * B * C * N + 4 * B * S * K + 8 * B * C * S * K), "GB/s", HBM_PEAK, "hbm"
    if name == "sa_group":       # xyz, new_xyz, points_t, idx, B, N, S, K, C, out, odt: per output row read
        B, S, K, C, odt = a[4], a[6], a[7], a[8], a[10]   # the index, 12 B of xyz + 4C of points, write 3+C
        rows = B * S * K
        return float(rows * (4 + 12 + 4 * C + (3 + C) * es(odt)) + 12 * B * S), "GB/s", HBM_PEAK, "hbm"
    if name == "sa_group_grad":  # g, gdt, idx, B, N, S, K, C, gp: zero gp, read g[..., 3:] + idx, scatter-add
        gdt, B, N, S, K, C = a[1], a[3], a[4], a[5], a[6], a[7]
        return float(4 * B * N * C + B * S * K * (4 + C * (es(gdt) + 4))), "GB/s", HBM_PEAK, "hbm"
    if name == "edge_group":     # x, idx, B, N, K, C, out, odt: read the (B,N,C) cloud + the index, write 2C per row
        B, N, K, C, odt = a[2], a[3], a[4], a[5], a[7]
        return float(B * N * C * 4 + B * N * K * (4 + 2 * C * es(odt))), "GB/s", HBM_PEAK, "hbm"
    if name == "edge_group_grad":  # g, gdt, idx, B, N, K, C, gx: read g once + idx, write gx, scatter-add C per row
        gdt, B, N, K, C = a[1], a[3], a[4], a[5], a[6]
        return float(B * N * K * (2 * C * es(gdt) + 4 + 4 * C) + B * N * C * 4), "GB/s", HBM_PEAK, "hbm"
    if name == "chamfer_3D.backward":  # xyz1, xyz2, B, n, m: per point read xyz, partner xyz, grad, idx; write own
        B, n, m = a[2], a[3], a[4]       # grad, scatter-add the partner's (12 + 12 + 4 + 4 + 12 + 12 B)
        return float(56 * B * (n + m)), "GB/s", HBM_PEAK, "hbm"
    if name == "batchnorm_fwd":  # x, dt, res, rdt, rows, C, ..., batch_stats (12): x read by the stats pass
        n, e = a[4] * a[5], es(a[1])   # and the apply pass (two passes: the statistics precede the
        return float(n * e * (2 if a[12] else 1) + (n * es(a[3]) if a[2] else 0) + n * e), "GB/s", HBM_PEAK, "hbm"
    if name == "batchnorm_bwd":  # dy, y, x, dt, rows, C, ..., act (10), ..., dres (13): dy / y / x read by the
        n, e = a[4] * a[5], es(a[3])   # reduce and the apply pass, dx (+ dres) written once
        rd = 3 if a[10] else 2
        return float(2 * rd * n * e + n * e * (2 if a[13] else 1)), "GB/s", HBM_PEAK, "hbm"
    if name in ("conv3x3_fwd", "conv3x3_dgrad"):  # x, w, N, H, W, C, y: read the input, write the output once
        return float(2 * 2 * a[2] * a[3] * a[4] * a[5]), "GB/s", HBM_PEAK, "hbm"
    if name == "conv3x3_wgrad":  # x, dy, N, H, W, C: read both activations once
        return float(2 * 2 * a[2] * a[3] * a[4] * a[5]), "GB/s", HBM_PEAK, "hbm"
    if name == "add":            # a, adt, b, bdt, out, odt, n
        return float(a[6] * (es(a[1]) + es(a[3]) + es(a[5]))), "GB/s", HBM_PEAK, "hbm"
    if name == "adam_flat":      # param, g16, g32, n16, n, m, v, shadow, ...: read g + p, m, v; write p, m, v (+ shadow)
        n16 = a[3] if a[1] else 0
        sh = a[3] if a[7] else 0
        return float(a[4] * 28 - n16 * 2 + sh * 2), "GB/s", HBM_PEAK, "hbm"
    if name == "blend":          # score, sdt, a, b, n, out, odt: read score + two fp32 streams, write out
        return float(a[4] * (es(a[1]) + 8 + es(a[6]))), "GB/s", HBM_PEAK, "hbm"
    if name == "blend_bwd":      # g, gdt, score, sdt, a, b, n, da, db, ds: read g, score, a, b; write da, db, ds
        return float(a[6] * (es(a[1]) + 2 * es(a[3]) + 16)), "GB/s", HBM_PEAK, "hbm"
    if name == "add_rows":       # a, adt, b, bdt, out, odt, rows, C, ld_out: read a + b, write out's rows
        return float(a[6] * a[7] * (es(a[1]) + es(a[3]) + es(a[5]))), "GB/s", HBM_PEAK, "hbm"
    if name == "linear_skinny":  # x, rows, K, A, bias, y, N: read x, write y (bf16; the weight stays on chip)
        return float(2 * a[1] * (a[2] + a[6])), "GB/s", HBM_PEAK, "hbm"
    if name == "add_posemb":     # a, adt, cd, div, B, N, H, out, odt: read a + cd, write out
        return float(a[4] * a[5] * (a[6] * (es(a[1]) + es(a[8])) + 4)), "GB/s", HBM_PEAK, "hbm"
    if name == "max_k":          # x, dt, rows, K, C, out, arg: read K rows, write the max + a uint8 argmax
        return float(a[2] * a[4] * ((a[3] + 1) * es(a[1]) + 1)), "GB/s", HBM_PEAK, "hbm"
    if name == "max_k_grad":     # g, dt, arg, rows, K, C, gx: read g + argmax, write the K rows
        return float(a[3] * a[5] * ((a[4] + 1) * es(a[1]) + 1)), "GB/s", HBM_PEAK, "hbm"
    if name == "sum_rows":       # part, S, N, out, odt: read S fp32 rows, write one
        return float(a[1] * a[2] * 4 + a[2] * es(a[4])), "GB/s", HBM_PEAK, "hbm"
    if name == "wgrad_skinny":   # g, x, T, Co, Ci: read both operands once
        return float(a[2] * (a[3] + a[4]) * 2), "GB/s", HBM_PEAK, "hbm"
    if name in ("conv3x3_c1_fwd", "conv3x3_c1_wgrad"):  # x, w|dy, N, H, W: fp32 image + 16-ch bf16 map
        return float(a[2] * a[3] * a[4] * (4 + 32)), "GB/s", HBM_PEAK, "hbm"
    if name == "gelu_bwd":       # dy, u, dt, rows, C, du: read dy and u, write du
        return float(3 * a[3] * a[4] * es(a[2])), "GB/s", HBM_PEAK, "hbm"
    if name == "points2depth":   # points, rot, trans, B, N, V, H, W: read the cloud, accumulate 8 B / pixel
        B, N, V, H, W = a[3], a[4], a[5], a[6], a[7]  # (written + re-read), write the image
        return float(12 * B * N + 20 * B * V * H * W), "GB/s", HBM_PEAK, "hbm"
    if name == "points2grid":    # points, rot, rot2, trans, B, N, V, R, D: read cloud, write the voxel grid
        B, N, V, R, D = a[4], a[5], a[6], a[7], a[8]
        return float(12 * B * N + 4 * B * V * D * R * R), "GB/s", HBM_PEAK, "hbm"
    if name == "grid2image":     # grid, kern, BV, D, R: read the grid, write 3-channel image
        BV, D, R = a[2], a[3], a[4]
        return float(4 * BV * D * R * R + 12 * BV * R * R), "GB/s", HBM_PEAK, "hbm"
    return None


def hw_work(name, a, visited=None):
    """(work, unit, peak, bound) on the work the kernel really executes, where that differs from
    kernel_work's reference model:
      FPS      8 FLOP per point-iteration (3 sub, mul, 2 fma of the reference's distance) on the
               VALU: the cloud stays in registers, so the 16-B/point-iteration HBM sweep of the
               reference's kernel (sampling_gpu.cu:69-173) never happens -- a hardware frac of the
               WHOLE chip, though one cloud occupies one CU;
      Chamfer  8 FLOP per pair over the pairs the culled search actually evaluates (the visited
               fraction per launch shape from a counting build, tools/chamfer_visited.py), the
               all-pairs kernels over all pairs."""
    if name == "furthest_point_sampling":
        B, N, M = a[1], a[2], a[3]
        return 8.0 * B * N * M, "TFLOP/s", VALU_F32_PEAK, "valu"
    if name == "chamfer_3D.forward":
        B, N, M = a[2], a[3], a[4]
        f = (visited or {}).get(f"{N}x{M}")
        if f is None:
            f = 1.0 if N * M < (1 << 24) else None   # below 2^24 pairs the all-pairs screens run
        return (None if f is None else 8.0 * 2 * B * N * M * f), "TFLOP/s", VALU_F32_PEAK, "valu"
    w = kernel_work(name, a)
    return w if w is None or w[3] != "hbm" else None


# libpcops call -> the HIP kernel symbol(s) it launches (for the PMC lookup)
_SYMBOLS = {"attention forward": "attn_fwd2_kernel", "attention bwd dq": "attn_dq2_kernel",
            "attention bwd": "attn_(delta2|dkv3|dqs)_kernel",
            "attention bwd dkv": "attn_dkv[23]_kernel", "furthest_point_sampling": "fps_(reg|stream|wave|mw)_kernel",
            "furthest_point_sampling_counts": "fps_reg_kernel<[0-9]+, (true|false), true>",
            "chamfer_3D.forward": (r"chamfer_(nn|screen|mfma|cull|cull_prep)_kernel", r"chamfer_(nn|screen|mfma|cull)_kernel"), "knn": "knn", "layernorm_fwd": "ln_fwd_kernel",
            "layernorm_bwd": "ln_bwd_kernel", "attention bwd delta": "attn_delta_kernel",
            "colsum": ("colsum", "colsum_partial"),
            "transpose_add": "transpose_add", "pcsa_forward": "pcsa_fwd", "pcsa_backward": "pcsa_bwd",
            "gather_points": "gather_kernel", "gather_points_grad": "gather_grad_kernel",
            "group_points": "group_kernel", "group_points_grad": "group_grad_kernel",
            "chamfer_3D.backward": "chamfer_grad_seg", "points2depth": "depth_", "points2grid": "points2grid",
            "grid2image": "grid2image|image_normalize", "sa_group": "sa_group_kernel",
            "sa_group_grad": "sa_group_grad_kernel",
            # calls that launch several kernels: (every kernel of the call, the one launched once per call)
            "batchnorm_fwd": (r"bn_partial_kernel<\d, 0>|bn_final_kernel<0|bn_apply_kernel|bn_eval_coef",
                              r"bn_apply_kernel"),
            "batchnorm_bwd": (r"bn_partial_kernel<\d, [123]>|bn_final_kernel<1|bn_bwd_apply_kernel",
                              r"bn_bwd_apply_kernel"),
            "conv3x3_fwd": r"conv3x3_fwd_kernel", "conv3x3_dgrad": r"conv3x3_fwd_kernel",
            "conv3x3_wgrad": (r"conv3x3_wgrad_kernel|conv3x3_wgrad_reduce", r"conv3x3_wgrad_kernel"),
            "add": r"add_kernel", "max_k": r"max_k_kernel", "max_k_grad": r"max_k_grad_kernel",
            "blend": r"blend_fwd_kernel", "blend_bwd": r"blend_bwd_kernel", "add_posemb": r"add_posemb_kernel",
            "adam_flat": r"adam_flat_kernel",
            "gelu_bwd": (r"gelu_bwd_partial_kernel|colsum_final", r"gelu_bwd_partial_kernel"),
            "edge_group": r"edge_group_kernel",
            "edge_group_grad": (r"edge_group_grad_own_kernel|edge_group_grad_scatter_kernel",
                                r"edge_group_grad_own_kernel")}


def pmc_traffic(path, key, name):
    """Launch-weighted HBM bytes per launch of the kernels behind one call group,
    from a tools/pmc_traffic.py summary (None if absent)."""
    import re
    if not path or not os.path.exists(path) or name not in _SYMBOLS:
        return None
    pat = _SYMBOLS[name]
    prim = None
    if isinstance(pat, tuple):   # several kernels per call: their bytes summed per launch of `prim`
        pat, prim = pat
    m = re.search(r"D=(\d+)", key)
    if m:  # attention kernels are instantiated per head dim: <D, ...> / ILiDE
        pat += r"(<|ILi)%s(,|E)" % m.group(1)
    table = json.load(open(path))
    rows = [v for k, v in table.items() if re.search(pat, k)]
    n = sum(r["launches"] for r in rows) if prim is None else \
        sum(v["launches"] for k, v in table.items() if re.search(prim, k))
    return sum(r["hbm_bytes_per_launch"] * r["launches"] for r in rows) / n if n else None


def kernel_table(spans):
    """Group recorded calls by (name, shape) and attach roofline fractions."""
    rows = {}
    for name, evs in spans.items():
        for e0, e1, args in evs:
            key = name
            if name in ATTN_ARGS:
                i = _attn_b(name, args)
                key = f"{name} [D={args[i + 4]}, {'bf16' if args[i + 6] == 1 else 'fp32'}]"
            r = rows.setdefault(key, {"name": name, "launches": 0, "ms": 0.0, "work": 0.0, "hw": 0.0})
            r["launches"] += 1
            r["ms"] += e0.elapsed_time(e1)
            w = kernel_work(name, args)
            if w is not None:
                r["work"] += w[0]
                r["unit"], r["peak"], r["bound"] = w[1], w[2], w[3]
            if name == "chamfer_3D.forward":
                r["allpairs"] = r.get("allpairs", 0.0) + 16.0 * args[2] * args[3] * args[4]
            h = hw_work(name, args, kernel_table.visited)
            if h is None or h[0] is None:
                r["hw"] = None
            elif r["hw"] is not None:
                r["hw"] += h[0]
                r["hw_unit"], r["hw_peak"] = h[1], h[2]
    for r in rows.values():
        if "peak" in r and r["ms"] > 0:
            rate = r["work"] / (r["ms"] * 1e-3)
            r["achieved"] = rate / (1e12 if r["unit"] == "TFLOP/s" else 1e9)
            r["frac"] = rate / r["peak"]
            r["roof_ms"] = r["work"] / r["peak"] * 1e3
        if r.get("hw") and r["ms"] > 0 and "hw_peak" in r:
            rate = r["hw"] / (r["ms"] * 1e-3)
            r["hw_achieved"] = rate / (1e12 if r["hw_unit"] == "TFLOP/s" else 1e9)
            r["hw_frac"] = rate / r["hw_peak"]
            r["hw_roof_ms"] = r["hw"] / r["hw_peak"] * 1e3
    return rows


kernel_table.visited = None   # "NxM" -> visited pair fraction of the culled Chamfer (tools/chamfer_visited.py)


def _attn_pmc(pa):
    """Time-weighted MFMA utilisation of the attention kernels from a tools/pmc_attn.py pass."""
    if not pa or not os.path.exists(pa):
        return None
    tab = json.load(open(pa))
    tw = sum(v["avg_us"] * v["launches"] for v in tab.values() if "mfma_util" in v)
    if tw <= 0:
        return None
    return round(sum(v["mfma_util"] * v["avg_us"] * v["launches"] for v in tab.values() if "mfma_util" in v) / tw, 4)


def _valu_pmc(path, name):
    """VALU busy fraction of the kernels behind one call group, launch-time weighted, from a
    tools/pmc_valu.py pass (SQ_ACTIVE_INST_VALU / SQ_BUSY_CU_CYCLES-style counters), or None."""
    import re
    if not path or not os.path.exists(path) or name not in _SYMBOLS:
        return None
    pat = _SYMBOLS[name]
    pat = pat[0] if isinstance(pat, tuple) else pat
    rows = [v for k, v in json.load(open(path)).items() if re.search(pat, k) and "valu_busy" in v]
    tw = sum(v["avg_us"] * v["launches"] for v in rows)
    return round(sum(v["valu_busy"] * v["avg_us"] * v["launches"] for v in rows) / tw, 4) if tw > 0 else None


def kernel_summary(rows, spans, span_steps, step_ms, pmc_json, pmc_attn=None, pmc_valu=None):
    """The kernel fields of one train leg (the FULL set, written to the detail file; `compact`
    cuts them for the driver's one-line JSON):
      roofline   the dominant libpcops op by time.  Ops are families: the attention core's
                 forward / dQ / dK-dV launches at every head dim are one op (the reference's one
                 attention call), every other call group is its own;
      fps_us_per_round, composite_fps_knn_chamfer (the reference-model composite),
      composite_hw (the same three groups priced on executed work: FPS on the VALU, Chamfer on
                 the visited pairs), north_star_kernels, attention, kernels (every call group)."""
    out = {}

    def pmc_row(k, r):
        t = pmc_traffic(pmc_json, k, r["name"])
        if t is None or not r["launches"] or r["ms"] <= 0:
            return {}
        # measured HBM bandwidth: PMC bytes per launch / this run's HIP-event launch time
        row = {"pmc_bytes_per_launch": round(t), "pmc_gbs": round(t / (r["ms"] / r["launches"] * 1e-3) / 1e9, 2)}
        if r.get("work") and r.get("unit") == "GB/s":
            row["pmc_traffic_ratio"] = round(t / (r["work"] / r["launches"]), 3)
        return row

    timed = {k: r for k, r in rows.items() if "frac" in r}
    if not timed:
        return out
    att = [(k, r) for k, r in timed.items() if r["name"] in ATTN_ARGS and r["unit"] == "TFLOP/s"]
    att_ms = sum(r["ms"] for _, r in att)
    dom_key = max(timed, key=lambda k: timed[k]["ms"])
    pa = pmc_attn
    if att and att_ms >= timed[dom_key]["ms"]:
        w = sum(r["work"] for _, r in att)
        n = sum(r["launches"] for _, r in att)
        peak = max(r["peak"] for _, r in att)
        tr = [pmc_traffic(pmc_json, k, r["name"]) for k, r in att]
        traffic = (sum(t * r["launches"] for t, (_, r) in zip(tr, att)) / n) if all(t is not None for t in tr) else None
        big = max(att, key=lambda kr: kr[1]["ms"])
        out["roofline"] = {"kernel": "attention core (fwd + dQ + dK/dV passes, every head dim; libpcops attn_*_kernel)",
                           "bound": "mfma", "achieved": round(w / (att_ms * 1e-3) / 1e12, 2), "peak": peak / 1e12,
                           "unit": "TFLOP/s", "frac": round(w / (att_ms * 1e-3) / peak, 4),
                           "traffic": None if traffic is None else round(traffic),
                           "traffic_source": os.path.relpath(pmc_json, ROOT) if pmc_json and traffic else None,
                           "avg_launch_ms": round(att_ms / n, 4), "launches": n,
                           "work_per_launch": w / n, "pmc_mfma_util": _attn_pmc(pa),
                           "largest_call": {"kernel": big[0], "frac": round(big[1]["frac"], 4),
                                            "avg_launch_ms": round(big[1]["ms"] / big[1]["launches"], 4)}}
    else:
        d = timed[dom_key]
        out["roofline"] = {"kernel": dom_key, "bound": d["bound"], "achieved": round(d["achieved"], 2),
                           "peak": d["peak"] / (1e12 if d["unit"] == "TFLOP/s" else 1e9), "unit": d["unit"],
                           "frac": round(d["frac"], 4),
                           "traffic": pmc_traffic(pmc_json, dom_key, d["name"]),
                           "traffic_source": os.path.relpath(pmc_json, ROOT) if pmc_json else None,
                           "avg_launch_ms": round(d["ms"] / d["launches"], 4),
                           "work_per_launch": d["work"] / d["launches"]}
    # FPS is M-1 serially dependent rounds: its honest figure is time per round
    fps = {}
    for e0, e1, a in spans.get("furthest_point_sampling", []):
        f = fps.setdefault(f"B{a[1]} {a[2]}->{a[3]}", [0, 0.0, a[3]])
        f[0] += 1
        f[1] += e0.elapsed_time(e1)
    # the zero-padded crop clouds with per-cloud valid counts (xyz, counts, B, N, M, ...): N is
    # the padded width; the sweep stops at each cloud's count (no algorithmic bytes credited --
    # the counts live on the device)
    for e0, e1, a in spans.get("furthest_point_sampling_counts", []):
        f = fps.setdefault(f"B{a[2]} <={a[3]}->{a[4]} (counts)", [0, 0.0, a[4]])
        f[0] += 1
        f[1] += e0.elapsed_time(e1)
    out["fps_us_per_round"] = {k: round(v[1] * 1e3 / v[0] / max(1, v[2] - 1), 3) for k, v in fps.items()}
    names3 = ("furthest_point_sampling", "knn", "chamfer_3D.forward")
    group = [r for r in timed.values() if r["name"] in names3]
    if group:
        out["composite_fps_knn_chamfer"] = round(sum(r["roof_ms"] for r in group) / sum(r["ms"] for r in group), 4)
        if all(r.get("hw_roof_ms") is not None for r in group):
            out["composite_hw"] = round(sum(r["hw_roof_ms"] for r in group) / sum(r["ms"] for r in group), 4)

    # SURVEY 8(d)'s three north_star kernel groups side by side: the reference-model rate and frac
    # (FPS: the reference kernel's 16-B/point-iteration HBM sweep; Chamfer: all pairs), the frac on
    # executed work (hw_frac) and the rocprof counters (HBM bytes, VALU busy)
    vj = pmc_valu
    out["north_star_kernels"] = {}
    for k in names3:
        r = rows.get(k)
        if r is None or "frac" not in r:
            continue
        row = {"ms_per_step": round(r["ms"] / span_steps, 4), "model_achieved": round(r["achieved"], 2),
               "model_unit": r["unit"], "model_frac": round(r["frac"], 4)}
        if r.get("hw_frac") is not None:
            row.update(hw_achieved=round(r["hw_achieved"], 2), hw_unit=r["hw_unit"], hw_frac=round(r["hw_frac"], 4))
        if k == "chamfer_3D.forward":
            # the reference's all-pairs work at this speed (a rate, not a fraction of any roof), and
            # whether every culled shape had a visited-pair count (else those launches are priced all-pairs)
            row["allpairs_equiv_tflops"] = round(r.get("allpairs", 0.0) / (r["ms"] * 1e-3) / 1e12, 2)
            row["pricing"] = "visited pairs" if r.get("hw") is not None else "all pairs (no visited count)"
        vb = _valu_pmc(vj, k)
        if vb is not None:
            row["pmc_valu_busy"] = vb
        row.update({k2: v for k2, v in pmc_row(k, r).items() if k2 != "pmc_bytes_per_launch"})
        out["north_star_kernels"][k] = row

    # attention as ONE figure: credited FLOPs of every attention call / their summed launch time,
    # and the time-weighted MFMA utilisation of the attention kernels from a rocprofv3 --pmc pass
    # (tools/pmc_attn.py: SQ_VALU_MFMA_BUSY_CYCLES / (cycles x SIMDs))
    if att:
        w = sum(r["work"] for _, r in att)
        peak = max(r["peak"] for _, r in att)
        agg = {"ms_per_step": round(att_ms / span_steps, 4), "achieved_tflops": round(w / (att_ms * 1e-3) / 1e12, 2),
               "peak_tflops": peak / 1e12, "frac": round(w / (att_ms * 1e-3) / peak, 4)}
        u = _attn_pmc(pa)
        if u is not None:
            agg["pmc_mfma_util"] = u
            agg["pmc_source"] = os.path.relpath(pa, ROOT)
        out["attention"] = agg

    out["kernels"] = {k: {"launches_per_step": r["launches"] / span_steps,
                          "ms_per_step": round(r["ms"] / span_steps, 4),
                          "share": round(r["ms"] / span_steps / step_ms, 4),
                          **({"frac": round(r["frac"], 4), "bound": r["bound"]} if "frac" in r else {}),
                          **({"hw_frac": round(r["hw_frac"], 4)} if r.get("hw_frac") is not None and
                             r.get("hw_frac") != r.get("frac") else {}),
                          **pmc_row(k, r)}
                      for k, r in sorted(rows.items(), key=lambda kv: -kv[1]["ms"])}
    return out


LINE_LIMIT = 8192   # bytes: the driver stopped parsing the line at 26 KB (BENCH_r05 parsed: null)


def _short_roof(r):
    return {k: r[k] for k in ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic") if k in r}


def _short_kernels(ks, top=10):
    keep = ("launches_per_step", "ms_per_step", "frac", "hw_frac", "bound", "pmc_traffic_ratio")
    return {k: {f: v[f] for f in keep if f in v} for k, v in list(ks.items())[:top]}


def _short_leg(leg):
    out = {k: leg[k] for k in ("batch", "dtype", "steps", "ms_per_step", "samples_per_s", "execution") if k in leg}
    for k in ("composite_fps_knn_chamfer", "composite_hw"):
        if k in leg:
            out[k] = leg[k]
    if "roofline" in leg:
        out["roofline"] = _short_roof(leg["roofline"])
    if "attention" in leg:
        out["attention_frac"] = leg["attention"].get("frac")
    if "kernels" in leg:
        out["kernels_top3"] = {k: v.get("ms_per_step") for k, v in list(leg["kernels"].items())[:3]}
    return out


def compact(full, limit=LINE_LIMIT):
    """The driver's one JSON line from the full result: the contract's fields, roofline,
    cpu_baseline, the north_star groups, the attention aggregate, a 10-row kernel table and one
    summary per extra leg.  Fields are dropped from the least important end until it fits."""
    line = {k: v for k, v in full.items() if k not in ("kernels", "fp32_train_step", "pointsea_train_step",
                                                      "fp32_forward_loss", "cpu_baseline", "emd", "roofline")}
    line["roofline"] = full["roofline"] if "roofline" in full else None
    if "kernels" in full:
        line["kernels"] = _short_kernels(full["kernels"])
    if "fp32_forward_loss" in full:
        line["fp32_forward_loss"] = {k: full["fp32_forward_loss"][k] for k in ("batch", "ms_per_step", "samples_per_s")
                                     if k in full["fp32_forward_loss"]}
    for k in ("fp32_train_step", "pointsea_train_step"):
        if k in full:
            line[k] = _short_leg(full[k])
    if "emd" in full:
        line["emd"] = full["emd"]
    if "cpu_baseline" in full:
        cb = dict(full["cpu_baseline"])
        cb.pop("step_s", None)
        line["cpu_baseline"] = cb
    for drop in ("kernels", "fps_us_per_round", "emd", "host_issue_ms_per_step", "kernel_timing"):
        if len(json.dumps(line)) < limit:
            break
        if drop == "kernels" and "kernels" in line:
            line["kernels"] = _short_kernels(full["kernels"], top=5)
        else:
            line.pop(drop, None)
    return json.dumps(line)


# ------------------------------------------------------------------ workloads
class Workload:
    """One of the two train steps: the reference loop it restates, its model,
    renderer, loss and optimizer."""

    def __init__(self, name):
        self.name = name
        if name == "svdformer":   # core/train_pcn.py:101-134
            from svdformer_pointsea_amd.render import PCViews
            from svdformer_pointsea_amd.svdformer import Model, PCNConfig
            self.Model, self.cfg, self.batch, self.n_out = Model, PCNConfig, 32, 16384
            self.render = PCViews(TRANS=-PCNConfig.NETWORK.view_distance, RESOLUTION=224)
            self.synth = synth_pcn
            self.metric = "train-step samples/sec (PCN, B=32, 2048->16384 pts)"
            self.desc = "SVDFormer PCN train step: render + fwd + get_loss + bwd + Adam"
        else:                      # core/train_55.py:141-181 with models_PointSea/PointSea.py
            from svdformer_pointsea_amd.pointsea import Config55, Model
            from svdformer_pointsea_amd.render import PCViews_Real
            self.Model, self.cfg, self.batch, self.n_out = Model, Config55, 16, 8192
            self.render = PCViews_Real(TRANS=-Config55.NETWORK.view_distance)
            self.synth = synth_55
            self.metric = "train-step samples/sec (PointSea ShapeNet-55, B=16, 2048->8192 pts)"
            self.desc = ("PointSea ShapeNet-55 train step: seprate_point_cloud + PCViews_Real render + fwd + "
                         "get_loss_PM + bwd + AdamW")

    def optimizer(self, params, lr=1e-4, **kw):
        if self.name == "svdformer":   # train_pcn.py:57-60
            return torch.optim.Adam(params, lr=lr, betas=(0.9, 0.999), weight_decay=0, **kw)
        return torch.optim.AdamW(params, lr=lr, weight_decay=0.0005, **kw)   # train_55.py:86-88

    def images(self, partial, cpu=False):
        if cpu:
            from oracle.cpu_path import depth_images, real_images
            if self.name == "svdformer":
                return depth_images(self.render, partial).unsqueeze(1)
            return real_images(self.render, partial)
        img = self.render.get_img(partial)
        return img.unsqueeze(1) if self.name == "svdformer" else img

    def inputs(self, partial, gt, generator=None):
        """The partial cloud the step sees: the loader's for PCN; for ShapeNet-55
        re-cropped from gt on the device every step (train_55.py:150)."""
        if self.name == "svdformer" or generator is None:
            return partial
        from svdformer_pointsea_amd.data import seprate_point_cloud
        n = gt.shape[1]
        return seprate_point_cloud(gt, n, [n // 4, 3 * n // 4], generator=generator, want_crop=False)[0]

    def gt_pyramid(self, gt):
        """The loss's gt FPS chain (n_out -> 2048 -> 256); depends on gt only."""
        from svdformer_pointsea_amd.metrics import gt_pyramid
        return gt_pyramid(gt, 2048, 256)

    def loss(self, pcds, partial, gt, gts=None):
        from svdformer_pointsea_amd.metrics import get_loss, get_loss_PM
        if self.name == "svdformer":
            return get_loss(pcds, gt, sqrt=True, gts=gts)[0]
        return get_loss_PM(pcds, partial, gt, sqrt=False, gts=gts)[0]


# ------------------------------------------------------------------ CPU baseline
def cpu_baseline(wl, steps):
    """The same train step on host cores for a bounded sample (1 sample/step)."""
    from oracle.cpu_path import cpu_ops

    nthreads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(nthreads)
    torch.manual_seed(0)
    model = wl.Model(wl.cfg)
    opt = wl.optimizer(model.parameters())
    partial, gt = wl.synth(1, 12345, "cpu")

    def step():
        depth = wl.images(partial, cpu=True)
        loss = wl.loss(model(partial, depth), partial, gt)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    with cpu_ops():
        step()  # warm-up
        times = []
        for _ in range(steps):
            t0 = time.perf_counter()
            step()
            times.append(time.perf_counter() - t0)
    med = sorted(times)[len(times) // 2]
    return {"value": 1.0 / med, "unit": "samples/s", "cores": nthreads, "kind": "port",
            "cpu_model": _cpu_model(), "host_cpus": os.cpu_count(),
            "cores_note": ("threads = OMP_NUM_THREADS: the GPU pool grants a one-GPU job a 16-CPU share of the "
                           "host (its OMP_NUM_THREADS); os.cpu_count() is the whole host's count"
                           if "OMP_NUM_THREADS" in os.environ else "threads = os.cpu_count()"),
            "step_s": [round(t, 3) for t in times],
            "sample": f"median of {steps} train steps of 1 {wl.name} sample (2048->{wl.n_out}) after 1 warm-up, "
                      f"fp32: torch CPU ({nthreads} threads) + oracle/pcops_oracle.c point ops (OpenMP, "
                      f"{nthreads} threads) + torch CPU attention"}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


# ------------------------------------------------------------------ configs[1] leg
def fp32_forward_loss(wl, model, partial, gt, device, steps, use_graph, batch=16):
    """BASELINE configs[1]: SVDFormer forward + get_loss on a PCN-shaped batch of
    16, fp32 throughout (no autocast; the fp32 master weights; exact-f32 MFMA
    attention core), timed per step with the inputs resident in HBM.  Captured
    in a HIP graph like the train step when the step is."""
    x, g = partial[:batch].contiguous(), gt[:batch].contiguous()
    was_training = model.training
    model.eval()   # forward + loss as the evaluation loop runs it (no BN-statistics update)

    def fwd():
        with torch.no_grad():
            depth = wl.images(x)
            return wl.loss(model(x, depth), x, g)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            fwd()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    run = fwd
    if use_graph:
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            fwd()
        run = gr.replay
    torch.cuda.synchronize()
    # PCOPS_TRACE_MARKS=configs1: spin kernels around these timed steps (tools/trace_window.py)
    marks = os.environ.get("PCOPS_TRACE_MARKS") == "configs1"
    if marks:
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    if marks:
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    model.train(was_training)
    return {"config": "BASELINE configs[1]: SVDFormer forward + get_loss, PCN shapes, fp32", "batch": batch,
            "steps": steps, "ms_per_step": round(dt * 1e3, 3), "samples_per_s": round(batch / dt, 2),
            "execution": "hip_graph" if use_graph else "eager"}


# ------------------------------------------------------------------ EMD (metrics/EMD, the auction)
def emd_leg(device, pairs_json=None, pmc_json=None, B=32, n=2048, eps=0.005, iters=50):
    """pcops_emd_forward / _backward at the reference's train settings (eps 0.005, 50 iterations:
    metrics/EMD/README.md:7) on uniform clouds (emd_module.py:90-106 draws torch.rand), timed live
    with HIP events (median of 3 after a warm-up); the bid pairs of the auction (unassigned bidders x
    objects, per launch shape, from the counting build: tools/emd_bench.py --count) turn the forward
    time into a pair rate, and a rocprofv3 pass over the bid kernel gives its VALU busy fraction."""
    from svdformer_pointsea_amd.emd_module import emdModule

    g = torch.Generator(device="cpu").manual_seed(n)
    x1 = torch.rand(B, n, 3, generator=g).to(device).requires_grad_(True)
    x2 = torch.rand(B, n, 3, generator=g).to(device)
    emd = emdModule()
    fw, bw = [], []
    for rep in range(4):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        x1.grad = None
        e0.record()
        dist, _ = emd(x1, x2, eps, iters)
        e1.record()
        dist.sum().backward()
        e2.record()
        torch.cuda.synchronize()
        if rep:
            fw.append(e0.elapsed_time(e1))
            bw.append(e1.elapsed_time(e2))
    out = {"shape": f"B{B} n{n}", "eps": eps, "iters": iters, "fwd_ms": round(sorted(fw)[1], 4),
           "bwd_ms": round(sorted(bw)[1], 4)}
    key = f"B{B} n{n}"
    if pairs_json and os.path.exists(pairs_json):
        c = json.load(open(pairs_json)).get(key)
        if c:
            out["bid_gpairs_per_s"] = round(c["active_pairs"] / (out["fwd_ms"] * 1e-3) / 1e9, 1)
            out["active_pair_frac"] = round(c["active_pairs"] / c["all_pairs"], 4)
    if pmc_json and os.path.exists(pmc_json):
        rows = [v for k, v in json.load(open(pmc_json)).items() if "emd_bid_kernel" in k and "valu_busy" in v]
        if rows:
            tw = sum(v["avg_us"] * v["launches"] for v in rows)
            out["bid_pmc_valu_busy"] = round(sum(v["valu_busy"] * v["avg_us"] * v["launches"] for v in rows) / tw, 4)
    return out


# ------------------------------------------------------------------ GEMM selection
def setup_tunableop(mode, model, rank):
    """hipBLASLt's default heuristic picks non-split-K tiles for the long-K
    weight-gradient GEMMs of this model ((512..3072) x 65536 x (512..1024)),
    leaving most of the 256 CUs idle.  PyTorch TunableOp times every hipBLASLt /
    rocBLAS solution per GEMM shape once; the winners are kept in a CSV that is
    committed and re-read on every run.  Returns the CSV path or None."""
    if mode == "off":
        return None
    import torch.cuda.tunable as tunable
    path = os.path.join(ROOT, "tuning", f"tunableop_{model}_gfx950.csv")
    if mode == "use" and not os.path.exists(path):
        return None
    tunable.enable(True)
    tunable.tuning_enable(mode == "tune")
    if mode == "tune":
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tunable.set_max_tuning_duration(5)     # ms per candidate solution
        tunable.set_max_tuning_iterations(8)
        import threading

        t0 = time.time()

        def beat():  # tuning is silent for minutes; keep the job's output alive
            while True:
                time.sleep(20)
                print(f"[tunableop] tuning, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

        threading.Thread(target=beat, daemon=True).start()
        tunable.set_filename(path if rank == 0 else path + f".rank{rank}", False)
    else:
        tunable.set_filename(path + ".unused", False)  # never write next to the committed file
        tunable.read_file(path)
    return path


# ------------------------------------------------------------------ main
_PHASE = ["start"]


def progress(msg):
    """One stderr line per phase: long phases stay visibly alive, and a stall names its phase."""
    _PHASE[0] = msg
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def heartbeat(every=30.0):
    """A daemon thread repeating the current phase (MIOpen's first-run kernel
    compilation and GEMM tuning are silent for minutes on a fresh box)."""
    import threading

    def beat():
        while True:
            time.sleep(every)
            print(f"[bench {time.strftime('%H:%M:%S')}] ... {_PHASE[0]}", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()


_RESULT_FD = None   # the original stdout when library banners are diverted (distributed runs)


def _free_port():
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_argv(argv, n, port):
    """The command `python bench.py --gpus N ...` (no WORLD_SIZE in the environment)
    runs as: one rank per GPU under torch.distributed.run on this node, the same
    arguments, rendezvous on 127.0.0.1 (the reference's counterpart is
    DataParallel over the node's GPUs, core/train_pcn.py:53-54)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def self_launch(args):
    """Start the N ranks as a child process (this process has not touched the GPU)
    and return its exit code; rank 0's JSON line reaches this stdout directly."""
    import subprocess

    cmd = launch_argv(sys.argv[1:], args.gpus, _free_port())
    if args.dry_run_launch:
        print(json.dumps({"launch": cmd}))
        return 0
    progress(f"launching {args.gpus} ranks: {' '.join(cmd)}")
    sys.stdout.flush()
    return subprocess.call(cmd, env=dict(os.environ))


class Leg:
    """One timed train-step measurement (model, flat parameters, optimizer,
    captured graphs, timings)."""


def train_leg(args, wl, batch, amp, steps, warmup, device, world, rank, use_dist, kernel_timing, tag):
    """Build wl's model, warm up, capture the step into HIP graphs (unless
    --no-graph) and time `steps` steps between barrier + synchronize pairs.
    Kernel timing (HIP events per libpcops launch) runs as eager steps after
    the timed replays; a non-finite loss anywhere -- warm-up, timed replays or
    the eager timing steps -- fails the run."""
    from svdformer_pointsea_amd import _lib
    from svdformer_pointsea_amd.train import BucketedAllReduce, FlatAdam, FlatParams, TrainSchedule

    L = Leg()
    torch.manual_seed(0)  # identical init on every rank
    model = wl.Model(wl.cfg).to(device)
    L.model, L.nparams = model, sum(p.numel() for p in model.parameters())
    # flat fp32 master weights + gradient bucket, bf16 shadows of the GEMM/conv
    # weights refreshed by one cast per step (svdformer_pointsea_amd/train.py)
    fp = L.fp = FlatParams(model, device, bf16=amp)
    use_graph = L.use_graph = not args.no_graph
    # one parameter group, elementwise update: Adam over the flat master buffer;
    # the LR is a device tensor so the captured optimizer graph reads the value
    # the schedule writes each step (warm-up per batch, train_pcn.py:132-134)
    opt = wl.optimizer([fp.master()], lr=torch.tensor(1e-4, device=device) if use_graph else 1e-4, fused=True,
                       capturable=use_graph)
    # the update itself on libpcops (train.FlatAdam): reads the bf16 gradient bucket, writes the bf16
    # shadows, keeps torch's optimizer state; PCOPS_FLAT_ADAM=0 runs torch's fused Adam (A/B)
    fopt = (FlatAdam(opt, fp) if fp.shadow and os.environ.get("PCOPS_FLAT_ADAM", "1") != "0" else None)
    L.optimizer_impl = "libpcops pcops_adam_flat" if fopt is not None else "torch fused Adam"
    if fopt is not None:
        fp.refresh()   # the first step's shadows; afterwards every update writes them
    schedule = TrainSchedule(opt, wl.name)
    partial, gt = wl.synth(batch, 1000 + rank, device)
    L.partial, L.gt = partial, gt
    # ShapeNet-55 re-crops its partial input from gt inside the step; the crop
    # draws come from the device's default generator (graph-capturable)
    crop_rng = torch.cuda.default_generators[device.index] if wl.name == "pointsea" else None
    loss_acc = torch.zeros((), device=device)
    progress(f"[{tag}] {wl.name} B={batch} {'bf16' if amp else 'fp32'}: {L.nparams} parameters; eager warm-up")
    sync = [BucketedAllReduce(fp, world, bucket_mb=args.bucket_mb) if use_dist and args.overlap == "auto" else None]

    # ShapeNet-55's input (seprate_point_cloud: crop + a 16-CU FPS, ~2 ms) depends on
    # gt and the crop draws only, not on the model: each step crops and FPS-samples
    # the NEXT step's input on a third stream beside its own forward/backward, as a
    # data loader's prefetch would (one crop per step, every one inside a timed
    # step; the first step's comes from before the clock).  --no-input-prefetch
    # puts it back at the head of the step's critical path (A/B).
    prefetch = crop_rng is not None and not args.no_input_prefetch
    staged = [wl.inputs(partial, gt, crop_rng)] if prefetch else None

    def fwd_bwd():
        fp.zero_grad()
        if fopt is None:
            fp.refresh()
        # the loss's gt FPS chain depends on gt only: it runs on a second
        # stream beside the whole forward pass (FPS occupies B CUs)
        with _lib.fork(device, lane=1, inputs=(gt,)) as br:
            gts = wl.gt_pyramid(gt)
        if prefetch:
            inp = staged[0].clone()   # this step's own buffer: the staged one is refilled below
            with _lib.fork(device, lane=2, inputs=(gt,)) as bn:
                nxt = wl.inputs(partial, gt, crop_rng)
        else:
            inp = wl.inputs(partial, gt, crop_rng)
        depth = wl.images(inp)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp, cache_enabled=not use_graph):
            pcds = fp.forward(inp, depth)
            loss = wl.loss(pcds, inp, gt, br.join(*gts))
        loss.backward()
        if sync[0] is not None:
            sync[0].finish()   # the bucketed all-reduces were issued during backward
        else:
            fp.collect(widen=fopt is None or use_dist)
        if prefetch:
            staged[0].copy_(bn.join(nxt))
        loss_acc.add_(loss.detach())  # logged without a host sync

    def grad_sync():
        if use_dist and sync[0] is None:
            fp.allreduce(world)

    def opt_step():
        if fopt is not None:
            fopt.step(bf16_grads=not use_dist)
        else:
            opt.step()

    def eager_step():
        fwd_bwd()
        grad_sync()
        opt_step()
        schedule.batch_end()

    def check_finite(what):
        v = loss_acc.item()
        if not math.isfinite(v):
            names = [n for n, q in model.named_parameters() if not torch.isfinite(q.detach()).all()]
            progress(f"[{tag}] non-finite running loss after {what}; master finite "
                     f"{bool(torch.isfinite(fp.flat).all())}, grad finite {bool(torch.isfinite(fp.grad[fp.n16:]).all())}"
                     # with FlatAdam the shadow region's gradients live in grad16 only (collect(widen=False))
                     f" / {bool(torch.isfinite(fp.grad16 if fopt is not None and not use_dist else fp.grad[:fp.n16]).all())}"
                     f" (fp32 / shadow region); "
                     f"{len(names)} parameters non-finite, first: {names[:6]}")
            raise RuntimeError(f"non-finite loss ({tag}, {what})")

    if use_graph:
        # The host cannot issue the ~3k launches of a step faster than the GPU
        # runs them (host_issue_ms_per_step), so the step is captured once
        # into two HIP graphs (forward+backward, optimizer) after eager
        # warm-up on a side stream (MIOpen algorithm search, lazy state)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(warmup, 2)):
                eager_step()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        check_finite("the eager warm-up")
        progress(f"[{tag}] eager warm-up done; capturing the step")
        g_fb, g_opt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        # RCCL's watchdog thread polls the warm-up collectives' events; under
        # "global" capture such a call from another thread invalidates the
        # capture, so collectives are captured in thread-local mode, after
        # the warm-up work has drained
        cap_mode = "global"
        if sync[0] is not None:
            dist.barrier()
            torch.cuda.synchronize()
            time.sleep(1.0)
            cap_mode = "thread_local"
        captured, err = True, None
        try:
            with torch.cuda.graph(g_fb, capture_error_mode=cap_mode):
                fwd_bwd()
        except RuntimeError as exc:
            if sync[0] is None:
                raise
            captured, err = False, exc
        if sync[0] is not None:
            # every rank must run the same collective schedule: the in-graph bucketed
            # all-reduces only if EVERY rank captured them (agreed over a host group,
            # outside any capture); otherwise every rank drops them together
            flag = torch.tensor([1 if captured else 0], dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=host_group())
            if int(flag.item()) == 0:
                progress(f"[{tag}] in-graph all-reduce not captured on every rank "
                         f"(this rank: {err or 'ok'}); one all-reduce after each replay on all ranks")
                for h in sync[0]._hooks:
                    h.remove()
                sync[0] = None
                torch.cuda.synchronize()
                g_fb = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g_fb):
                    fwd_bwd()
        with torch.cuda.graph(g_opt):
            opt_step()

        def step():
            g_fb.replay()
            grad_sync()
            g_opt.replay()
            schedule.batch_end()
        # one untimed replay first: the FIRST launch of the captured PointSea step gives the
        # MIOpen-run ResNet layers 1-3 gradients off by up to 3 % (later launches match eager within
        # its run-to-run spread; tools/capture_grad_report.py) -- a train step like
        # the warm-up ones, outside the clock
        step()
        torch.cuda.synchronize()
        check_finite("the first graph replay")
        span_steps = args.timing_steps
    else:
        step = eager_step
        for _ in range(warmup):
            step()
        check_finite("the eager warm-up")
        if kernel_timing:
            _lib.KernelTimer.enable()
        span_steps = steps

    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    progress(f"[{tag}] timing {steps} steps")
    # PCOPS_TRACE_MARKS=1: a spin kernel on each side of the timed steps, so a rocprofv3 kernel
    # trace can be cut to exactly the timed replays (tools/trace_window.py); outside the clock
    marks = os.environ.get("PCOPS_TRACE_MARKS") == "1" and tag == "headline"
    if marks:
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = 0.0  # time the host spends issuing a step (launches are asynchronous)
    for _ in range(steps):
        h0 = time.perf_counter()
        step()
        host += time.perf_counter() - h0
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if marks:
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    check_finite("the timed steps")
    L.idle_issue_ms = None
    if use_graph:
        # host cost of issuing one step's graph replays against an IDLE GPU: separates
        # the graph-launch cost of ~1.5 k nodes from queue back-pressure in host_issue
        # (these replays are extra train steps, outside the clock)
        idle = []
        for _ in range(3):
            torch.cuda.synchronize()
            h0 = time.perf_counter()
            step()
            idle.append(time.perf_counter() - h0)
        torch.cuda.synchronize()
        check_finite("the idle-issue steps")
        L.idle_issue_ms = 1e3 * sorted(idle)[1]
    if use_graph and kernel_timing:
        # ROCm torch refuses timing events inside a captured graph ("External
        # events are disallowed in rocm"), so the per-launch HIP events come
        # from eager steps of the same work right after the timed replays --
        # on a side stream, like the warm-up.  They are real train steps: a
        # non-finite loss there fails the run like one in the replays.
        _lib.KernelTimer.enable()
        tstream = torch.cuda.Stream()
        tstream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(tstream):
            for _ in range(args.timing_steps):
                eager_step()
        torch.cuda.current_stream().wait_stream(tstream)
        torch.cuda.synchronize()
        check_finite("the eager kernel-timing steps")
    L.spans = _lib.KernelTimer.spans or {}
    _lib.KernelTimer.disable()
    if use_dist:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    L.elapsed, L.host, L.span_steps, L.sync = elapsed, host, span_steps, sync[0]
    L.ms_per_step = elapsed * 1e3 / steps
    return L


_HOST_GROUP = [None]


def host_group():
    """A gloo group over the same ranks for host-side agreement (created collectively at start-up)."""
    return _HOST_GROUP[0]


def pmc_files(args, model, amp):
    """The counter files measured on THIS workload's own launches (traffic, attention MFMA, VALU): a
    table measured on another workload's shapes would misprice every ratio (round 5's PointSea
    leg read the PCN step's LayerNorm bytes against PointSea's algorithmic bytes)."""
    if not amp:
        return None, None, None
    if model == "pointsea":
        return args.pmc_json_pointsea, None, None
    return args.pmc_json, args.pmc_attn_json, args.pmc_valu_json


def extra_leg(args, name, batch, amp, device, steps):
    """A second train-step figure beside the headline (rank 0, N = 1)."""
    wl = Workload(name)
    setup_tunableop(args.tunableop, name, 0)
    leg = train_leg(args, wl, batch, amp, steps, 2, device, 1, 0, False, not args.no_kernel_timing,
                    name + ("" if amp else "-fp32"))
    out = {"workload": wl.desc, "batch": batch, "dtype": "bf16" if amp else "f32", "steps": steps,
           "ms_per_step": round(leg.ms_per_step, 3), "samples_per_s": round(batch * 1e3 / leg.ms_per_step, 2),
           "execution": "hip_graph" if leg.use_graph else "eager", "optimizer": leg.optimizer_impl}
    if name == "pointsea" and amp:
        out["input_prefetch"] = not args.no_input_prefetch
    # the leg's own libpcops kernel table (HIP events of its eager timing steps)
    out.update(kernel_summary(kernel_table(leg.spans), leg.spans, leg.span_steps, leg.ms_per_step,
                              *pmc_files(args, name, amp)))
    del leg
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def main():
    global _RESULT_FD
    args = parse()
    if args.visited_json and os.path.exists(args.visited_json):
        kernel_table.visited = {k: v["visited_frac"] for k, v in json.load(open(args.visited_json)).items()}
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N`: one rank per GPU, started before anything touches the GPU
        sys.exit(self_launch(args))
    heartbeat()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; the line would misreport n_gpus")
    use_dist = world > 1 or args.dist_selftest
    if use_dist:
        # RCCL prints its version banner on stdout at communicator set-up; stdout must carry
        # exactly one JSON line, so fd 1 points at stderr from here and the line goes to the
        # saved original
        sys.stdout.flush()
        _RESULT_FD = os.dup(1)
        os.dup2(2, 1)
        torch.cuda.set_device(local)
        if args.dist_selftest and "MASTER_ADDR" not in os.environ:
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        _HOST_GROUP[0] = dist.new_group(backend="gloo")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    # MIOpen picks the fastest conv algorithm per shape during the warm-up
    # steps (the image branch's NHWC convs: 14 -> 11 ms fwd+bwd)
    torch.backends.cudnn.benchmark = True

    import svdformer_pointsea_amd as pkg

    pkg.lib()  # fail loudly if libpcops.so is missing
    tuned = setup_tunableop(args.tunableop, args.model, rank)
    wl = Workload(args.model)
    if args.batch is None:
        args.batch = wl.batch
    amp = not args.fp32
    leg = train_leg(args, wl, args.batch, amp, args.steps, args.warmup, device, world, rank, use_dist,
                    not args.no_kernel_timing, "headline")
    elapsed, spans, span_steps, sync = leg.elapsed, leg.spans, leg.span_steps, leg.sync
    use_graph, host_ms, nparams = leg.use_graph, leg.host * 1e3 / args.steps, leg.nparams
    idle_issue_ms = leg.idle_issue_ms
    optimizer_impl = leg.optimizer_impl

    fp32_leg = None
    extra = {}
    if args.model == "svdformer" and not args.fp32 and not args.no_fp32_leg:
        progress("configs[1] leg: fp32 forward + get_loss, B=16")
        fp32_leg = fp32_forward_loss(wl, leg.model, leg.partial, leg.gt, device, steps=max(3, args.steps // 2),
                                     use_graph=use_graph)
    rows = kernel_table(spans)
    if world == 1 and not args.no_extra_legs and args.model == "svdformer" and not args.fp32:
        del leg
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        leg_steps = max(3, args.steps // 2)
        # the reference's own arithmetic (fp32, core/train_pcn.py:101-134 has no AMP) at the headline shape
        extra["fp32_train_step"] = extra_leg(args, "svdformer", args.batch, False, device, leg_steps)
        # configs[4]: the ShapeNet-55 PointSea step (core/train_55.py:141-181), one GPU's B = 16
        extra["pointsea_train_step"] = extra_leg(args, "pointsea", 16, True, device, leg_steps)
    out = None
    if rank == 0:
        samples = args.batch * world * args.steps
        out = {
            "metric": wl.metric,
            "value": samples / elapsed,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "host_issue_ms_per_step": host_ms,
            "host_issue_idle_gpu_ms": None if idle_issue_ms is None else round(idle_issue_ms, 3),
            "execution": "hip_graph" if use_graph else "eager",
            "optimizer": optimizer_impl,
            "grad_sync": ("none (single GPU)" if not use_dist else
                          f"bucketed all-reduce from backward hooks ({len(sync.buckets)} buckets of "
                          f"<= {args.bucket_mb:g} MB){' inside the captured graph' if use_graph else ''}"
                          if sync is not None else "one all-reduce of the flat bucket after backward"),
            "gemm_selection": (f"TunableOp ({args.tunableop}): {os.path.relpath(tuned, ROOT)}" if tuned
                               else "hipBLASLt heuristics"),
            "kernel_timing": ("HIP events per libpcops launch, %d eager steps after the timed graph replays"
                              % args.timing_steps) if use_graph else "HIP events per libpcops launch, timed steps",
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if args.fp32 else "bf16",
            "data": f"synthetic (random ellipsoid-surface {args.model} clouds, random-init weights)",
            "config": {"workload": wl.desc,
                       "global_batch": args.batch * world, "per_gpu_batch": args.batch, "points_in": 2048,
                       "points_out": wl.n_out, "params": nparams,
                       "parallelism": f"dp{world}" if world > 1 else "single"},
        }
        out.update(kernel_summary(rows, spans, span_steps, elapsed * 1e3 / args.steps,
                                  *pmc_files(args, args.model, amp)))
        if fp32_leg is not None:
            out["fp32_forward_loss"] = fp32_leg
        out.update(extra)
        if world == 1 and not args.no_extra_legs:
            progress("EMD at the reference's train settings")
            out["emd"] = emd_leg(device, args.emd_pairs_json, args.emd_pmc_json)
        if world == 1 and not args.no_cpu_baseline:
            progress(f"timed {out['ms_per_step']:.2f} ms/step; CPU baseline")
            out["cpu_baseline"] = cpu_baseline(wl, args.cpu_steps)
        # the full per-kernel tables go to a detail file and to stderr; stdout carries the compact line
        detail = args.detail_json or os.path.join(ROOT, "profiles", f"bench_detail_{time.strftime('%Y%m%d_%H%M%S')}.json")
        try:
            os.makedirs(os.path.dirname(detail), exist_ok=True)
            with open(detail, "w") as f:
                json.dump(out, f, indent=1)
        except OSError as exc:
            progress(f"detail file not written ({exc})")
        print("[bench detail] " + json.dumps(out), file=sys.stderr, flush=True)
        line = compact(out) + "\n"
        if _RESULT_FD is not None:
            sys.stdout.flush()
            os.write(_RESULT_FD, line.encode())
        else:
            print(line, end="", flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
