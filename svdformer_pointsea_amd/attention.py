"""Attention blocks of models/model_utils.py (:542-629) and
models_PointSea/model_utils.py (:385-509) on libpcops.so.

Parameter names match the reference exactly (multihead_attn.in_proj_weight,
multihead_attn.out_proj.weight, linear11, linear12, norm12, norm13,
input_proj, ...), so reference state_dicts load unchanged, and every block
keeps the reference's call signature: (B, C_in, L) in, (B, C_out, L) out.

Inside, a block runs token-major (B, L, C) -- the MI355X layout for it:
  * input_proj is a plain GEMM on the transposed input (the transpose is one
    LDS-tiled pass, csrc/blockops.hip, instead of permute + .contiguous());
  * norm13 / norm12 (with the residual add folded in) are one-pass fused
    LayerNorms that also emit the bf16 copy the next GEMM reads under
    autocast (no separate cast kernels);
  * the q/k/v projections stay packed: the attention core reads q, k and v as
    column windows of the projection output and writes dq/dk/dv into one
    packed gradient (no chunk / cat copies);
  * the output leaves through one fused add + transpose pass.
The attention core (softmax(QK^T/sqrt(hd)) V, forward and backward) is the
flash-style MFMA kernel: fp32 (exact f32 MFMA, the parity build) or bf16
(fp32 accumulate) following the dtype of its inputs (e.g. torch.autocast).
"""
import math
import os

import torch
import torch.nn.functional as F
from torch import nn
from torch.autograd import Function

from . import _lib
from ._lib import call, lib, ptr, stream_of

_DT = {torch.float32: 0, torch.bfloat16: 1}


def _dt(t):
    if t.dtype not in _DT:
        raise RuntimeError(f"unsupported dtype {t.dtype}")
    return _DT[t.dtype]


def _vptr(t, off=0):
    import ctypes

    return ctypes.c_void_p(t.data_ptr() + off * t.element_size())


# ------------------------------------------------------------------ linear layers
def _wgrad(g2, x2, wdt):
    """g2^T x2 for (T, Cout) x (T, Cin) with T = B*L tokens (up to 65536).

    hipBLASLt tiles this long-K, small-output GEMM (e.g. 512 x 512 x 65536)
    into a handful of workgroups (145-450 TFLOP/s).  Split-K instead: S
    batched partial GEMMs over T/S-token slices with fp32 outputs
    (torch.bmm(..., out_dtype=float32)), one fp32 sum, one rounding to the
    weight dtype -- 2-4x faster at these shapes (tools/gemm_bench.py)."""
    T, Cout = g2.shape
    Cin = x2.shape[1]
    if Cin == 6 and not g2.is_contiguous():
        g2 = g2.contiguous()
    if (Cin == 6 and Cout % 8 == 0 and Cout <= 64 and g2.is_cuda and g2.dtype == torch.bfloat16
            and x2.dtype == torch.bfloat16 and wdt in _DT and g2.data_ptr() % 16 == 0):
        # EdgeConv's 6 -> Cout conv: one streaming pass (as a split-K bmm it ran at 1.5 TFLOP/s)
        out = torch.empty(Cout, Cin, dtype=wdt, device=g2.device)
        wsb = lib().pcops_wgrad_skinny_workspace_bytes(Cout, Cin)
        ws = _lib.Workspace.get(g2.device, wsb)
        with torch.cuda.device(g2.device):
            call("wgrad_skinny", lib().pcops_wgrad_skinny, ptr(g2), ptr(x2), T, Cout, Cin, ptr(out), _DT[wdt], ptr(ws),
                 wsb, stream_of(g2))
        return out
    if not _WGRAD_SPLITK:
        return (g2.t() @ x2).to(wdt)
    S = 16 if Cout * Cin <= (2 << 20) else 4
    if Cout * Cin < (1 << 18) and _WGRAD_SMALL:
        # small outputs: 16 slices gave hipBLASLt 16 workgroups for the whole GEMM
        # (3 x 64 / 64 x 32 / 128 x 128 over 0.5-1 M tokens ran at 1.6-109 TFLOP/s);
        # about 2^20 partial elements over all slices: enough workgroups, and the
        # fixed-order sum of the slices (pcops_sum_rows) stays a few MB
        S = max(S, min(512, (1 << _WGRAD_SMALL_LOG2) // (Cout * Cin)))
        S = 1 << (S.bit_length() - 1)
    while S > 1 and (T % S or T // S < (1024 if S > 16 else _WGRAD_MINK)):
        S //= 2
    if S == 1 or g2.dtype != torch.bfloat16 or x2.dtype != torch.bfloat16:
        return (g2.t() @ x2).to(wdt)
    part = torch.bmm(g2.view(S, T // S, Cout).transpose(1, 2), x2.view(S, T // S, Cin), out_dtype=torch.float32)
    if wdt not in _DT or (Cout * Cin) % 4 or not part.is_cuda:
        return part.sum(0).to(wdt)
    # the S partials summed in a fixed order and rounded once, in one launch (pcops_sum_rows)
    out = torch.empty(Cout, Cin, dtype=wdt, device=part.device)
    with torch.cuda.device(part.device):
        call("sum_rows", lib().pcops_sum_rows, ptr(part), S, Cout * Cin, ptr(out), _DT[wdt], stream_of(part))
    return out


class _Linear(Function):
    """F.linear whose weight gradient is the split-K form of _wgrad; the input
    gradient (g @ W) and the bias gradient (a column sum) are torch's.  Under
    autocast the inputs are cast to bf16 like F.linear's autocast rule."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.bfloat16)
    def forward(ctx, x, w, b, b_dtype=None):
        ctx.save_for_backward(x, w)
        if _DEBUG_CONTIG:   # diagnostic: where the backward's operand copies come from
            import traceback
            ctx.site = " < ".join(f"{f.name}:{f.lineno}" for f in traceback.extract_stack(limit=7)[-7:-1][::-1])
        ctx.has_b = b is not None
        ctx.b_dtype = b_dtype   # the bias's own dtype (custom_fwd hands forward the bf16 cast)
        # on a side stream: GEMMs without stream-K (forward here, backward on
        # the same stream later -- autograd replays the forward's streams)
        ctx.side = _lib.on_side_stream()
        with _lib.no_stream_k() if ctx.side else _nullctx():
            return F.linear(x, w, b)

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        if _DEBUG_CONTIG and (not g.is_contiguous() or not x.is_contiguous()):
            import sys
            print(f"[contig] g {tuple(g.shape)} {g.stride()} x {tuple(x.shape)} {x.stride()} at {ctx.site}",
                  file=sys.stderr)
        C = g.shape[-1]
        g2 = g.reshape(-1, C)
        if not g2.is_contiguous() and not (_STRIDED_G and _row_strided(g2)):
            g2 = g2.contiguous()   # once, for all three uses
        # else g is a channel slice of a wider gradient (the output was concatenated with
        # others): the GEMMs read it with a leading dimension, colsum with a row stride
        gx = gw = gb = None
        with _lib.no_stream_k() if ctx.side else _nullctx():
            if ctx.needs_input_grad[0]:
                gx = (g2 @ w).view(x.shape)
            if ctx.needs_input_grad[1]:
                gw = _wgrad(g2, x.reshape(-1, x.shape[-1]).contiguous(), w.dtype)
        if ctx.has_b and ctx.needs_input_grad[2]:
            # a LayerNorm backward that consumed this output may have summed g
            # already (pcops_layernorm_bwd_colsum, attached to g); else one colsum
            pre = _take_sum(g)
            gb = pre if pre is not None else colsum(g2, out_dtype=ctx.b_dtype)
        if gb is not None and ctx.b_dtype is not None and gb.dtype != ctx.b_dtype:
            gb = gb.to(ctx.b_dtype)
        return gx, gw, gb, None


class _SkinnyLinear(Function):
    """F.linear for EdgeConv's skinny 1x1 convs under bf16 autocast (Cin in {6, 32, 64}, Cout in {32, 64},
    ~1 M edge rows): forward and input gradient on pcops_linear_skinny (the weight in registers, one
    32-row MFMA tile per wave) instead of the GEMM library's 32 x 256 tiles; weight gradient by _wgrad,
    bias gradient as _Linear's."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.bfloat16)
    def forward(ctx, x, w, b, b_dtype=None):
        K, N = x.shape[-1], w.shape[0]
        x2 = x.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        w = w.contiguous()
        y = torch.empty(x2.shape[0], N, dtype=torch.bfloat16, device=x.device)
        with torch.cuda.device(x.device):
            call("linear_skinny", lib().pcops_linear_skinny, ptr(x2), x2.shape[0], K, ptr(w),
                 ptr(None if b is None else b.contiguous()), ptr(y), N, stream_of(x))
        ctx.save_for_backward(x2, w)
        ctx.has_b, ctx.b_dtype, ctx.xshape = b is not None, b_dtype, x.shape
        ctx.side = _lib.on_side_stream()
        return y.view(*x.shape[:-1], N)

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, g):
        x2, w = ctx.saved_tensors
        N, K = w.shape
        g2 = g.reshape(-1, N)
        if not g2.is_contiguous() or g2.dtype != torch.bfloat16:
            g2 = g2.contiguous().to(torch.bfloat16)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            if N in (32, 64) and K in (32, 64):
                gx = torch.empty(g2.shape[0], K, dtype=torch.bfloat16, device=g2.device)
                with torch.cuda.device(g2.device):
                    call("linear_skinny", lib().pcops_linear_skinny, ptr(g2), g2.shape[0], N, ptr(w.t().contiguous()),
                         ptr(None), ptr(gx), K, stream_of(g2))
            else:
                with _lib.no_stream_k() if ctx.side else _nullctx():
                    gx = g2 @ w
            gx = gx.view(ctx.xshape)
        if ctx.needs_input_grad[1]:
            with _lib.no_stream_k() if ctx.side else _nullctx():
                gw = _wgrad(g2, x2, w.dtype)
        if ctx.has_b and ctx.needs_input_grad[2]:
            pre = _take_sum(g)
            gb = pre if pre is not None else colsum(g2, out_dtype=ctx.b_dtype)
            if ctx.b_dtype is not None and gb.dtype != ctx.b_dtype:
                gb = gb.to(ctx.b_dtype)
        return gx, gw, gb, None


# A/B switch (default off): EdgeConv's skinny 1x1 convs on pcops_linear_skinny.  Their kernels are 2-6x faster
# than the side stream's rocBLAS GEMMs (gcn_1 forward 395 -> 136 us, the input gradients too), but the local
# encoder runs beside the critical path in both models: PCN 47.93-48.03 -> 48.09-48.33 ms, PointSea 30.49 ->
# 30.53 ms (profiles/r6_skinny_ab.txt) -- no step gain, so the GEMM library path stays the default
_SKINNY = os.environ.get("PCOPS_SKINNY", "0") == "1"


def linear_skinny(x, w, b=None):
    """_SkinnyLinear when x / w fit it (bf16 autocast, CUDA, K in {6, 32, 64}, N in {32, 64}), else None."""
    if not (_SKINNY and x.is_cuda and _want_bf16() and x.shape[-1] in (6, 32, 64) and w.shape[0] in (32, 64)
            and w.dim() == 2 and w.shape[1] == x.shape[-1] and x.dtype == torch.bfloat16
            and x.data_ptr() % (16 if x.shape[-1] % 8 == 0 else 8) == 0):
        return None
    return _SkinnyLinear.apply(x, w, b, _bdt(b))


_PRESUM = "_pcops_bias_colsum"   # attribute a gradient tensor carries when its column sum is known


def _sum_dtype(t):
    """The dtype the fused bias sum of t's gradient is stored in: the bias dtype of the _Linear that
    produced t (its backward then takes the sum without a cast launch), fp32 otherwise."""
    fn = t.grad_fn if t is not None else None
    bdt = getattr(fn, "b_dtype", None) if fn is not None and type(fn).__name__ == "_LinearBackward" else None
    return bdt if bdt in (torch.float32, torch.bfloat16) and _SUM_IN_BIAS_DTYPE else torch.float32


def _attach_sum(g, dsum):
    """Hand the column sum of gradient `g` (computed by the launch that wrote g)
    to the _Linear backward that consumes g, as (sum, producing stream)."""
    setattr(g, _PRESUM, (dsum, torch.cuda.current_stream(g.device)))


def _take_sum(g):
    """The column sum attached to `g`, made safe on the consuming stream, or None.

    The sum reaches the consumer outside autograd, so autograd's cross-stream
    ordering and allocator bookkeeping do not cover it: the consumer waits for
    the producing stream when it differs (it is the same stream in every path
    the blocks issue today), records the sum on its own stream so the
    allocator keeps the block until the consumer's kernels have run, and
    detaches it from g (taken exactly once)."""
    ent = getattr(g, _PRESUM, None)
    if ent is None:
        return None
    delattr(g, _PRESUM)
    dsum, producer = ent
    cur = torch.cuda.current_stream(g.device)
    if producer != cur:
        _lib.guarded_wait(cur, producer)
    dsum.record_stream(cur)
    return dsum


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def _row_strided(g):
    """g (rows, C) has unit column stride and rows ld >= C elements apart (ld % 8 == 0,
    16-byte aligned): a channel slice of a wider gradient, usable in place."""
    return (g.dim() == 2 and g.stride(1) == 1 and g.stride(0) >= g.shape[1] and g.stride(0) % 8 == 0
            and g.data_ptr() % 16 == 0)


def colsum(g, out_dtype=None):
    """g.sum(0) of a (rows, C) CUDA tensor (g's dtype unless out_dtype): pcops_colsum (fp32
    accumulation, deterministic order) when C % 8 == 0 or a row fold makes it so, torch's
    reduction otherwise.  Rows evenly strided (a channel slice of a wider gradient) are
    summed in place (pcops_colsum_ld)."""
    rows, C = g.shape
    if (not g.is_contiguous() and C % 8 == 0 and g.dtype in _DT and _row_strided(g) and rows > 1
            and g.is_cuda):
        out = torch.empty(C, dtype=g.dtype if out_dtype is None else out_dtype, device=g.device)
        wsb = lib().pcops_colsum_workspace_bytes(rows, C)
        ws = _lib.Workspace.get(g.device, wsb)
        with torch.cuda.device(g.device):
            call("colsum", lib().pcops_colsum_ld, ptr(g), _dt(g), rows, C, g.stride(0), ptr(out),
                 _DT[out.dtype], ptr(ws), wsb, stream_of(g))
        return out
    if C % 8 and g.dtype in _DT and g.is_contiguous() and C < 64:
        # narrow outputs (conv_out: C = 3): torch's reduction ran on 4 blocks (~100 us);
        # fold k rows into one of k*C columns (k*C % 8 == 0), sum those in fp32, add the k groups
        import math
        k = 8 // math.gcd(C, 8)
        if rows % k == 0 and rows >= k:
            wide = colsum(g.view(rows // k, k * C), out_dtype=torch.float32)
            return wide.view(k, C).sum(0).to(g.dtype)
    if C % 8 or g.dtype not in _DT or not g.is_contiguous():
        return g.sum(0)
    out = torch.empty(C, dtype=g.dtype if out_dtype is None else out_dtype, device=g.device)
    wsb = lib().pcops_colsum_workspace_bytes(rows, C)
    ws = _lib.Workspace.get(g.device, wsb)
    with torch.cuda.device(g.device):
        call("colsum", lib().pcops_colsum, ptr(g), _dt(g), rows, C, ptr(out), _DT[out.dtype], ptr(ws), wsb,
             stream_of(g))
    return out


def linear(x, w, b=None):
    """F.linear for the blocks' Linear / 1x1-conv layers: the _Linear path when
    the weight gradient is a long-K GEMM (>= 8192 tokens), else F.linear.
    Inside a _lib.fork block (a side stream) every GEMM, forward and backward,
    goes through _lib.no_stream_k."""
    if _lib.on_side_stream() and x.is_cuda:
        if torch.is_grad_enabled() and (w.requires_grad or x.requires_grad):
            return _Linear.apply(x, w, b, _bdt(b))      # both directions without stream-K
        with _lib.no_stream_k():
            return F.linear(x, w, b)
    if not (x.is_cuda and torch.is_grad_enabled() and w.requires_grad and x.numel() // x.shape[-1] >= 8192):
        return F.linear(x, w, b)
    return _Linear.apply(x, w, b, _bdt(b))


def _bdt(b):
    return b.dtype if b is not None else None


# ------------------------------------------------------------------ attention core
def _layout(t, batch_first):
    """(sb, srow) element strides of a (B, L, W) / (L, B, W) tensor."""
    return (t.stride(0), t.stride(1)) if batch_first else (t.stride(1), t.stride(0))


class AttentionCore(Function):
    """o = softmax(scale q k^T) v per head.

    q, k and v are the column windows [off, off + E) of one to three distinct
    source tensors (meta = (heads, scale, E, batch_first, (src, off) x 3[,
    want_sum])), so packed projection outputs are read in place and their
    gradients written in place.  want_sum (one flag per source): the source is
    a biased _Linear's output, so the backward (bf16) also forms each gradient's
    column sums inside the attention passes (pcops_attention_bwd_*_colsum) and
    hands them to that Linear's bias gradient (_attach_sum)."""

    @staticmethod
    def forward(ctx, meta, *srcs):
        heads, scale, E, bf, qw, kw, vw = meta[:7]
        srcs = tuple(s.contiguous() for s in srcs)
        for s in srcs:
            if not s.is_cuda:
                raise RuntimeError("attention core: tensors must be CUDA tensors")
            if s.dtype not in _DT or s.dtype != srcs[0].dtype:
                raise RuntimeError(f"attention core: unsupported dtype {s.dtype}")
        q_t, k_t, v_t = srcs[qw[0]], srcs[kw[0]], srcs[vw[0]]
        if bf:
            B, Lq = q_t.shape[:2]
            Lk = k_t.shape[1]
        else:
            Lq, B = q_t.shape[:2]
            Lk = k_t.shape[0]
        hd = E // heads
        o = torch.empty((B, Lq, E) if bf else (Lq, B, E), dtype=q_t.dtype, device=q_t.device)
        lse = torch.empty(B * heads, Lq, dtype=torch.float32, device=q_t.device)
        (qb, qr), (kb, kr), (vb, vr), (ob, orow) = (_layout(t, bf) for t in (q_t, k_t, v_t, o))
        with torch.cuda.device(q_t.device):
            call("attention forward", lib().pcops_attention_forward, _vptr(q_t, qw[1]), _vptr(k_t, kw[1]),
                 _vptr(v_t, vw[1]), ptr(o), ptr(lse), B, heads, Lq, Lk, hd, float(scale), _DT[q_t.dtype], qb, hd, qr,
                 kb, hd, kr, vb, hd, vr, ob, hd, orow, stream_of(q_t))
        ctx.save_for_backward(*srcs, o, lse)
        ctx.meta, ctx.dims = meta[:7], (B, Lq, Lk, hd)
        ctx.want_sum = meta[7] if len(meta) > 7 else None
        return o

    @staticmethod
    def backward(ctx, do):
        *srcs, o, lse = ctx.saved_tensors
        heads, scale, E, bf, qw, kw, vw = ctx.meta
        B, Lq, Lk, hd = ctx.dims
        do = do.contiguous().to(o.dtype)
        covered = [0] * len(srcs)
        for w in (qw, kw, vw):
            covered[w[0]] += E
        grads = [torch.empty_like(s) if covered[i] == s.shape[-1] else torch.zeros_like(s)
                 for i, s in enumerate(srcs)]
        q_t, k_t, v_t = srcs[qw[0]], srcs[kw[0]], srcs[vw[0]]
        (qb, qr), (kb, kr), (vb, vr), (ob, orow) = (_layout(t, bf) for t in (q_t, k_t, v_t, o))
        st = (qb, hd, qr, kb, hd, kr, vb, hd, vr, ob, hd, orow)
        dt = _DT[o.dtype]
        qp, kp, vp = _vptr(q_t, qw[1]), _vptr(k_t, kw[1]), _vptr(v_t, vw[1])
        want = ctx.want_sum
        sum_ok = (want is not None and any(want) and _ATTN_COLSUM and o.dtype == torch.bfloat16
                  and all(covered[i] == s.shape[-1] for i, s in enumerate(srcs)))
        if o.dtype == torch.bfloat16 and hd >= 96 and _ATTN_FUSED:
            # one call: delta, the dK/dV pass storing dS^T, dQ = dS K read back (no S / dP
            # recompute; libpcops pcops_attention_bwd_fused), the bias sums when wanted
            sums = ([torch.empty(s.shape[-1], dtype=torch.float32, device=o.device) for s in srcs]
                    if sum_ok else None)
            wsb = lib().pcops_attention_bwd_fused_workspace_bytes(B, heads, Lq, Lk, hd, dt)
            ws = _lib.Workspace.get(o.device, wsb)
            sp = ((_vptr(sums[qw[0]], qw[1]), _vptr(sums[kw[0]], kw[1]), _vptr(sums[vw[0]], vw[1]))
                  if sums else (None, None, None))
            with torch.cuda.device(o.device):
                call("attention bwd", lib().pcops_attention_bwd_fused, qp, kp, vp, ptr(o), ptr(do), ptr(lse),
                     _vptr(grads[qw[0]], qw[1]), _vptr(grads[kw[0]], kw[1]), _vptr(grads[vw[0]], vw[1]), *sp,
                     B, heads, Lq, Lk, hd, float(scale), dt, *st, ptr(ws), wsb, stream_of(o))
            if sums:
                for g, dsum, w in zip(grads, sums, want):
                    if w:
                        _attach_sum(g, dsum)
            return (None, *grads)
        if sum_ok:
            # one fp32 sum per source column, written by the passes in window order
            sums = [torch.empty(s.shape[-1], dtype=torch.float32, device=o.device) for s in srcs]
            wsb = lib().pcops_attention_bwd_colsum_workspace_bytes(B, heads, Lq, Lk, hd)
            ws = _lib.Workspace.get(o.device, wsb)
            with torch.cuda.device(o.device):
                stream = stream_of(o)
                call("attention bwd dq", lib().pcops_attention_bwd_dq_delta_colsum, qp, kp, vp, ptr(o), ptr(do),
                     ptr(lse), _vptr(grads[qw[0]], qw[1]), _vptr(sums[qw[0]], qw[1]), B, heads, Lq, Lk, hd,
                     float(scale), dt, *st, ptr(ws), wsb, stream)
                call("attention bwd dkv", lib().pcops_attention_bwd_dkv_colsum, qp, kp, vp, ptr(do), ptr(lse),
                     _vptr(grads[kw[0]], kw[1]), _vptr(grads[vw[0]], vw[1]), _vptr(sums[kw[0]], kw[1]),
                     _vptr(sums[vw[0]], vw[1]), B, heads, Lq, Lk, hd, float(scale), dt, *st, ptr(ws), wsb, stream)
            for g, dsum, w in zip(grads, sums, want):
                if w:
                    _attach_sum(g, dsum)
            return (None, *grads)
        wsb = lib().pcops_attention_bwd_workspace_bytes(B, heads, Lq, Lk, hd)
        ws = _lib.Workspace.get(o.device, wsb)
        with torch.cuda.device(o.device):
            stream = stream_of(o)
            # delta = rowsum(dO * O) is formed inside the dQ launch (bf16) and left in ws for dK/dV
            call("attention bwd dq", lib().pcops_attention_bwd_dq_delta, qp, kp, vp, ptr(o), ptr(do), ptr(lse),
                 _vptr(grads[qw[0]], qw[1]), B, heads, Lq, Lk, hd, float(scale), dt, *st, ptr(ws), wsb, stream)
            call("attention bwd dkv", lib().pcops_attention_bwd_dkv, qp, kp, vp, ptr(do), ptr(lse),
                 _vptr(grads[kw[0]], kw[1]), _vptr(grads[vw[0]], vw[1]), B, heads, Lq, Lk, hd, float(scale), dt,
                 *st, ptr(ws), wsb, stream)
        return (None, *grads)


def _windows(q, k, v):
    """Deduplicate the q/k/v sources -> (srcs, (src, 0) windows)."""
    srcs, wins = [], []
    for t in (q, k, v):
        for i, s in enumerate(srcs):
            if s is t:
                wins.append((i, 0))
                break
        else:
            srcs.append(t)
            wins.append((len(srcs) - 1, 0))
    return srcs, wins


def attention_core(q, k, v, heads, scale=None, batch_first=False):
    """softmax(q k^T * scale) v for (L, B, E) (or (B, L, E)) q / k / v."""
    E = q.shape[-1]
    if scale is None:
        scale = 1.0 / math.sqrt(E // heads)
    srcs, wins = _windows(q, k, v)
    return AttentionCore.apply((heads, scale, E, batch_first, *wins), *srcs)


class _RowSplit(Function):
    """(t[c0:c1], t[c1:c2], ...) of a parameter along dim 0, as separate outputs; the backward
    concatenates the blocks' gradients (zeros for a block that received none) into the parameter's
    gradient in one launch.  The values are exactly those of per-slice SliceBackward + accumulation
    (disjoint blocks: every element is one block's gradient)."""

    @staticmethod
    def forward(ctx, t, cuts):
        ctx.cuts = cuts
        ctx.set_materialize_grads(False)   # a block without a gradient arrives as None: one zero fill, here
        return tuple(t[a:b] for a, b in zip(cuts[:-1], cuts[1:]))

    @staticmethod
    def backward(ctx, *gs):
        ref = next((g for g in gs if g is not None), None)
        if ref is None:
            return None, None
        parts = [torch.zeros((b - a,) + tuple(ref.shape[1:]), dtype=ref.dtype, device=ref.device) if g is None else g
                 for g, a, b in zip(gs, ctx.cuts[:-1], ctx.cuts[1:])]
        return torch.cat(parts, 0), None


_ROW_SPLIT = os.environ.get("PCOPS_ROW_SPLIT", "1") != "0"   # A/B switch: packed in_proj row blocks by _RowSplit


class MultiheadAttention(nn.Module):
    """nn.MultiheadAttention(embed_dim, num_heads) subset used by the reference:
    no masks, dropout 0, returns (output, None); seq-first by default like
    torch, batch_first=True for the token-major blocks.  The projections are
    fused per distinct input (q = k = v -> one (.., 3E) GEMM; q = k -> (.., 2E)
    + (.., E); k = v -> (.., E) + (.., 2E)) and handed to the core packed."""

    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=True, batch_first=False):
        super().__init__()
        if dropout != 0.0:
            raise NotImplementedError("attention dropout is not used by the reference models (dropout=0.0)")
        if embed_dim % num_heads:
            raise ValueError("embed_dim must be divisible by num_heads")
        self.embed_dim, self.num_heads, self.batch_first = embed_dim, num_heads, batch_first
        self.head_dim = embed_dim // num_heads
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * embed_dim)) if bias else None
        self.out_proj = nn.Linear(embed_dim, embed_dim, bias=bias)
        self._reset_parameters()

    def _reset_parameters(self):  # torch.nn.MultiheadAttention._reset_parameters
        nn.init.xavier_uniform_(self.in_proj_weight)
        if self.in_proj_bias is not None:
            nn.init.constant_(self.in_proj_bias, 0.0)
            nn.init.constant_(self.out_proj.bias, 0.0)

    def _projs(self, xs, cuts):
        """The in-projections of the inputs xs by the packed weight's row blocks [cuts[i], cuts[i+1]).
        One input: the whole packed weight unsliced.  Several: the row blocks come from _RowSplit,
        whose backward assembles the weight's (and bias's) gradient in one concatenation -- a
        plain slice per block cost a SliceBackward (full-size zero fill + copy) per block and an
        accumulating add, for the weight and for the bias, every step."""
        if len(xs) == 1:
            return (linear(xs[0], self.in_proj_weight, self.in_proj_bias),)
        ws = _RowSplit.apply(self.in_proj_weight, cuts) if _ROW_SPLIT else tuple(
            self.in_proj_weight[a:b] for a, b in zip(cuts[:-1], cuts[1:]))
        if self.in_proj_bias is None:
            bs = (None,) * len(xs)
        else:
            bs = _RowSplit.apply(self.in_proj_bias, cuts) if _ROW_SPLIT else tuple(
                self.in_proj_bias[a:b] for a, b in zip(cuts[:-1], cuts[1:]))
        return tuple(linear(x, w, b) for x, w, b in zip(xs, ws, bs))

    def forward(self, query, key, value, need_weights=True):
        E, H = self.embed_dim, self.num_heads
        scale = 1.0 / math.sqrt(self.head_dim)
        if query is key and key is value:
            srcs = self._projs((query,), (0, 3 * E))
            wins = ((0, 0), (0, E), (0, 2 * E))
        elif query is key:
            srcs = self._projs((query, value), (0, 2 * E, 3 * E))
            wins = ((0, 0), (0, E), (1, 0))
        elif key is value:
            srcs = self._projs((query, key), (0, E, 3 * E))
            wins = ((0, 0), (1, 0), (1, E))
        else:
            srcs = self._projs((query, key, value), (0, E, 2 * E, 3 * E))
            wins = ((0, 0), (1, 0), (2, 0))
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else None
        if dt is not None and any(s.dtype != dt for s in srcs):
            srcs = tuple(s.to(dt) for s in srcs)
        # sources whose gradient feeds a _Linear bias gradient: summed inside the attention backward
        want = tuple(self.in_proj_bias is not None and _ATTN_COLSUM and type(s.grad_fn).__name__ == "_LinearBackward"
                     and (_FUSED_SIDE or not _lib.on_side_stream()) for s in srcs)
        o = AttentionCore.apply((H, scale, E, self.batch_first, *wins, want), *srcs)
        return linear(o, self.out_proj.weight, self.out_proj.bias), None


# ------------------------------------------------------------------ fused block glue
def _cuda_only(what, *ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError(f"{what}: tensors must be CUDA tensors")


class _TransposeAdd(Function):
    """(B, R, C) [+ (B, R, C)] -> (B, C, R) in `out_dtype`, one LDS-tiled pass."""

    @staticmethod
    def forward(ctx, a, b, out_dtype):
        _cuda_only("transpose_add", a, b)
        a = a.contiguous()
        b = None if b is None else b.contiguous()
        B, R, C = a.shape
        out = torch.empty(B, C, R, dtype=out_dtype, device=a.device)
        with torch.cuda.device(a.device):
            call("transpose_add", lib().pcops_transpose_add, ptr(a), _dt(a), ptr(b), 0 if b is None else _dt(b),
                 ptr(out), _DT[out_dtype], None, 0, B, R, C, stream_of(a))
        ctx.dtypes = (a.dtype, None if b is None else b.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        B, C, R = g.shape
        adt, bdt = ctx.dtypes
        ga = torch.empty(B, R, C, dtype=adt, device=g.device)
        gb = None if bdt is None else torch.empty(B, R, C, dtype=bdt, device=g.device)
        with torch.cuda.device(g.device):
            call("transpose_add", lib().pcops_transpose_add, ptr(g), _dt(g), None, 0, ptr(ga), _DT[adt], ptr(gb),
                 0 if gb is None else _DT[bdt], B, C, R, stream_of(g))
        return ga, gb, None


def to_tokens(x):
    """(B, C, L) -> contiguous (B, L, C), same dtype."""
    return _TransposeAdd.apply(x, None, x.dtype)


def to_channels(a, b=None, dtype=None):
    """(B, L, C) (+ b) -> contiguous (B, C, L)."""
    return _TransposeAdd.apply(a, b, dtype or a.dtype)


def _want_bf16():
    return torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16


class _LayerNorm(Function):
    """y = LayerNorm(a (+ b)) over the last dim -> (y fp32, y bf16 or None).

    sum_of (0 = a, 1 = b, None): that input is the output of a biased Linear
    (the _Linear path); the backward then also column-sums its gradient in the
    same launch and attaches the sum to the gradient it returns, which the
    Linear's backward uses as its bias gradient instead of a separate colsum."""

    @staticmethod
    def forward(ctx, a, b, weight, bias, eps, want16, sum_of=None):
        _cuda_only("layer_norm", a, b)
        a = a.contiguous()
        b = None if b is None else b.contiguous()
        C = a.shape[-1]
        rows = a.numel() // C
        y32 = torch.empty(a.shape, dtype=torch.float32, device=a.device)
        y16 = torch.empty(a.shape, dtype=torch.bfloat16, device=a.device) if want16 else None
        mean = torch.empty(rows, dtype=torch.float32, device=a.device)
        rstd = torch.empty_like(mean)
        w, bb = weight.float().contiguous(), bias.float().contiguous()
        with torch.cuda.device(a.device):
            call("layernorm_fwd", lib().pcops_layernorm_fwd, ptr(a), _dt(a), ptr(b), 0 if b is None else _dt(b),
                 ptr(w), ptr(bb), float(eps), rows, C, ptr(y32), ptr(y16), ptr(mean), ptr(rstd), stream_of(a))
        ctx.save_for_backward(a, b, w, mean, rstd)
        ctx.wdt = weight.dtype
        ctx.sum_of = sum_of
        ctx.sum_dt = _sum_dtype((a, b)[sum_of]) if sum_of is not None else torch.float32
        if y16 is None:
            return y32
        return y32, y16

    @staticmethod
    def backward(ctx, g32, g16=None):
        a, b, w, mean, rstd = ctx.saved_tensors
        C = a.shape[-1]
        rows = a.numel() // C
        ga16 = _take_g16(g32)   # y32's gradient as the bf16 block sum handed it down (_AddToBf16)
        gx = _take_gx(ctx)      # y32's second gradient, bf16: the SDG query's positional add (_AddPosBf16)
        g16 = None if g16 is None else g16.contiguous().to(torch.bfloat16)
        if ga16 is not None and (g16 is None or gx is not None):
            ga16, g32 = None, ga16.float()
        if gx is not None and g32 is None:
            gx, g32 = None, gx.float()
        g32 = None if (g32 is None or ga16 is not None) else g32.contiguous().float()
        ld = _rows_ld(ga16) if ga16 is not None else C
        if ld is None:
            ga16, ld = ga16.contiguous(), C
        dtypes = {a.dtype} | ({b.dtype} if b is not None else set())
        dx32 = torch.empty(a.shape, dtype=torch.float32, device=a.device) if torch.float32 in dtypes else None
        dx16 = torch.empty(a.shape, dtype=torch.bfloat16, device=a.device) if torch.bfloat16 in dtypes else None
        dw = torch.empty(C, dtype=torch.float32, device=a.device)
        db = torch.empty_like(dw)
        src = None if ctx.sum_of is None else (a, b)[ctx.sum_of]
        need = (ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        sflag = 2 if ctx.sum_dt == torch.bfloat16 else 0   # dsum_src bit 1: the sum stored bf16
        if ga16 is not None or gx is not None:
            # ga16: both upstream gradients bf16, widened inside the launch (its rows ld apart: a
            # channel slice of the concatenation's gradient, _AddToBf16Cat); gx: added to g32 first
            dy, dyt = (ga16, 1) if ga16 is not None else (g32, 0)
            dsum = (torch.empty(C, dtype=ctx.sum_dt, device=a.device) if (src is not None and need[ctx.sum_of])
                    else None)
            wsb = (lib().pcops_layernorm_bwd_colsum_workspace_bytes(rows, C) if dsum is not None
                   else lib().pcops_layernorm_bwd_workspace_bytes(rows, C))
            ws = _lib.Workspace.get(a.device, wsb)
            with torch.cuda.device(a.device):
                call("layernorm_bwd", lib().pcops_layernorm_bwd_ex, ptr(dy), dyt, ld, ptr(gx), ptr(g16), ptr(a),
                     _dt(a), ptr(b), 0 if b is None else _dt(b), ptr(w), ptr(mean), ptr(rstd), rows, C, ptr(dx32),
                     ptr(dx16), ptr(dw), ptr(db), ptr(dsum), (_DT[src.dtype] | sflag) if dsum is not None else 0,
                     ptr(ws), wsb, stream_of(a))
        elif src is not None and need[ctx.sum_of]:
            dsum = torch.empty(C, dtype=ctx.sum_dt, device=a.device)
            wsb = lib().pcops_layernorm_bwd_colsum_workspace_bytes(rows, C)
            ws = _lib.Workspace.get(a.device, wsb)
            with torch.cuda.device(a.device):
                call("layernorm_bwd", lib().pcops_layernorm_bwd_colsum, ptr(g32), ptr(g16), ptr(a), _dt(a), ptr(b),
                     0 if b is None else _dt(b), ptr(w), ptr(mean), ptr(rstd), rows, C, ptr(dx32), ptr(dx16),
                     ptr(dw), ptr(db), ptr(dsum), _DT[src.dtype] | sflag, ptr(ws), wsb, stream_of(a))
        else:
            dsum = None
            wsb = lib().pcops_layernorm_bwd_workspace_bytes(rows, C)
            ws = _lib.Workspace.get(a.device, wsb)
            with torch.cuda.device(a.device):
                call("layernorm_bwd", lib().pcops_layernorm_bwd, ptr(g32), ptr(g16), ptr(a), _dt(a), ptr(b),
                     0 if b is None else _dt(b), ptr(w), ptr(mean), ptr(rstd), rows, C, ptr(dx32), ptr(dx16),
                     ptr(dw), ptr(db), ptr(ws), wsb, stream_of(a))
        pick = {torch.float32: dx32, torch.bfloat16: dx16}
        ga = pick[a.dtype]
        gb = None if b is None else pick[b.dtype]
        if dsum is not None:
            # a and b may share one gradient tensor: the sum goes on a view
            # of its own, so only the summed input's producer sees it
            g = ga.view_as(ga) if ctx.sum_of == 0 else gb.view_as(gb)
            _attach_sum(g, dsum)
            if ctx.sum_of == 0:
                ga = g
            else:
                gb = g
        return ga, gb, dw.to(ctx.wdt), db.to(ctx.wdt), None, None, None


def layer_norm(norm, a, b=None, sum_of=None):
    """norm(a (+ b)) -> (fp32 output, GEMM operand: its bf16 copy under autocast).
    sum_of: see _LayerNorm (only taken when that input came from _Linear)."""
    if sum_of is not None and not _from_linear((a, b)[sum_of]):
        sum_of = None
    if _want_bf16():
        return _LayerNorm.apply(a, b, norm.weight, norm.bias, norm.eps, True, sum_of)
    y = _LayerNorm.apply(a, b, norm.weight, norm.bias, norm.eps, False, sum_of)
    return y, y


def _from_linear(t):
    """t is the output of a biased _Linear whose bias needs a gradient, issued
    on the main stream.  Inside side-stream blocks the separate colsum stays
    (PCOPS_FUSED_SIDE=1 lifts that for A/B runs): the fused sums were measured
    as a main-stream optimisation only."""
    fn = t.grad_fn if t is not None else None
    return (fn is not None and type(fn).__name__ == "_LinearBackward" and _FUSED_BIAS_SUM
            and (_FUSED_SIDE or not _lib.on_side_stream()))


class _Gelu(Function):
    """Exact (erf) GELU whose backward is pcops_gelu_bwd_colsum: with the input
    the output of a biased _Linear, the same launch column-sums du and hands
    the sum to that Linear's backward (its bias gradient), like _LayerNorm."""

    @staticmethod
    def forward(ctx, u, want_sum):
        ctx.save_for_backward(u)
        ctx.want_sum = want_sum
        ctx.sum_dt = _sum_dtype(u) if want_sum else torch.float32
        return F.gelu(u)   # torch's vectorised kernel runs this 1:1 stream at ~4.1 TB/s; a libpcops
        # kernel (4 x 8 elements in flight per thread) measured the same step time (r4 A/B)

    @staticmethod
    def backward(ctx, g):
        (u,) = ctx.saved_tensors
        g = g.contiguous().to(u.dtype)
        C = u.shape[-1]
        rows = u.numel() // C
        du = torch.empty_like(u)
        dsum = torch.empty(C, dtype=ctx.sum_dt, device=u.device) if ctx.want_sum else None
        wsb = lib().pcops_colsum_workspace_bytes(rows, C) if ctx.want_sum else 0
        ws = _lib.Workspace.get(u.device, wsb) if ctx.want_sum else None
        with torch.cuda.device(u.device):
            call("gelu_bwd", lib().pcops_gelu_bwd_colsum, ptr(g), ptr(u), _dt(u), rows, C, ptr(du), ptr(dsum),
                 _DT[ctx.sum_dt], ptr(ws), wsb, stream_of(u))
        if dsum is not None:
            _attach_sum(du, dsum)
        return du, None


def gelu(act, u):
    """act(u) for the blocks' nn.GELU(): the fused-backward _Gelu on CUDA."""
    if (_PCOPS_GELU and u.is_cuda and isinstance(act, nn.GELU) and act.approximate == "none" and u.dtype in _DT
            and u.shape[-1] % 8 == 0 and u.is_contiguous() and torch.is_grad_enabled() and u.requires_grad):
        return _Gelu.apply(u, _GELU_SUM and _from_linear(u))
    return act(u)


def _conv1x1_tokens(conv, x_tok):
    """Conv1d(k=1) applied to token-major (B, L, C_in) input as a GEMM."""
    return linear(x_tok, conv.weight.view(conv.weight.shape[0], -1), conv.bias)


class _BlockBase(nn.Module):
    """Shared body of self_attention / cross_attention / self_attention_woinp."""

    def __init__(self, d_model, d_model_out, nhead, dim_feedforward, dropout, input_proj=True):
        super().__init__()
        self.multihead_attn = MultiheadAttention(d_model_out, nhead, dropout=dropout, batch_first=True)
        self.linear11 = nn.Linear(d_model_out, dim_feedforward)
        self.dropout1 = nn.Dropout(dropout)
        self.linear12 = nn.Linear(dim_feedforward, d_model_out)
        self.norm12 = nn.LayerNorm(d_model_out)
        self.norm13 = nn.LayerNorm(d_model_out)
        self.dropout12 = nn.Dropout(dropout)
        self.dropout13 = nn.Dropout(dropout)
        self.activation1 = torch.nn.GELU()
        if input_proj:
            self.input_proj = nn.Conv1d(d_model, d_model_out, kernel_size=1)
        if dropout != 0.0:
            raise NotImplementedError("dropout is 0 in every reference configuration")

    @staticmethod
    def with_pos_embed(tensor, pos):
        return tensor if pos is None else tensor + pos

    def _tail(self, s1, attn):
        """norm12(s1 + attn) -> FFN -> (residual stream fp32, FFN output)."""
        s2, s2h = layer_norm(self.norm12, s1, attn, sum_of=1)   # attn = out_proj(...)
        h = gelu(self.activation1, linear(s2h, self.linear11.weight, self.linear11.bias))
        f = linear(h, self.linear12.weight, self.linear12.bias)
        return s2, f

    def _in(self, x_tok):
        if isinstance(x_tok, tuple):
            # (s, f): the previous block's residual stream and FFN output, whose sum is only this
            # block's LayerNorm input (no input_proj) -- LN(s + f) in one launch, and f's Linear
            # gets its bias gradient from the LayerNorm backward
            assert not hasattr(self, "input_proj")
            return layer_norm(self.norm13, x_tok[0], x_tok[1], sum_of=1)
        y = _conv1x1_tokens(self.input_proj, x_tok) if hasattr(self, "input_proj") else x_tok
        return layer_norm(self.norm13, y, sum_of=0 if hasattr(self, "input_proj") else None)


# The bf16 gradient of a LayerNorm's fp32 output, handed from _AddToBf16.backward to
# _LayerNorm.backward without the widening pass autograd would otherwise run (2 GB of
# casts per PCN step).  Autograd insists on an fp32 gradient for the fp32 output, so
# the hand-off returns a stride-0 view of a NaN scalar carrying the bf16 tensor; the
# LayerNorm backward reads the bf16 tensor.  Only taken when the sum is the LayerNorm
# output's only consumer (the blocks' residual stream s2); if autograd ever had to add
# another gradient to it, the NaN poisons the sum loudly instead of dropping a term.
_LN_G16 = os.environ.get("PCOPS_LN_G16", "1") != "0"   # A/B switch
_NAN_SCALAR = {}


def _g16_handoff(g, shape):
    dev = g.device
    nan = _NAN_SCALAR.get(dev)
    if nan is None:
        nan = _NAN_SCALAR[dev] = torch.full((), float("nan"), dtype=torch.float32, device=dev)
    fake = nan.expand(shape)
    # a channel slice of the concatenation's gradient (_AddToBf16Cat) is read in place
    fake._pcops_g16 = g if (_LN_G16_LD and g.dtype == torch.bfloat16 and _rows_ld(g) is not None) else g.contiguous()
    return fake


def _take_g16(g):
    if g is None:
        return None
    h = getattr(g, "_pcops_g16", None)
    if h is not None:
        del g._pcops_g16
    return h


def _rows_ld(t):
    """Row stride (elements) of t viewed as (rows, C) with unit column stride and rows evenly
    spaced -- a channel slice of a wider tensor -- or None."""
    if t.stride(-1) != 1 or t.data_ptr() % 16:
        return None
    if t.dim() < 2:
        return t.shape[-1]
    ld = t.stride(-2)
    span = ld
    for d in range(t.dim() - 2, -1, -1):
        if t.shape[d] > 1 and t.stride(d) != span:
            return None
        span *= t.shape[d]
    return ld if (ld >= t.shape[-1] and ld % 8 == 0) else None


def _take_gx(ctx):
    """The bf16 gradient an _AddPosBf16 consumer of this LayerNorm's fp32 output left in the
    node's mailbox (taken once, made safe on the consuming stream like _take_sum), or None."""
    box = getattr(ctx, "gx_box", None)
    if not box:
        return None
    g, producer = box.pop()
    cur = torch.cuda.current_stream(g.device)
    if producer != cur:
        _lib.guarded_wait(cur, producer)
    g.record_stream(cur)
    return g


class _AddToBf16(Function):
    """bf16(a + b) in one kernel for a block output that only feeds GEMMs:
    the same value autocast would produce from the fp32 sum (one rounding),
    without materialising the fp32 sum; backward casts the bf16 gradient once
    (a's dtype) instead of widening it and narrowing it again -- or, when a is a
    LayerNorm's fp32 output read by nothing else (single_use), hands the bf16
    gradient to that LayerNorm's backward uncast (_g16_handoff)."""

    @staticmethod
    def forward(ctx, a, b, single_use=False):
        out = torch.empty(a.shape, dtype=torch.bfloat16, device=a.device)
        if _PCOPS_ADD and a.shape == b.shape and a.dtype in _DT and b.dtype in _DT:
            a, b = a.contiguous(), b.contiguous()
            with torch.cuda.device(a.device):
                call("add", lib().pcops_add, ptr(a), _dt(a), ptr(b), _dt(b), ptr(out), 1, a.numel(), stream_of(a))
        else:   # broadcasting (never in the models): torch's add
            torch.add(a, b, out=out)
        ctx.dts = (a.dtype, b.dtype)
        fn = a.grad_fn
        ctx.handoff = (single_use and _LN_G16 and a.dtype == torch.float32 and fn is not None
                       and type(fn).__name__ == "_LayerNormBackward" and a.output_nr == 0)
        ctx.shape = a.shape
        return out

    @staticmethod
    def backward(ctx, g):
        gb = g.to(ctx.dts[1])
        if ctx.handoff and g.dtype == torch.bfloat16:
            return _g16_handoff(g, ctx.shape), gb, None
        ga = g.to(ctx.dts[0])
        return ga, (ga if ctx.dts[1] == ctx.dts[0] else gb), None


class _AddToBf16Cat(Function):
    """torch.cat([bf16(s1 + f1), bf16(s2 + f2)], -1) written in place: each pair's sum stored by
    pcops_add_rows into its channel half (the refinement stage's two decoder outputs feeding conv_ps,
    SVDFormer.py:86) -- the values _AddToBf16 + cat produce, without the concatenation's copy.
    Backward hands each pair its channel slice of the gradient in place: the Linear producing f
    reads it with a leading dimension, the LayerNorm producing s (its only reader) through the
    strided bf16 hand-off (_g16_handoff; pcops_layernorm_bwd_ex), where the slice was copied
    contiguous before."""

    @staticmethod
    def forward(ctx, s1, f1, s2, f2):
        C1, C2 = s1.shape[-1], s2.shape[-1]
        out = torch.empty(s1.shape[:-1] + (C1 + C2,), dtype=torch.bfloat16, device=s1.device)
        rows = out.numel() // (C1 + C2)
        ctx.meta = []
        off = 0
        for a, b in ((s1, f1), (s2, f2)):
            C = a.shape[-1]
            a, b = a.contiguous(), b.contiguous()
            with torch.cuda.device(a.device):
                call("add_rows", lib().pcops_add_rows, ptr(a), _dt(a), ptr(b), _dt(b),
                     out.data_ptr() + off * 2, 1, rows, C, C1 + C2, stream_of(a))
            fn = a.grad_fn
            handoff = (_LN_G16 and a.dtype == torch.float32 and fn is not None
                       and type(fn).__name__ == "_LayerNormBackward" and a.output_nr == 0)
            ctx.meta.append((off, C, a.dtype, b.dtype, handoff, a.shape))
            off += C
        return out

    @staticmethod
    def backward(ctx, g):
        g = g if g.is_contiguous() else g.contiguous()
        grads = []
        for off, C, adt, bdt, handoff, shape in ctx.meta:
            gh = g[..., off:off + C]
            gb = gh.to(bdt)
            if handoff and g.dtype == torch.bfloat16:
                ga = _g16_handoff(gh, shape)
            else:
                ga = gh.to(adt)
                if adt == bdt:
                    gb = ga
            grads += [ga, gb]
        return tuple(grads)


def block_sum_cat(p1, p2):
    """torch.cat([block_sum(*p1, True), block_sum(*p2, True)], -1) for two (s, f) pairs of block
    outputs read only by the GEMM the concatenation feeds (each s a block tail's LayerNorm output
    nothing else reads): one bf16 buffer written in place under bf16 autocast."""
    (s1, f1), (s2, f2) = p1, p2
    if (_CAT_ROWS and _BLOCK_SUM16 and _PCOPS_ADD and _want_bf16() and s1.is_cuda
            and s1.shape == f1.shape and s2.shape == f2.shape and s1.shape[:-1] == s2.shape[:-1]
            and s1.shape[-1] % 8 == 0 and s2.shape[-1] % 8 == 0
            and all(t.dtype in _DT for t in (s1, f1, s2, f2))):
        return _AddToBf16Cat.apply(s1, f1, s2, f2)
    a, b = block_sum(s1, f1, True), block_sum(s2, f2, True)
    return torch.cat([a, b.to(a.dtype)], dim=-1)


class PosEmbedding:
    """SDG's positional term, kept lazy: SinusoidalPositionalEmbedding(cd) (models/model_utils.py:
    883-917) read through the reference's raw .reshape(B, hidden, N).permute (SVDFormer.py:77-80),
    token-major (B, N, hidden).  Its only consumer is `with_pos_embed(src1, pos)` feeding the q / k
    projection; block_sum adds it there in one kernel (pcops_add_posemb) instead of materialising
    sin, cos, the interleave and the transposed copy.  `tensor()` is the plain torch expression."""

    def __init__(self, cd, embedding, hidden):
        self.cd = cd.float().contiguous()            # (B, N) half Chamfer distances / sigma
        self.embedding, self.hidden = embedding, hidden

    def tensor(self):
        B, N = self.cd.shape
        return self.embedding(self.cd).reshape(B, self.hidden, N).transpose(1, 2)


class _AddPosBf16(Function):
    """bf16(s + pos) with pos = PosEmbedding computed in the kernel (no gradient: the reference
    .detach()es the embedding); backward: the gradient of s, cast once like _AddToBf16."""

    @staticmethod
    def forward(ctx, s, cd, div):
        B, N, H = s.shape
        s = s.contiguous()
        out = torch.empty(s.shape, dtype=torch.bfloat16, device=s.device)
        with torch.cuda.device(s.device):
            call("add_posemb", lib().pcops_add_posemb, ptr(s), _dt(s), ptr(cd), ptr(div), B, N, H, ptr(out), 1,
                 stream_of(s))
        ctx.sdt = s.dtype
        # s is a LayerNorm's fp32 output that the block also reads elsewhere (the residual into
        # norm12): instead of widening this gradient and letting autograd add it to the other one,
        # hand it to that LayerNorm's backward, which adds it in the same order inside its launch
        fn = s.grad_fn
        ctx.box = None
        if (_POS_GX and s.dtype == torch.float32 and fn is not None and type(fn).__name__ == "_LayerNormBackward"
                and s.output_nr == 0 and getattr(fn, "gx_box", None) is None):
            ctx.box = fn.gx_box = []
        return out

    @staticmethod
    def backward(ctx, g):
        if ctx.box is not None and g.dtype == torch.bfloat16 and g.is_contiguous() and not ctx.box:
            ctx.box.append((g, torch.cuda.current_stream(g.device)))
            return None, None, None
        return g.to(ctx.sdt), None, None


class _Blend(Function):
    """PointSea's path selection score * a + (1 - score) * b (models_PointSea/PointSea.py:128-131) in one
    launch each way (pcops_blend_fwd / _bwd), with torch's roundings: the same values and gradients as
    the four-op expression (score bf16 under autocast, a / b the fp32 residual streams)."""

    @staticmethod
    def forward(ctx, score, a, b, out_dtype):
        out = torch.empty(a.shape, dtype=out_dtype, device=a.device)
        with torch.cuda.device(a.device):
            call("blend", lib().pcops_blend_fwd, ptr(score), _dt(score), ptr(a), ptr(b), a.numel(), ptr(out),
                 _DT[out_dtype], stream_of(a))
        ctx.save_for_backward(score, a, b)
        return out

    @staticmethod
    def backward(ctx, g):
        score, a, b = ctx.saved_tensors
        g = g.contiguous()
        if g.dtype not in _DT:
            g = g.float()
        ds = torch.empty_like(score) if ctx.needs_input_grad[0] else None
        da = torch.empty_like(a) if ctx.needs_input_grad[1] else None
        db = torch.empty_like(b) if ctx.needs_input_grad[2] else None
        with torch.cuda.device(g.device):
            call("blend_bwd", lib().pcops_blend_bwd, ptr(g), _dt(g), ptr(score), _dt(score), ptr(a), ptr(b),
                 g.numel(), ptr(da), ptr(db), ptr(ds), stream_of(g))
        return ds, da, db, None


def blend(score, a, b, gemm_only=False):
    """score * a + (1 - score) * b (PointSea's SDG path selection).  gemm_only: the result feeds only a
    GEMM, so under bf16 autocast it is produced as the bf16 operand the cast would make (its gradient
    arrives as the GEMM's bf16 input gradient, the value the widening cast would have carried)."""
    if (_PCOPS_BLEND and score.is_cuda and a.dtype == torch.float32 and b.dtype == torch.float32
            and score.dtype in _DT and score.shape == a.shape == b.shape and a.numel() % 8 == 0):
        odt = torch.bfloat16 if (gemm_only and _want_bf16()) else torch.float32
        return _Blend.apply(score.contiguous(), a.contiguous(), b.contiguous(), odt)
    return score * a + (1 - score) * b


def block_sum(s, f, single_use=False):
    """s + f of a block's (residual, FFN) outputs whose consumers are GEMMs
    (input_proj / conv_ps): bf16 directly under bf16 autocast, else s + f.
    f may be a PosEmbedding (the SDG query's positional term).  single_use: s is
    a block tail's LayerNorm output that nothing else reads (see _AddToBf16)."""
    if isinstance(f, PosEmbedding):
        if (_PCOPS_POSEMB and _want_bf16() and s.is_cuda and s.dim() == 3 and s.shape[-1] % 8 == 0
                and s.dtype in _DT):
            div = f.embedding.div_term.float().contiguous()
            return _AddPosBf16.apply(s, f.cd, div)
        f = f.tensor()
    if _BLOCK_SUM16 and _want_bf16() and s.is_cuda:
        return _AddToBf16.apply(s, f, single_use)
    return s + f


_BLOCK_SUM16 = os.environ.get("PCOPS_BLOCKSUM16", "1") != "0"   # A/B switch
_PCOPS_POSEMB = os.environ.get("PCOPS_POSEMB", "1") != "0"          # A/B switch: fused add + positional embedding
_POS_GX = os.environ.get("PCOPS_POS_GX", "1") != "0"   # A/B switch: positional add's gradient summed in the LN backward
_CAT_ROWS = os.environ.get("PCOPS_CAT_ROWS", "1") != "0"   # A/B switch: decoder outputs written into their concatenation
_LN_G16_LD = os.environ.get("PCOPS_LN_G16_LD", "1") != "0"   # A/B switch: strided bf16 hand-off read in place
_FUSED_BIAS_SUM = os.environ.get("PCOPS_LN_BIASSUM", "1") != "0"   # A/B switch: LayerNorm-fused bias column sums
_PCOPS_ADD = os.environ.get("PCOPS_ADD", "1") != "0"                 # A/B switch: pcops_add for the block sums
_WGRAD_SPLITK = os.environ.get("PCOPS_WGRAD_SPLITK", "1") != "0"     # A/B switch: split-K weight gradients
_WGRAD_SMALL = os.environ.get("PCOPS_WGRAD_SMALL", "1") != "0"    # A/B switch: more split-K slices for small weights
_WGRAD_SMALL_LOG2 = int(os.environ.get("PCOPS_WGRAD_SMALL_LOG2", "20"))  # partial elements aimed at (log2)
_WGRAD_MINK = int(os.environ.get("PCOPS_WGRAD_MINK", "2048"))   # tokens per split-K slice at least (S <= 16)
# PCOPS_SUM_BIAS_DTYPE=0: fused bias sums stay fp32 and the Linear backward casts them (A/B runs)
_SUM_IN_BIAS_DTYPE = os.environ.get("PCOPS_SUM_BIAS_DTYPE", "1") != "0"
_PCOPS_GELU = os.environ.get("PCOPS_GELU", "1") != "0"               # A/B switch: fused-backward GELU
_FUSED_SIDE = os.environ.get("PCOPS_FUSED_SIDE", "0") == "1"          # diagnostic: fused sums in side-stream blocks too
# linear11's bias sum inside the GELU backward (A/B switch); the sum reaches the
# Linear's backward through _attach_sum / _take_sum (stream-safe hand-off)
_GELU_SUM = os.environ.get("PCOPS_GELU_SUM", "1") == "1"
_PCOPS_BLEND = os.environ.get("PCOPS_BLEND", "1") != "0"   # A/B switch: PointSea path selection in one launch
# in_proj bias sums inside the attention backward passes (A/B switch)
# the in-pass bias sums exist only in the v2/v3 bf16 kernels: the PCOPS_ATTN_V1 A/B
# switch (libpcops returns UNSUPPORTED for *_colsum there) takes the plain passes
# bf16, head_dim >= 96: the one-call backward with dQ read back from the dS the dK/dV pass
# stores (opt-in, PCOPS_ATTN_FUSED=1): measured no faster than recomputing S / dP -- at
# 2048^2 hd 128 the dS^T stores add 0.38 ms to the dK/dV pass and the dQ read-back takes
# 0.57 ms, against the 0.91 ms dQ pass it replaces (profiles/r4_attn_ds_ab.txt)
_ATTN_FUSED = os.environ.get("PCOPS_ATTN_FUSED", "0") == "1"
_ATTN_COLSUM = (os.environ.get("PCOPS_ATTN_COLSUM", "1") != "0"
                and os.environ.get("PCOPS_ATTN_V1", "0") != "1")
_DEBUG_CONTIG = os.environ.get("PCOPS_DEBUG_CONTIG", "0") == "1"   # diagnostic: report _Linear operand copies
_STRIDED_G = os.environ.get("PCOPS_STRIDED_G", "1") != "0"           # A/B switch: row-strided output gradients in place


def _pos_tokens(pos):
    # the reference passes pos seq-first (L, B, C)
    return None if pos is None else pos.transpose(0, 1)


class self_attention(_BlockBase):
    """models/model_utils.py:584-617."""

    def __init__(self, d_model=256, d_model_out=256, nhead=4, dim_feedforward=1024, dropout=0.0):
        super().__init__(d_model, d_model_out, nhead, dim_feedforward, dropout)

    def forward_tokens(self, x_tok, pos=None):
        """(B, L, C_in) -> (s2, f) with the block output = s2 + f (B, L, C_out)."""
        s1, s1h = self._in(x_tok)
        if pos is None:
            attn = self.multihead_attn(s1h, s1h, s1h)[0]
        else:
            q = block_sum(s1, pos)   # only the q/k projection GEMM reads it
            attn = self.multihead_attn(q, q, s1h)[0]
        return self._tail(s1, attn)

    def forward(self, src1, pos=None):
        s2, f = self.forward_tokens(to_tokens(src1), _pos_tokens(pos))
        return to_channels(s2, f, s2.dtype)


class cross_attention(_BlockBase):
    """models/model_utils.py:542-582 (PointSea copy :385-426 is identical)."""

    def __init__(self, d_model=256, d_model_out=256, nhead=4, dim_feedforward=1024, dropout=0.0):
        super().__init__(d_model, d_model_out, nhead, dim_feedforward, dropout)

    def forward_tokens(self, x1_tok, x2_tok, pos=None):
        s1, s1h = self._in(x1_tok)
        _, s2h = self._in(x2_tok)
        # the query only feeds its projection GEMM: the LN's bf16 copy is
        # exactly what autocast would cast s1 to
        q = s1h if pos is None else block_sum(s1, pos)
        attn = self.multihead_attn(q, s2h, s2h)[0]
        return self._tail(s1, attn)

    def forward(self, src1, src2, pos=None):
        s2, f = self.forward_tokens(to_tokens(src1), to_tokens(src2), _pos_tokens(pos))
        return to_channels(s2, f, s2.dtype)


class self_attention_woinp(_BlockBase):
    """models_PointSea/model_utils.py:463-494 (no input projection)."""

    def __init__(self, d_model=256, d_model_out=256, nhead=4, dim_feedforward=1024, dropout=0.0):
        super().__init__(d_model, d_model_out, nhead, dim_feedforward, dropout, input_proj=False)

    forward_tokens = self_attention.forward_tokens
    forward = self_attention.forward


class SDG_Decoder(nn.Module):
    """models/model_utils.py:619-629; the two blocks hand over token-major."""

    def __init__(self, hidden_dim, channel, ratio):
        super().__init__()
        self.sa1 = self_attention(hidden_dim, hidden_dim, dropout=0.0, nhead=8)
        self.sa2 = self_attention(hidden_dim, channel * ratio, dropout=0.0, nhead=8)

    def forward_tokens(self, x_tok):
        return block_sum(*self.forward_pair(x_tok), True)   # SDG feeds it to input_proj / conv_ps

    def forward_pair(self, x_tok):
        """The output as sa2's (residual, FFN) pair, summed by the consumer."""
        s, f = self.sa1.forward_tokens(x_tok)
        return self.sa2.forward_tokens(block_sum(s, f, True))   # sa2 starts with input_proj (a GEMM)

    def forward(self, input):
        s, f = self.sa1.forward_tokens(to_tokens(input))
        s, f = self.sa2.forward_tokens(s + f)
        return to_channels(s, f, s.dtype)


class SDG_Decoder_PointSea(nn.Module):
    """models_PointSea/model_utils.py:496-509 (SDG_Decoder of PointSea)."""

    def __init__(self, hidden_dim, channel, ratio, dropout=0.0):
        super().__init__()
        self.sa1 = self_attention_woinp(hidden_dim, hidden_dim, dropout=dropout, nhead=8)
        self.sa2 = self_attention_woinp(hidden_dim, hidden_dim, dropout=dropout, nhead=8)

    def forward_tokens(self, x_tok):
        """x_tok: (B, L, C) or an (s, f) pair whose sum is the input (see _BlockBase._in)."""
        s, f = self.sa1.forward_tokens(x_tok)
        s, f = self.sa2.forward_tokens((s, f))   # sa2 starts with its LayerNorm
        return s + f

    def forward(self, input, pos=None):  # pos is accepted and unused, as in the reference
        s, f = self.sa1.forward_tokens(to_tokens(input))
        s, f = self.sa2.forward_tokens((s, f))
        return to_channels(s, f, s.dtype)
