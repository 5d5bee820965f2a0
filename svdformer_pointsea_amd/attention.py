"""Attention blocks of models/model_utils.py (:542-629) and
models_PointSea/model_utils.py (:385-509) with the attention core
(softmax(QK^T/sqrt(hd)) V, forward and backward) on libpcops.so MFMA kernels.

Parameter names match the reference exactly (multihead_attn.in_proj_weight,
multihead_attn.out_proj.weight, linear11, linear12, norm12, norm13,
input_proj, ...) so reference state_dicts load unchanged.  The projections,
LayerNorms, GELU and residuals are the same torch ops the reference uses; only
the O(L^2) part is replaced.  The core reads the seq-first (L, B, E) projection
outputs in place (stride tricks, no transposes) and runs in fp32 (exact f32
MFMA, parity build) or bf16 (bf16 MFMA, fp32 accumulation) following the
dtype of its inputs (e.g. under torch.autocast).
"""
import math

import torch
import torch.nn.functional as F
from torch import nn
from torch.autograd import Function

from . import _lib
from ._lib import call, lib, ptr, stream_of

_DT = {torch.float32: 0, torch.bfloat16: 1}


def _strides(t, heads):
    # t: (L, B, E) contiguous seq-first -> element (bh, row, d) at bh*hd + row*B*E + d
    L, B, E = t.shape
    return E // heads, B * E


class AttentionCore(Function):
    """o = softmax(scale * q k^T) v per head; q (Lq,B,E), k/v (Lk,B,E) seq-first."""

    @staticmethod
    def forward(ctx, q, k, v, heads, scale):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        if not (q.is_cuda and k.is_cuda and v.is_cuda):
            raise RuntimeError("attention core: tensors must be CUDA tensors")
        if q.dtype not in _DT or k.dtype != q.dtype or v.dtype != q.dtype:
            raise RuntimeError(f"attention core: unsupported dtype {q.dtype}")
        Lq, B, E = q.shape
        Lk = k.shape[0]
        hd = E // heads
        o = torch.empty_like(q)
        lse = torch.empty(B * heads, Lq, dtype=torch.float32, device=q.device)
        sq, rq = _strides(q, heads)
        sk, rk = _strides(k, heads)
        with torch.cuda.device(q.device):
            call("attention forward", lib().pcops_attention_forward, ptr(q), ptr(k), ptr(v), ptr(o), ptr(lse),
                 B * heads, Lq, Lk, hd, float(scale), _DT[q.dtype], sq, rq, sk, rk, sk, rk, sq, rq, stream_of(q))
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.heads, ctx.scale = heads, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        heads, scale = ctx.heads, ctx.scale
        do = do.contiguous().to(q.dtype)
        Lq, B, E = q.shape
        Lk = k.shape[0]
        hd = E // heads
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        sq, rq = _strides(q, heads)
        sk, rk = _strides(k, heads)
        wsb = lib().pcops_attention_bwd_workspace_bytes(B * heads, Lq, Lk, hd)
        ws = _lib.Workspace.get(q.device, wsb)
        BH, dt = B * heads, _DT[q.dtype]
        st = (sq, rq, sk, rk, sk, rk, sq, rq)
        with torch.cuda.device(q.device):
            stream = stream_of(q)
            call("attention bwd delta", lib().pcops_attention_bwd_preprocess, ptr(o), ptr(do), BH, Lq, hd, dt, sq, rq,
                 ptr(ws), wsb, stream)
            call("attention bwd dq", lib().pcops_attention_bwd_dq, ptr(q), ptr(k), ptr(v), ptr(do), ptr(lse), ptr(dq),
                 BH, Lq, Lk, hd, float(scale), dt, *st, ptr(ws), wsb, stream)
            call("attention bwd dkv", lib().pcops_attention_bwd_dkv, ptr(q), ptr(k), ptr(v), ptr(do), ptr(lse), ptr(dk),
                 ptr(dv), BH, Lq, Lk, hd, float(scale), dt, *st, ptr(ws), wsb, stream)
        return dq, dk, dv, None, None


def attention_core(q, k, v, heads, scale=None):
    E = q.shape[-1]
    if scale is None:
        scale = 1.0 / math.sqrt(E // heads)
    return AttentionCore.apply(q, k, v, heads, scale)


class MultiheadAttention(nn.Module):
    """nn.MultiheadAttention(embed_dim, num_heads) subset used by the reference:
    seq-first inputs, no masks, dropout 0, returns (output, None)."""

    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=True):
        super().__init__()
        if dropout != 0.0:
            raise NotImplementedError("attention dropout is not used by the reference models (dropout=0.0)")
        if embed_dim % num_heads:
            raise ValueError("embed_dim must be divisible by num_heads")
        self.embed_dim, self.num_heads = embed_dim, num_heads
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

    def forward(self, query, key, value, need_weights=True):
        E = self.embed_dim
        w, b = self.in_proj_weight, self.in_proj_bias
        bq, bk, bv = (None, None, None) if b is None else (b[:E], b[E:2 * E], b[2 * E:])
        if query is key and key is value:
            q, k, v = F.linear(query, w, b).chunk(3, dim=-1)
        elif query is key:
            q, k = F.linear(query, w[:2 * E], None if b is None else b[:2 * E]).chunk(2, dim=-1)
            v = F.linear(value, w[2 * E:], bv)
        else:
            q = F.linear(query, w[:E], bq)
            if key is value:
                k, v = F.linear(key, w[E:], None if b is None else b[E:]).chunk(2, dim=-1)
            else:
                k = F.linear(key, w[E:2 * E], bk)
                v = F.linear(value, w[2 * E:], bv)
        o = attention_core(q, k, v, self.num_heads)
        return self.out_proj(o), None


class self_attention(nn.Module):
    """models/model_utils.py:584-617."""

    def __init__(self, d_model=256, d_model_out=256, nhead=4, dim_feedforward=1024, dropout=0.0):
        super().__init__()
        self.multihead_attn = MultiheadAttention(d_model_out, nhead, dropout=dropout)
        self.linear11 = nn.Linear(d_model_out, dim_feedforward)
        self.dropout1 = nn.Dropout(dropout)
        self.linear12 = nn.Linear(dim_feedforward, d_model_out)
        self.norm12 = nn.LayerNorm(d_model_out)
        self.norm13 = nn.LayerNorm(d_model_out)
        self.dropout12 = nn.Dropout(dropout)
        self.dropout13 = nn.Dropout(dropout)
        self.activation1 = torch.nn.GELU()
        self.input_proj = nn.Conv1d(d_model, d_model_out, kernel_size=1)

    def with_pos_embed(self, tensor, pos):
        return tensor if pos is None else tensor + pos

    def forward(self, src1, pos=None):
        src1 = self.input_proj(src1)
        b, c, _ = src1.shape
        src1 = src1.reshape(b, c, -1).permute(2, 0, 1)
        src1 = self.norm13(src1)
        q = k = self.with_pos_embed(src1, pos)
        src12 = self.multihead_attn(query=q, key=k, value=src1)[0]
        src1 = src1 + self.dropout12(src12)
        src1 = self.norm12(src1)
        src12 = self.linear12(self.dropout1(self.activation1(self.linear11(src1))))
        src1 = src1 + self.dropout13(src12)
        return src1.permute(1, 2, 0)


class cross_attention(nn.Module):
    """models/model_utils.py:542-582 (PointSea copy :385-426 is identical)."""

    def __init__(self, d_model=256, d_model_out=256, nhead=4, dim_feedforward=1024, dropout=0.0):
        super().__init__()
        self.multihead_attn = MultiheadAttention(d_model_out, nhead, dropout=dropout)
        self.linear11 = nn.Linear(d_model_out, dim_feedforward)
        self.dropout1 = nn.Dropout(dropout)
        self.linear12 = nn.Linear(dim_feedforward, d_model_out)
        self.norm12 = nn.LayerNorm(d_model_out)
        self.norm13 = nn.LayerNorm(d_model_out)
        self.dropout12 = nn.Dropout(dropout)
        self.dropout13 = nn.Dropout(dropout)
        self.activation1 = torch.nn.GELU()
        self.input_proj = nn.Conv1d(d_model, d_model_out, kernel_size=1)

    def with_pos_embed(self, tensor, pos):
        return tensor if pos is None else tensor + pos

    def forward(self, src1, src2, pos=None):
        src1 = self.input_proj(src1)
        src2 = self.input_proj(src2)
        b, c, _ = src1.shape
        src1 = src1.reshape(b, c, -1).permute(2, 0, 1)
        src2 = src2.reshape(b, c, -1).permute(2, 0, 1)
        src1 = self.norm13(src1)
        src2 = self.norm13(src2)
        q = self.with_pos_embed(src1, pos)
        src12 = self.multihead_attn(query=q, key=src2, value=src2)[0]
        src1 = src1 + self.dropout12(src12)
        src1 = self.norm12(src1)
        src12 = self.linear12(self.dropout1(self.activation1(self.linear11(src1))))
        src1 = src1 + self.dropout13(src12)
        return src1.permute(1, 2, 0)


class self_attention_woinp(nn.Module):
    """models_PointSea/model_utils.py:463-494 (no input projection)."""

    def __init__(self, d_model=256, d_model_out=256, nhead=4, dim_feedforward=1024, dropout=0.0):
        super().__init__()
        self.multihead_attn = MultiheadAttention(d_model_out, nhead, dropout=dropout)
        self.linear11 = nn.Linear(d_model_out, dim_feedforward)
        self.dropout1 = nn.Dropout(dropout)
        self.linear12 = nn.Linear(dim_feedforward, d_model_out)
        self.norm12 = nn.LayerNorm(d_model_out)
        self.norm13 = nn.LayerNorm(d_model_out)
        self.dropout12 = nn.Dropout(dropout)
        self.dropout13 = nn.Dropout(dropout)
        self.activation1 = torch.nn.GELU()

    def with_pos_embed(self, tensor, pos):
        return tensor if pos is None else tensor + pos

    def forward(self, src1, pos=None):
        b, c, _ = src1.shape
        src1 = src1.reshape(b, c, -1).permute(2, 0, 1)
        src1 = self.norm13(src1)
        q = k = self.with_pos_embed(src1, pos)
        src12 = self.multihead_attn(query=q, key=k, value=src1)[0]
        src1 = src1 + self.dropout12(src12)
        src1 = self.norm12(src1)
        src12 = self.linear12(self.dropout1(self.activation1(self.linear11(src1))))
        src1 = src1 + self.dropout13(src12)
        return src1.permute(1, 2, 0)


class SDG_Decoder(nn.Module):
    """models/model_utils.py:619-629."""

    def __init__(self, hidden_dim, channel, ratio):
        super().__init__()
        self.sa1 = self_attention(hidden_dim, hidden_dim, dropout=0.0, nhead=8)
        self.sa2 = self_attention(hidden_dim, channel * ratio, dropout=0.0, nhead=8)

    def forward(self, input):
        return self.sa2(self.sa1(input))


class SDG_Decoder_PointSea(nn.Module):
    """models_PointSea/model_utils.py:496-509 (SDG_Decoder of PointSea)."""

    def __init__(self, hidden_dim, channel, ratio, dropout=0.0):
        super().__init__()
        self.sa1 = self_attention_woinp(hidden_dim, hidden_dim, dropout=dropout, nhead=8)
        self.sa2 = self_attention_woinp(hidden_dim, hidden_dim, dropout=dropout, nhead=8)

    def forward(self, input, pos=None):
        return self.sa2(self.sa1(input))
