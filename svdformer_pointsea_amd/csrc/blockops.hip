// Memory-bound glue of the attention blocks (models/model_utils.py:542-617):
// the (B, C, L) <-> (B, L, C) layout changes around the blocks and the two
// LayerNorms (norm13, norm12 after the residual add), fused so every
// activation is read and written once per pass.
//
//   pcops_transpose_add : out[b][c][r] = a[b][r][c] (+ b[b][r][c]), LDS-tiled
//                         64x64 transpose, optional second output dtype
//   pcops_layernorm_fwd : y = LN(a (+ b)) * gamma + beta per row, fp32 and/or
//                         bf16 outputs, per-row mean / rstd saved
//   pcops_layernorm_bwd : dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),
//                         g = (dy32 + dy16) * gamma; dgamma / dbeta as per-wave
//                         partial sums in a scratch, then a column reduction
// dtype codes: 0 = fp32, 1 = bf16.  One wave per row for the LayerNorms
// (C <= 1024, C % 8 == 0: 16-B vector loads, two-pass statistics in registers).
#include <cstdlib>

#include "common.h"

namespace {

__device__ __forceinline__ float ld(const void *p, int dt, long long i) {
  return dt == 0 ? reinterpret_cast<const float *>(p)[i] : (float)reinterpret_cast<const __bf16 *>(p)[i];
}
__device__ __forceinline__ void st(void *p, int dt, long long i, float v) {
  if (dt == 0)
    reinterpret_cast<float *>(p)[i] = v;
  else
    reinterpret_cast<__bf16 *>(p)[i] = (__bf16)v;
}

// ---------------------------------------------------------------- transpose
constexpr int kT = 64;

__global__ __launch_bounds__(256) void transpose_add_kernel(const void *__restrict__ a, int adt,
                                                            const void *__restrict__ b, int bdt, void *__restrict__ out,
                                                            int odt, void *__restrict__ out2, int o2dt, int R, int C) {
  __shared__ float tile[kT][kT + 1];
  const int bb = blockIdx.z;
  const int r0 = blockIdx.y * kT, c0 = blockIdx.x * kT;
  const long long in_base = (long long)bb * R * C, out_base = (long long)bb * C * R;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
#pragma unroll 4
  for (int i = ty; i < kT; i += 4) {
    const int r = r0 + i, c = c0 + tx;
    float v = 0.f;
    if (r < R && c < C) {
      const long long e = in_base + (long long)r * C + c;
      v = ld(a, adt, e);
      if (b) v += ld(b, bdt, e);
    }
    tile[i][tx] = v;
  }
  __syncthreads();
#pragma unroll 4
  for (int i = ty; i < kT; i += 4) {
    const int c = c0 + i, r = r0 + tx;
    if (r < R && c < C) {
      const long long e = out_base + (long long)c * R + r;
      const float v = tile[tx][i];
      st(out, odt, e, v);
      if (out2) st(out2, o2dt, e, v);
    }
  }
}

// ---------------------------------------------------------------- LayerNorm
// A row is read as 8-element chunks (one 16-B load for bf16, two for fp32);
// chunk ch = lane + 64*i, so C <= 1024 needs at most 2 chunks per lane.
// The operand configuration (dtypes, residual present, which upstream
// gradients) is a template: with runtime dtype / presence tests hipcc split
// every load into its own branch and waited for each one (vmcnt(0) six times
// per row) -- the backward ran at 2.5 TB/s.  Now a row's loads issue together.
constexpr int kMaxCh = 2;

struct V8 {
  float v[8];
};

template <int DT>
__device__ __forceinline__ void ld8c(V8 &o, const void *p, long long e) {
  if constexpr (DT == 0) {
    const float4 x = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(p) + e);
    const float4 y = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(p) + e + 4);
    o.v[0] = x.x, o.v[1] = x.y, o.v[2] = x.z, o.v[3] = x.w, o.v[4] = y.x, o.v[5] = y.y, o.v[6] = y.z, o.v[7] = y.w;
  } else {
    typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
    const bf16x8_t x = *reinterpret_cast<const bf16x8_t *>(reinterpret_cast<const __bf16 *>(p) + e);
#pragma unroll
    for (int k = 0; k < 8; ++k) o.v[k] = (float)x[k];
  }
}
__device__ __forceinline__ void st8_f32(float *p, long long e, const V8 &o) {
  *reinterpret_cast<float4 *>(p + e) = make_float4(o.v[0], o.v[1], o.v[2], o.v[3]);
  *reinterpret_cast<float4 *>(p + e + 4) = make_float4(o.v[4], o.v[5], o.v[6], o.v[7]);
}
__device__ __forceinline__ void st8_bf16(__bf16 *p, long long e, const V8 &o) {
  typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
  bf16x8_t x;
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = (__bf16)o.v[k];
  *reinterpret_cast<bf16x8_t *>(p + e) = x;
}

// 8 elements as raw 16-byte vectors (fp32: two, bf16: one), converted at their use by cvt8 (the values of
// ld8c): the LayerNorm backward holds a row's bf16 operands packed, 4 registers per 8 elements, instead of 8
template <int DT>
struct Raw8;
template <>
struct Raw8<0> {
  float4 x, y;
};
template <>
struct Raw8<1> {
  uint4 x;
};
template <int DT>
__device__ __forceinline__ void ldraw(Raw8<DT> &r, const void *p, long long e) {
  if constexpr (DT == 0) {
    r.x = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(p) + e);
    r.y = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(p) + e + 4);
  } else {
    r.x = *reinterpret_cast<const uint4 *>(reinterpret_cast<const __bf16 *>(p) + e);
  }
}
template <int DT>
__device__ __forceinline__ float raw_at(const Raw8<DT> &r, int k) {
  if constexpr (DT == 0) {
    const float v[8] = {r.x.x, r.x.y, r.x.z, r.x.w, r.y.x, r.y.y, r.y.z, r.y.w};
    return v[k];
  } else {
    const unsigned w = k < 2 ? r.x.x : k < 4 ? r.x.y : k < 6 ? r.x.z : r.x.w;
    return __uint_as_float((k & 1) ? (w & 0xffff0000u) : (w << 16));   // bf16 -> fp32 is a shift
  }
}

// AT: a's dtype; BT: b's dtype or -1 (no residual)
template <int CH, int AT, int BT>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const void *__restrict__ a, const void *__restrict__ b,
                                                     const float *__restrict__ gamma,
                                                     const float *__restrict__ beta, float eps, int rows, int C,
                                                     float *__restrict__ y32, __bf16 *__restrict__ y16,
                                                     float *__restrict__ mean_out, float *__restrict__ rstd_out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int nch = C >> 3;
  const long long base = (long long)row * C;
  // every lane loads (chunk index clamped, no branches: the loads of both
  // chunks and both operands issue back to back); lanes past the row end
  // contribute zeros
  V8 x[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int ch = min(lane + 64 * i, nch - 1);
    ld8c<AT>(x[i], a, base + 8 * ch);
    if constexpr (BT >= 0) {
      V8 t;
      ld8c<BT>(t, b, base + 8 * ch);
#pragma unroll
      for (int k = 0; k < 8; ++k) x[i].v[k] += t.v[k];
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const bool ok = lane + 64 * i < nch;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += ok ? x[i].v[k] : 0.f;
  }
  const float mean = wave_sum_f32_dpp(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const bool ok = lane + 64 * i < nch;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float d = ok ? x[i].v[k] - mean : 0.f;
      q = __builtin_fmaf(d, d, q);
    }
  }
  const float rstd = 1.f / sqrtf(wave_sum_f32_dpp(q) / (float)C + eps);
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int ch = lane + 64 * i;
    if (ch < nch) {
      V8 y;
#pragma unroll
      for (int k = 0; k < 8; ++k) y.v[k] = (x[i].v[k] - mean) * rstd * gamma[8 * ch + k] + beta[8 * ch + k];
      if (y32) st8_f32(y32, base + 8 * ch, y);
      if (y16) st8_bf16(y16, base + 8 * ch, y);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Each wave owns rpw consecutive rows (one at a time, full row in registers;
// rpw = 4..16 so that large inputs get ~2048 blocks); the block's dgamma /
// dbeta partial sums are reduced through LDS (dynamic, 4 x 2C floats) and
// written once per block to a [blocks][2C] scratch (plain stores -- thousands
// of waves atomically adding into the same 2C floats serialise), then summed
// by colsum_final_kernel in a fixed order.
#ifndef PCOPS_LN_RAW
#define PCOPS_LN_RAW 1   // LayerNorm backward: bf16 operands held packed until used (A/B builds: 0)
#endif

int ln_bwd_rpw(int rows) {
  static const int forced = [] {   // PCOPS_LN_RPW: rows per wave forced (A/B runs)
    const char *e = getenv("PCOPS_LN_RPW");
    return e ? atoi(e) : 0;
  }();
  if (forced > 0) return forced;
  const int r = (rows + 8191) / 8192;
  return r < 4 ? 4 : (r > 16 ? 16 : r);
}

// CH: 8-element chunks per lane (1 for C <= 512, 2 for C <= 1024); AT / BT as
// the forward; GM: which upstream gradients are present (bit 0 = dy32, bit 1 = dy16;
// bit 2: the first one bf16 (the fp32 output's gradient as the bf16 block sum handed
// it down, widened here instead of by a separate cast pass), its rows ldg elements
// apart (a channel slice of the concatenation's gradient); bit 3: a second bf16
// gradient of the fp32 output, gx (the SDG query's positional add), added to dy32
// first -- autograd's accumulation of the two, then the sum with dy16 as before).
// Instantiated: 1, 2, 3, 5, 7, 9, 11.  CS: also the column sums of dx (the bias gradient of the Linear
// whose output is a or b) over the values as stored -- bf16-rounded when
// sum16 -- as a third C-wide partial row.
template <int CH, int AT, int BT, int GM, bool CS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CH == 1 ? 4 : 3))) void ln_bwd_kernel(
    const float *__restrict__ g32, const __bf16 *__restrict__ g16, const __bf16 *__restrict__ gx, long long ldg,
    const void *__restrict__ a, const void *__restrict__ b, const float *__restrict__ gamma,
    const float *__restrict__ mean_in, const float *__restrict__ rstd_in, int rows, int C, float *__restrict__ dx32,
    __bf16 *__restrict__ dx16, int rpw, float *__restrict__ part, bool sum16) {
  constexpr int NP = CS ? 3 : 2;     // partial rows per block: dgamma | dbeta (| dsum)
  extern __shared__ float ln_red[];  // [4][NP*C]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nch = C >> 3;
  V8 dg[CH], db[CH], gm[CH], dsm[CS ? CH : 1];
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    ld8c<0>(gm[i], gamma, 8 * min(lane + 64 * i, nch - 1));  // hoisted out of the row loop
#pragma unroll
    for (int k = 0; k < 8; ++k) dg[i].v[k] = db[i].v[k] = 0.f;
    if constexpr (CS)
#pragma unroll
      for (int k = 0; k < 8; ++k) dsm[i].v[k] = 0.f;
  }
  const int r0 = (blockIdx.x * 4 + w) * rpw;
  for (int row = r0; row < r0 + rpw && row < rows; ++row) {
    const long long base = (long long)row * C;
    const float mean = mean_in[row], rstd = rstd_in[row];
    // all loads of the row first (clamped chunk index, no branches), then the
    // arithmetic; lanes past the row end carry dy = xh = 0
    V8 xh[CH], dy[CH];
#if PCOPS_LN_RAW
    // the row's operands as loaded, bf16 ones packed (converted where used: a shift per value)
    Raw8<AT> ra[CH];
    Raw8<BT < 0 ? 1 : BT> rb[CH];
    Raw8<(GM & 4) ? 1 : 0> ru[CH];
    Raw8<1> rq[(GM & 8) ? CH : 1], rv[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c8 = 8 * min(lane + 64 * i, nch - 1);
      const long long e = base + c8;
      ldraw<AT>(ra[i], a, e);
      if constexpr (BT >= 0) ldraw<BT>(rb[i], b, e);
      if constexpr (GM & 1) ldraw<(GM & 4) ? 1 : 0>(ru[i], g32, (long long)row * ldg + c8);
      if constexpr (GM & 8) ldraw<1>(rq[i], gx, e);
      if constexpr (GM & 2) ldraw<1>(rv[i], g16, e);
    }
#else
    V8 t[CH], u[CH], v[CH], q[(GM & 8) ? CH : 1];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c8 = 8 * min(lane + 64 * i, nch - 1);
      const long long e = base + c8;
      ld8c<AT>(xh[i], a, e);
      if constexpr (BT >= 0) ld8c<BT>(t[i], b, e);
      if constexpr (GM & 1) ld8c<(GM & 4) ? 1 : 0>(u[i], g32, (long long)row * ldg + c8);
      if constexpr (GM & 8) ld8c<1>(q[i], gx, e);
      if constexpr (GM & 2) ld8c<1>(v[i], g16, e);
    }
#endif
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const bool ok = lane + 64 * i < nch;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
#if PCOPS_LN_RAW
        float x = raw_at<AT>(ra[i], k);
        if constexpr (BT >= 0) x += raw_at<BT < 0 ? 1 : BT>(rb[i], k);
        float d;
        if constexpr (GM & 1) {
          d = raw_at<(GM & 4) ? 1 : 0>(ru[i], k);
          if constexpr (GM & 8) d = d + raw_at<1>(rq[i], k);
          if constexpr (GM & 2) d = d + raw_at<1>(rv[i], k);
        } else {
          d = raw_at<1>(rv[i], k);
        }
#else
        float x = xh[i].v[k];
        if constexpr (BT >= 0) x += t[i].v[k];
        float d;
        if constexpr (GM & 1) {
          d = u[i].v[k];
          if constexpr (GM & 8) d = d + q[i].v[k];
          if constexpr (GM & 2) d = d + v[i].v[k];
        } else {
          d = v[i].v[k];
        }
#endif
        xh[i].v[k] = ok ? (x - mean) * rstd : 0.f;
        dy[i].v[k] = ok ? d : 0.f;
        dg[i].v[k] = __builtin_fmaf(dy[i].v[k], xh[i].v[k], dg[i].v[k]);
        db[i].v[k] += dy[i].v[k];
        const float g = dy[i].v[k] * gm[i].v[k];
        sg += g;
        sgx = __builtin_fmaf(g, xh[i].v[k], sgx);
      }
    }
    const float mg = wave_sum_f32_dpp(sg) / (float)C;
    const float mgx = wave_sum_f32_dpp(sgx) / (float)C;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int ch = lane + 64 * i;
      if (ch < nch) {
        V8 dx;
#pragma unroll
        for (int k = 0; k < 8; ++k) dx.v[k] = rstd * (dy[i].v[k] * gm[i].v[k] - mg - xh[i].v[k] * mgx);
        if (dx32) st8_f32(dx32, base + 8 * ch, dx);
        if (dx16) st8_bf16(dx16, base + 8 * ch, dx);
        if constexpr (CS)
#pragma unroll
          for (int k = 0; k < 8; ++k) dsm[i].v[k] += sum16 ? (float)(__bf16)dx.v[k] : dx.v[k];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int ch = lane + 64 * i;
    if (ch < nch)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        ln_red[w * NP * C + 8 * ch + k] = dg[i].v[k];
        ln_red[w * NP * C + C + 8 * ch + k] = db[i].v[k];
        if constexpr (CS) ln_red[w * NP * C + 2 * C + 8 * ch + k] = dsm[i].v[k];
      }
  }
  __syncthreads();
  float *pb = part + (long long)blockIdx.x * NP * C;
  for (int c = threadIdx.x; c < NP * C; c += 256)
    pb[c] = ((ln_red[c] + ln_red[NP * C + c]) + ln_red[2 * NP * C + c]) + ln_red[3 * NP * C + c];
}

// ---- host dispatch over the operand configurations
struct LnArgs {
  const void *a, *b;
  const float *g32;
  const __bf16 *g16;
  const __bf16 *gx;  // backward: second bf16 gradient of the fp32 output (GM bit 3)
  long long ldg;     // backward: row stride of g32 (elements)
  const float *gamma, *beta, *mean, *rstd;
  float eps;
  int rows, C;
  float *y32;
  __bf16 *y16;
  float *part;
  bool cs, sum16;  // backward: fused bias column sum, over bf16-rounded dx
  hipStream_t s;
};

template <int CH, int AT, int BT>
void ln_fwd_go(const LnArgs &p) {
  hipLaunchKernelGGL((ln_fwd_kernel<CH, AT, BT>), dim3((p.rows + 3) / 4), dim3(256), 0, p.s, p.a, p.b, p.gamma,
                     p.beta, p.eps, p.rows, p.C, p.y32, p.y16, const_cast<float *>(p.mean),
                     const_cast<float *>(p.rstd));
}

template <int CH, int AT, int BT, int GM>
void ln_bwd_go(const LnArgs &p, int blocks, int rpw) {
  if (p.cs)
    hipLaunchKernelGGL((ln_bwd_kernel<CH, AT, BT, GM, true>), dim3(blocks), dim3(256), 4 * 3 * p.C * sizeof(float),
                       p.s, p.g32, p.g16, p.gx, p.ldg, p.a, p.b, p.gamma, p.mean, p.rstd, p.rows, p.C, p.y32, p.y16,
                       rpw, p.part,
                       p.sum16);
  else
    hipLaunchKernelGGL((ln_bwd_kernel<CH, AT, BT, GM, false>), dim3(blocks), dim3(256), 4 * 2 * p.C * sizeof(float),
                       p.s, p.g32, p.g16, p.gx, p.ldg, p.a, p.b, p.gamma, p.mean, p.rstd, p.rows, p.C, p.y32, p.y16,
                       rpw, p.part,
                       false);
}

// CH x AT x BT resolved at compile time from runtime codes (bt = -1: no b)
template <template <int, int, int> class F, typename... A>
void ln_dispatch(int ch, int at, int bt, A &&...args) {
#define LN_BT(CH_, AT_)                                  \
  if (bt < 0)                                            \
    F<CH_, AT_, -1>::go(args...);                        \
  else if (bt == 0)                                      \
    F<CH_, AT_, 0>::go(args...);                         \
  else                                                   \
    F<CH_, AT_, 1>::go(args...);
  if (ch == 1) {
    if (at == 0) {
      LN_BT(1, 0)
    } else {
      LN_BT(1, 1)
    }
  } else {
    if (at == 0) {
      LN_BT(2, 0)
    } else {
      LN_BT(2, 1)
    }
  }
#undef LN_BT
}

template <int CH, int AT, int BT>
struct LnFwdF {
  static void go(const LnArgs &p) { ln_fwd_go<CH, AT, BT>(p); }
};
template <int CH, int AT, int BT>
struct LnBwdF {
  static void go(const LnArgs &p, int gm, int blocks, int rpw) {
    if (gm == 11)
      ln_bwd_go<CH, AT, BT, 11>(p, blocks, rpw);
    else if (gm == 9)
      ln_bwd_go<CH, AT, BT, 9>(p, blocks, rpw);
    else if (gm == 7)
      ln_bwd_go<CH, AT, BT, 7>(p, blocks, rpw);
    else if (gm == 5)
      ln_bwd_go<CH, AT, BT, 5>(p, blocks, rpw);
    else if (gm == 3)
      ln_bwd_go<CH, AT, BT, 3>(p, blocks, rpw);
    else if (gm == 1)
      ln_bwd_go<CH, AT, BT, 1>(p, blocks, rpw);
    else
      ln_bwd_go<CH, AT, BT, 2>(p, blocks, rpw);
  }
};

int ln_bwd_blocks(int rows) {
  const int rpb = 4 * ln_bwd_rpw(rows);
  return (rows + rpb - 1) / rpb;
}

bool dt_ok(int dt) { return dt == 0 || dt == 1; }

// ---------------------------------------------------------------- add
// out = a + b in the promoted dtype (fp32 unless both are bf16), then the
// output dtype: torch.add(a, b, out=out) with type promotion (fp32 + bf16 -> bf16 is the block outputs that
// feed only GEMMs).  torch runs mixed-dtype adds on its unvectorised dynamic-
// cast kernel (~2.5x the HBM time); here 8 elements per thread, 16-B accesses.
template <int AT, int BT, int OT>
__global__ __launch_bounds__(256) void add_kernel(const void *__restrict__ a, const void *__restrict__ b,
                                                  void *__restrict__ out, long long n8) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    V8 x, y;
    ld8c<AT>(x, a, 8 * i);
    ld8c<BT>(y, b, 8 * i);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      x.v[k] += y.v[k];
      if constexpr (AT == 1 && BT == 1) x.v[k] = (float)(__bf16)x.v[k];  // promoted dtype bf16
    }
    if constexpr (OT == 0)
      st8_f32(reinterpret_cast<float *>(out), 8 * i, x);
    else
      st8_bf16(reinterpret_cast<__bf16 *>(out), 8 * i, x);
  }
}

__global__ void add_tail_kernel(const void *__restrict__ a, int adt, const void *__restrict__ b, int bdt,
                                void *__restrict__ out, int odt, long long i0, long long n) {
  const long long i = i0 + threadIdx.x;
  if (i < n) {
    float v = ld(a, adt, i) + ld(b, bdt, i);
    if (adt == 1 && bdt == 1) v = (float)(__bf16)v;  // promoted dtype bf16
    st(out, odt, i, v);
  }
}

template <int AT, int BT, int OT>
void add_go(const void *a, const void *b, void *out, long long n8, hipStream_t s) {
  long long g = (n8 + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL((add_kernel<AT, BT, OT>), dim3((unsigned)(g < 1 ? 1 : g)), dim3(256), 0, s, a, b, out, n8);
}

// out rows ldo elements apart, a / b contiguous (rows, C): the refinement stage's two decoder
// outputs written straight into the halves of their concatenation (SVDFormer.py:86) instead of
// summed and then copied by torch.cat.  Index arithmetic in 32 bits (n8 < 2^32, host-checked).
template <int AT, int BT, int OT>
__global__ __launch_bounds__(256) void add_rows_kernel(const void *__restrict__ a, const void *__restrict__ b,
                                                       void *__restrict__ out, unsigned n8, unsigned c8,
                                                       long long ldo) {
  for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < n8; i += gridDim.x * 256) {
    const unsigned r = i / c8, c = i - r * c8;
    V8 x, y;
    ld8c<AT>(x, a, 8LL * i);
    ld8c<BT>(y, b, 8LL * i);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      x.v[k] += y.v[k];
      if constexpr (AT == 1 && BT == 1) x.v[k] = (float)(__bf16)x.v[k];  // promoted dtype bf16
    }
    const long long e = (long long)r * ldo + 8 * c;
    if constexpr (OT == 0)
      st8_f32(reinterpret_cast<float *>(out), e, x);
    else
      st8_bf16(reinterpret_cast<__bf16 *>(out), e, x);
  }
}

template <int AT, int BT, int OT>
void add_rows_go(const void *a, const void *b, void *out, unsigned n8, unsigned c8, long long ldo, hipStream_t s) {
  unsigned g = (n8 + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL((add_rows_kernel<AT, BT, OT>), dim3(g < 1 ? 1 : g), dim3(256), 0, s, a, b, out, n8, c8, ldo);
}

// ---------------------------------------------------------------- path-selection blend
// PointSea's SDG path selection F_L = score * F_Q_ + (1 - score) * F_H_ (models_PointSea/PointSea.py:128-131)
// in one pass each way, reproducing torch's per-op roundings: with a bf16 score (autocast: sigmoid of
// a Linear output) t2 = bf16(1 - s), out = s * a + t2 * b in fp32; backward da = g * s, db = g * t2 and
// the score's gradient bf16(bf16(g * a) - bf16(g * b)) -- the two bf16-cast contributions autograd
// adds (MulBackward for score * F_Q_, RsubBackward of MulBackward for (1 - score) * F_H_).  fp32
// score: everything fp32.  Replaces 4 forward and ~8 backward elementwise launches.
template <int ST>
__device__ __forceinline__ float blend_t2(float s) {
  const float t = 1.0f - s;
  return ST == 1 ? (float)(__bf16)t : t;
}

template <int ST, int OT>
__global__ __launch_bounds__(256) void blend_fwd_kernel(const void *__restrict__ score, const float *__restrict__ a,
                                                        const float *__restrict__ b, void *__restrict__ out,
                                                        long long n8) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    V8 sv, av, bv, o;
    ld8c<ST>(sv, score, 8 * i);
    ld8c<0>(av, a, 8 * i);
    ld8c<0>(bv, b, 8 * i);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float t1 = sv.v[k] * av.v[k];
      const float t3 = blend_t2<ST>(sv.v[k]) * bv.v[k];
      o.v[k] = t1 + t3;
    }
    if constexpr (OT == 0)
      st8_f32(reinterpret_cast<float *>(out), 8 * i, o);
    else
      st8_bf16(reinterpret_cast<__bf16 *>(out), 8 * i, o);  // the GEMM operand autocast would cast it to
  }
}

template <int ST, int GT>
__global__ __launch_bounds__(256) void blend_bwd_kernel(const void *__restrict__ g, const void *__restrict__ score,
                                                        const float *__restrict__ a, const float *__restrict__ b,
                                                        float *__restrict__ da, float *__restrict__ db,
                                                        void *__restrict__ ds, long long n8) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    V8 gv, sv, av, bv, oa, ob, os;
    ld8c<GT>(gv, g, 8 * i);
    ld8c<ST>(sv, score, 8 * i);
    ld8c<0>(av, a, 8 * i);
    ld8c<0>(bv, b, 8 * i);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float gk = gv.v[k];
      oa.v[k] = gk * sv.v[k];
      ob.v[k] = gk * blend_t2<ST>(sv.v[k]);
      const float u = gk * av.v[k], w = gk * bv.v[k];
      os.v[k] = ST == 1 ? (float)(__bf16)u - (float)(__bf16)w : u - w;
    }
    if (da) st8_f32(da, 8 * i, oa);
    if (db) st8_f32(db, 8 * i, ob);
    if (ds) {
      if constexpr (ST == 1)
        st8_bf16(reinterpret_cast<__bf16 *>(ds), 8 * i, os);
      else
        st8_f32(reinterpret_cast<float *>(ds), 8 * i, os);
    }
  }
}

// ---------------------------------------------------------------- add + positional embedding
// out[b][m][h] = a[b][m][h] + E[b][h*N + m], E = SinusoidalPositionalEmbedding(cd) flattened per
// batch: E[b][n*H + 2i + c] = (c ? cos : sin)(cd[b][n] * div[i])  (models/model_utils.py:883-917,
// with SDG's raw .reshape(B, hidden, N).permute of it, SVDFormer.py:77-80) -- the sum computed in
// fp32 and stored once in out's dtype, as autocast does before the q / k projection GEMM.
// Replaces torch's sin, cos, mul, cat, the transposed view's copy and the add (7 launches, ~1.4 GB
// per SDG stage at PCN shapes) by one pass over a.
template <int AT, int OT>
__global__ __launch_bounds__(256) void add_posemb_kernel(const void *__restrict__ a, const float *__restrict__ cd,
                                                         const float *__restrict__ div, int N, int H,
                                                         void *__restrict__ out, long long n8) {
  const int H8 = H >> 3;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    V8 x;
    ld8c<AT>(x, a, 8 * i);
    const long long row = i / H8;            // b * N + m
    const int h0 = (int)(i - row * H8) * 8;
    const int b = (int)(row / N), m = (int)(row - (long long)b * N);
    const float *cdb = cd + (long long)b * N;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const long long f = (long long)(h0 + k) * N + m;
      const int n = (int)(f / H), j = (int)(f - (long long)n * H);
      const float w = cdb[n] * div[j >> 1];
      x.v[k] += (j & 1) ? cosf(w) : sinf(w);
    }
    if constexpr (OT == 0)
      st8_f32(reinterpret_cast<float *>(out), 8 * i, x);
    else
      st8_bf16(reinterpret_cast<__bf16 *>(out), 8 * i, x);
  }
}

// ---------------------------------------------------------------- column sum
// out[c] = sum_r g[r][c]: the bias gradient of the blocks' Linear / 1x1-conv
// layers (torch's bf16 sum(0) runs at 0.8-3 TB/s on these (65536, C) inputs).
// Stage 1: grid (chunks, strips), ~1024 blocks; a wave covers V vector columns
// (8 elements: one 16-B load for bf16) x 64/V rows per step, 4 waves step
// through the chunk's rows with up to 16 loads in flight per lane, fp32
// registers; the chunk's partial row is folded by lane shuffles + LDS and
// stored once.  Stage 2: 32 columns x 32 chunk groups per block add the
// <= 1024 partial rows in a fixed order (deterministic, no atomics).
constexpr int kCsMaxChunks = 1024;
constexpr int kCsU = 8;

template <int DT>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const void *__restrict__ g, long long rows, int C, int V,
                                                             long long rpc, float *__restrict__ part, long long ld) {
  __shared__ float red[4][64 * 8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rw = 64 / V;                         // rows per wave step
  const int rsub = lane / V, vi = lane - rsub * V;
  const int col = (blockIdx.y * V + vi) * 8;     // first element column
  const long long r0 = blockIdx.x * rpc, r1 = min(rows, r0 + rpc);
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  // kCsU rows per lane per batch, their loads issued together (rows past r1 read a
  // valid row and count 0): a runtime-count `#pragma unroll` loop here compiled to
  // one load + vmcnt(0) per row (2.5 TB/s)
  const long long step = 4LL * rw;
  for (long long rb = r0 + w * rw + rsub; rb < r1; rb += kCsU * step) {
    V8 t[kCsU];
#pragma unroll
    for (int u = 0; u < kCsU; ++u) {
      const long long r = rb + u * step;
      ld8c<DT>(t[u], g, (r < r1 ? r : rb) * ld + col);
    }
#pragma unroll
    for (int u = 0; u < kCsU; ++u) {
      const bool ok = rb + u * step < r1;
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += ok ? t[u].v[k] : 0.f;
    }
  }
  for (int o = V; o < 64; o <<= 1)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += __shfl_xor(acc[k], o, 64);
  if (rsub == 0)
#pragma unroll
    for (int k = 0; k < 8; ++k) red[w][vi * 8 + k] = acc[k];
  __syncthreads();
  const int t = threadIdx.x;
  for (int i = t; i < V * 8; i += 256) {
    const float s = ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
    part[blockIdx.x * (long long)C + blockIdx.y * V * 8 + i] = s;
  }
}

// columns [0, split) go to out, [split, split2) to out2, [split2, C) to out3
// (the LayerNorm's dgamma | dbeta | fused bias sum, all in odt)
__global__ __launch_bounds__(1024) void colsum_final_kernel(const float *__restrict__ part, int chunks, int C,
                                                            void *__restrict__ out, int odt, int split,
                                                            void *__restrict__ out2, int split2,
                                                            void *__restrict__ out3, int odt3) {
  __shared__ float red[32][33];
  const int cl = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int col = blockIdx.x * 32 + cl;
  float s = 0.f;
  if (col < C)
#pragma unroll 16
    for (int k = grp; k < chunks; k += 32) s += part[(long long)k * C + col];
  red[grp][cl] = s;
  __syncthreads();
  if (grp == 0 && col < C) {
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) tot += red[i][cl];
    if (col < split)
      st(out, odt, col, tot);
    else if (col < split2)
      st(out2, odt, col - split, tot);
    else
      st(out3, odt3, col - split2, tot);
  }
}

// Opt-in variant of colsum_final_kernel (PCOPS_COLSUM_FINAL_CW=16, untimed): CW columns x (1024 / CW)
// row groups per block with 8 loads in flight per thread -- twice the blocks and half the serial
// loads per thread of the 32-column form at CW = 16 (a ~1024-chunk final is latency-bound on 16-96
// blocks).  Fixed order for a given CW.
template <int CW>
__global__ __launch_bounds__(1024) void colsum_final_cw_kernel(const float *__restrict__ part, int chunks, int C,
                                                               void *__restrict__ out, int odt, int split,
                                                               void *__restrict__ out2, int split2,
                                                               void *__restrict__ out3, int odt3) {
  constexpr int G = 1024 / CW, U = 8;
  __shared__ float red[G][CW + 1];
  const int cl = threadIdx.x % CW, grp = threadIdx.x / CW;
  const int col = blockIdx.x * CW + cl;
  float s = 0.f;
  if (col < C)
    for (int k0 = grp; k0 < chunks; k0 += U * G) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + u * G;
        v[u] = part[(long long)(k < chunks ? k : k0) * C + col];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) s += (k0 + u * G < chunks) ? v[u] : 0.f;
    }
  red[grp][cl] = s;
  __syncthreads();
  if (grp == 0 && col < C) {
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < G; ++i) tot += red[i][cl];
    if (col < split)
      st(out, odt, col, tot);
    else if (col < split2)
      st(out2, odt, col - split, tot);
    else
      st(out3, odt3, col - split2, tot);
  }
}

// out3 (the fused bias sum) in its own dtype odt3: the consuming Linear's bias dtype, so no cast follows
void launch_colsum_final(const float *part, int chunks, int C, void *out, int odt, int split, void *out2,
                         int split2, void *out3, hipStream_t s, int odt3 = -1) {
  if (odt3 < 0) odt3 = odt;
  static const int cw = [] {
    const char *e = getenv("PCOPS_COLSUM_FINAL_CW");
    return e ? atoi(e) : 32;
  }();
  if (cw == 16)
    hipLaunchKernelGGL(colsum_final_cw_kernel<16>, dim3((C + 15) / 16), dim3(1024), 0, s, part, chunks, C, out, odt,
                       split, out2, split2, out3, odt3);
  else
    hipLaunchKernelGGL(colsum_final_kernel, dim3((C + 31) / 32), dim3(1024), 0, s, part, chunks, C, out, odt, split,
                       out2, split2, out3, odt3);
}

// GELU backward (exact erf form, torch's GeluBackward expression in fp32) fused
// with the column sum of its output -- the bias gradient of the Linear whose
// output the GELU consumed -- in colsum_partial_kernel's launch shape:
//   du = dy * (Phi(u) + u * phi(u)),  partial[chunk][c] = sum over the chunk's rows of du as stored.
// SUM = false: the GELU backward alone.
template <int DT, bool SUM>
__global__ __launch_bounds__(256) void gelu_bwd_partial_kernel(const void *__restrict__ dy, const void *__restrict__ u,
                                                               void *__restrict__ du, long long rows, int C, int V,
                                                               long long rpc, float *__restrict__ part) {
  __shared__ float red[4][64 * 8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rw = 64 / V;
  const int rsub = lane / V, vi = lane - rsub * V;
  const int col = (blockIdx.y * V + vi) * 8;
  const long long r0 = blockIdx.x * rpc, r1 = min(rows, r0 + rpc);
  constexpr float kAlpha = 0.70710678118654752440f;                      // M_SQRT1_2
  constexpr float kBeta = 1.12837916709551257390f * 0.70710678118654752440f * 0.5f;  // M_2_SQRTPI * M_SQRT1_2 / 2
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  const long long step = 4LL * rw;
  constexpr int U = 4;  // rows per lane per batch, loads issued together (see colsum_partial_kernel)
  for (long long rb = r0 + w * rw + rsub; rb < r1; rb += U * step) {
    V8 g[U], x[U];
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const long long r = rb + i * step;
      const long long e = (r < r1 ? r : rb) * C + col;
      ld8c<DT>(g[i], dy, e);
      ld8c<DT>(x[i], u, e);
    }
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const long long r = rb + i * step;
      const bool ok = r < r1;
      V8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float cdf = 0.5f * (1.0f + erff(x[i].v[k] * kAlpha));
        const float pdf = expf(-0.5f * x[i].v[k] * x[i].v[k]) * kBeta;
        o.v[k] = g[i].v[k] * (cdf + x[i].v[k] * pdf);
      }
      if constexpr (DT == 0) {
        if (ok) st8_f32(reinterpret_cast<float *>(du), r * C + col, o);
      } else {
        if (ok) st8_bf16(reinterpret_cast<__bf16 *>(du), r * C + col, o);
#pragma unroll
        for (int k = 0; k < 8; ++k) o.v[k] = (float)(__bf16)o.v[k];  // the sum sees du as stored
      }
      if constexpr (SUM)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += ok ? o.v[k] : 0.f;
    }
  }
  if constexpr (SUM) {
    for (int o = V; o < 64; o <<= 1)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += __shfl_xor(acc[k], o, 64);
    if (rsub == 0)
#pragma unroll
      for (int k = 0; k < 8; ++k) red[w][vi * 8 + k] = acc[k];
    __syncthreads();
    for (int i = threadIdx.x; i < V * 8; i += 256) {
      const float sm = ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
      part[blockIdx.x * (long long)C + blockIdx.y * V * 8 + i] = sm;
    }
  }
}

// Split-K weight-gradient epilogue: out[i] = sum_{s < S} part[s][i] (fixed order),
// rounded once to out's dtype -- torch ran part.sum(0) (a reduce kernel) and .to(bf16)
// (a copy kernel) per Linear.  Four elements per thread (16-B loads per row).
__global__ __launch_bounds__(256) void sum_rows_kernel(const float *__restrict__ part, int S, long long n4,
                                                       long long N, void *__restrict__ out, int odt) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  // four rows' loads in flight; rows summed in a fixed order (r, r+1, r+2, r+3 into four partials)
  float4 a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  int r = 0;
  for (; r + 3 < S; r += 4)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 v = *reinterpret_cast<const float4 *>(part + (long long)(r + j) * N + 4 * i);
      a[j].x += v.x, a[j].y += v.y, a[j].z += v.z, a[j].w += v.w;
    }
  for (; r < S; ++r) {
    const float4 v = *reinterpret_cast<const float4 *>(part + (long long)r * N + 4 * i);
    a[0].x += v.x, a[0].y += v.y, a[0].z += v.z, a[0].w += v.w;
  }
  float4 acc;
  acc.x = (a[0].x + a[1].x) + (a[2].x + a[3].x);
  acc.y = (a[0].y + a[1].y) + (a[2].y + a[3].y);
  acc.z = (a[0].z + a[1].z) + (a[2].z + a[3].z);
  acc.w = (a[0].w + a[1].w) + (a[2].w + a[3].w);
  if (odt == 0) {
    *reinterpret_cast<float4 *>(reinterpret_cast<float *>(out) + 4 * i) = acc;
  } else {
    typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
    bf16x4_t o;
    o[0] = (__bf16)acc.x, o[1] = (__bf16)acc.y, o[2] = (__bf16)acc.z, o[3] = (__bf16)acc.w;
    *reinterpret_cast<bf16x4_t *>(reinterpret_cast<__bf16 *>(out) + 4 * i) = o;
  }
}

// Many rows over few columns (the split-K weight gradient of a small weight: S = 64..512 slices of
// 192..16K values): a block takes 16 column quads x 16 row slices; slice sl sums rows sl, sl + 16,
// ... with eight loads in flight, then the 16 slices are added in slice order through LDS -- a
// fixed order, so still deterministic.  One thread per column quad walking all S rows (the plain
// kernel) was latency-bound there: 512 dependent-in-groups-of-4 loads in 1..16 blocks.
__global__ __launch_bounds__(256) void sum_rows_sliced_kernel(const float *__restrict__ part, int S, long long n4,
                                                              long long N, void *__restrict__ out, int odt) {
  __shared__ float4 red[16][16];
  const int cq = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const long long i = (long long)blockIdx.x * 16 + cq;
  float4 a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
    int r = sl;
    for (; r + 7 * 16 < S; r += 8 * 16)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float4 v = *reinterpret_cast<const float4 *>(part + (long long)(r + 16 * j) * N + 4 * i);
        a[j].x += v.x, a[j].y += v.y, a[j].z += v.z, a[j].w += v.w;
      }
    for (; r < S; r += 16) {
      const float4 v = *reinterpret_cast<const float4 *>(part + (long long)r * N + 4 * i);
      a[0].x += v.x, a[0].y += v.y, a[0].z += v.z, a[0].w += v.w;
    }
  }
#pragma unroll
  for (int j = 1; j < 8; ++j) a[0].x += a[j].x, a[0].y += a[j].y, a[0].z += a[j].z, a[0].w += a[j].w;
  red[sl][cq] = a[0];
  __syncthreads();
  if (sl != 0 || i >= n4) return;
  float4 acc = red[0][cq];
#pragma unroll
  for (int j = 1; j < 16; ++j) {
    const float4 v = red[j][cq];
    acc.x += v.x, acc.y += v.y, acc.z += v.z, acc.w += v.w;
  }
  if (odt == 0) {
    *reinterpret_cast<float4 *>(reinterpret_cast<float *>(out) + 4 * i) = acc;
  } else {
    typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
    bf16x4_t o;
    o[0] = (__bf16)acc.x, o[1] = (__bf16)acc.y, o[2] = (__bf16)acc.z, o[3] = (__bf16)acc.w;
    *reinterpret_cast<bf16x4_t *>(reinterpret_cast<__bf16 *>(out) + 4 * i) = o;
  }
}

// stage 1 of a long row sum: part2[y][i] = sum_{s = y, y + P, ...} part[s][i] (grid.y = P slices),
// eight independent loads in flight per thread (a single pass over 512 rows was latency-bound)
__global__ __launch_bounds__(256) void sum_rows_split_kernel(const float *__restrict__ part, int S, long long n4,
                                                             long long N, float *__restrict__ part2) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int P = gridDim.y;
  float4 a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  int r = blockIdx.y;
  for (; r + 7 * P < S; r += 8 * P)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float4 v = *reinterpret_cast<const float4 *>(part + (long long)(r + j * P) * N + 4 * i);
      a[j].x += v.x, a[j].y += v.y, a[j].z += v.z, a[j].w += v.w;
    }
  for (; r < S; r += P) {
    const float4 v = *reinterpret_cast<const float4 *>(part + (long long)r * N + 4 * i);
    a[0].x += v.x, a[0].y += v.y, a[0].z += v.z, a[0].w += v.w;
  }
#pragma unroll
  for (int j = 1; j < 8; ++j) a[0].x += a[j].x, a[0].y += a[j].y, a[0].z += a[j].z, a[0].w += a[j].w;
  *reinterpret_cast<float4 *>(part2 + (long long)blockIdx.y * N + 4 * i) = a[0];
}

// Weight gradient of a skinny 1x1 conv / Linear (EdgeConv's first conv: 6 -> 32 channels
// over B*N*K = 1M rows): dW[co][ci] = sum_t g[t][co] * x[t][ci].  As a split-K bmm this
// ran at 1.5 TFLOP/s (N = 6 tiles); here it is one streaming pass: a thread owns 8 output
// channels (one 16-B load of g per row) x CI inputs, RL row lanes per block sum their
// rows, fixed-order block reduce -> part[block][Co*CI], then sum_rows over the blocks.
template <int CI>
__global__ __launch_bounds__(256) void wgrad_skinny_kernel(const __bf16 *__restrict__ g,
                                                           const __bf16 *__restrict__ x, long long T, int Co,
                                                           long long rpb, float *__restrict__ part) {
  __shared__ float red[2048 * CI];  // [RL][Co*CI]: RL * Co <= 256 * 8
  const int ng = Co >> 3, cg = threadIdx.x % ng, rl = threadIdx.x / ng, RL = 256 / ng;
  const long long r0 = blockIdx.x * rpb, r1 = min(T, r0 + rpb);
  float acc[8][CI];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < CI; ++i) acc[j][i] = 0.f;
  if (rl < RL) {
#pragma unroll 4
    for (long long t = r0 + rl; t < r1; t += RL) {
      typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
      const bf16x8_t gv = *reinterpret_cast<const bf16x8_t *>(g + t * Co + 8 * cg);
      float xv[CI];
#pragma unroll
      for (int i = 0; i < CI; ++i) xv[i] = (float)x[t * CI + i];
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int i = 0; i < CI; ++i) acc[j][i] = __builtin_fmaf((float)gv[j], xv[i], acc[j][i]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < CI; ++i) red[rl * Co * CI + (8 * cg + j) * CI + i] = acc[j][i];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < Co * CI; e += 256) {
    float v = 0.f;
    for (int q = 0; q < RL; ++q) v += red[q * Co * CI + e];
    part[(long long)blockIdx.x * Co * CI + e] = v;
  }
}

int colsum_v(int C) {  // vector columns per wave: largest power of two <= 64 dividing C / 8
  const int nv = C / 8;
  int V = 64;
  while (nv % V) V >>= 1;
  return V;
}

// tuning knobs (A/B only): PCOPS_COLSUM_BLOCKS (stage-1 blocks aimed at),
// PCOPS_COLSUM_CHUNKS (cap on partial rows, <= kCsMaxChunks)
int colsum_env(const char *name, int dflt) {
  const char *v = getenv(name);
  return v ? atoi(v) : dflt;
}

void colsum_shape(long long rows, int C, int &chunks, long long &rpc) {
  static const int target = colsum_env("PCOPS_COLSUM_BLOCKS", 1024);
  static const int cap = min(kCsMaxChunks, colsum_env("PCOPS_COLSUM_CHUNKS", kCsMaxChunks));
  const int strips = C / 8 / colsum_v(C);
  long long want = (target + strips - 1) / strips;
  if (want > cap) want = cap;
  if (want > (rows + 15) / 16) want = (rows + 15) / 16;  // >= 16 rows per chunk
  if (want < 1) want = 1;
  rpc = (rows + want - 1) / want;
  chunks = (int)((rows + rpc - 1) / rpc);
}

}  // namespace

extern "C" int pcops_add_posemb(const void *a, int a_dtype, const float *cd, const float *div_term, int B, int N,
                                int H, void *out, int out_dtype, pcops_stream_t stream) {
  if (B < 0 || N < 0 || H <= 0 || (H & 7) || !dt_ok(a_dtype) || !dt_ok(out_dtype)) return PCOPS_ERR_INVALID;
  if (B == 0 || N == 0) return PCOPS_OK;
  if (!a || !cd || !div_term || !out) return PCOPS_ERR_INVALID;
  const long long n8 = (long long)B * N * H / 8;
  long long g = (n8 + 255) / 256;
  if (g > 8192) g = 8192;
  hipStream_t s = (hipStream_t)stream;
  switch (a_dtype * 2 + out_dtype) {
    case 0: hipLaunchKernelGGL((add_posemb_kernel<0, 0>), dim3((unsigned)g), dim3(256), 0, s, a, cd, div_term, N, H, out, n8); break;
    case 1: hipLaunchKernelGGL((add_posemb_kernel<0, 1>), dim3((unsigned)g), dim3(256), 0, s, a, cd, div_term, N, H, out, n8); break;
    case 2: hipLaunchKernelGGL((add_posemb_kernel<1, 0>), dim3((unsigned)g), dim3(256), 0, s, a, cd, div_term, N, H, out, n8); break;
    default: hipLaunchKernelGGL((add_posemb_kernel<1, 1>), dim3((unsigned)g), dim3(256), 0, s, a, cd, div_term, N, H, out, n8); break;
  }
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_add(const void *a, int a_dtype, const void *b, int b_dtype, void *out, int out_dtype,
                         long long n, pcops_stream_t stream) {
  if (n < 0 || !dt_ok(a_dtype) || !dt_ok(b_dtype) || !dt_ok(out_dtype)) return PCOPS_ERR_INVALID;
  if (n == 0) return PCOPS_OK;
  if (!a || !b || !out) return PCOPS_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  const long long n8 = n / 8;
  if (n8 > 0) {
    const int code = a_dtype * 4 + b_dtype * 2 + out_dtype;
    switch (code) {
      case 0: add_go<0, 0, 0>(a, b, out, n8, s); break;
      case 1: add_go<0, 0, 1>(a, b, out, n8, s); break;
      case 2: add_go<0, 1, 0>(a, b, out, n8, s); break;
      case 3: add_go<0, 1, 1>(a, b, out, n8, s); break;
      case 4: add_go<1, 0, 0>(a, b, out, n8, s); break;
      case 5: add_go<1, 0, 1>(a, b, out, n8, s); break;
      case 6: add_go<1, 1, 0>(a, b, out, n8, s); break;
      default: add_go<1, 1, 1>(a, b, out, n8, s); break;
    }
    PC_CHECK_LAUNCH();
  }
  if (n8 * 8 < n) {
    hipLaunchKernelGGL(add_tail_kernel, dim3(1), dim3(64), 0, s, a, a_dtype, b, b_dtype, out, out_dtype, n8 * 8, n);
    PC_CHECK_LAUNCH();
  }
  return PCOPS_OK;
}

extern "C" int pcops_add_rows(const void *a, int a_dtype, const void *b, int b_dtype, void *out, int out_dtype,
                              long long rows, int C, long long ld_out, pcops_stream_t stream) {
  if (rows < 0 || C <= 0 || !dt_ok(a_dtype) || !dt_ok(b_dtype) || !dt_ok(out_dtype)) return PCOPS_ERR_INVALID;
  if (rows == 0) return PCOPS_OK;
  if (!a || !b || !out || ld_out < C) return PCOPS_ERR_INVALID;
  if (C % 8 || ld_out % 8 || rows * (C / 8) >= (1LL << 32)) return PCOPS_ERR_UNSUPPORTED;
  if ((reinterpret_cast<unsigned long long>(a) | reinterpret_cast<unsigned long long>(b) |
       reinterpret_cast<unsigned long long>(out)) & 15)
    return PCOPS_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const unsigned n8 = (unsigned)(rows * (C / 8)), c8 = (unsigned)(C / 8);
  switch (a_dtype * 4 + b_dtype * 2 + out_dtype) {
    case 0: add_rows_go<0, 0, 0>(a, b, out, n8, c8, ld_out, s); break;
    case 1: add_rows_go<0, 0, 1>(a, b, out, n8, c8, ld_out, s); break;
    case 2: add_rows_go<0, 1, 0>(a, b, out, n8, c8, ld_out, s); break;
    case 3: add_rows_go<0, 1, 1>(a, b, out, n8, c8, ld_out, s); break;
    case 4: add_rows_go<1, 0, 0>(a, b, out, n8, c8, ld_out, s); break;
    case 5: add_rows_go<1, 0, 1>(a, b, out, n8, c8, ld_out, s); break;
    case 6: add_rows_go<1, 1, 0>(a, b, out, n8, c8, ld_out, s); break;
    default: add_rows_go<1, 1, 1>(a, b, out, n8, c8, ld_out, s); break;
  }
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

namespace {
unsigned blend_grid(long long n8) {
  long long g = (n8 + 255) / 256;
  return (unsigned)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}
}  // namespace

extern "C" int pcops_blend_fwd(const void *score, int score_dtype, const float *a, const float *b, long long n,
                               void *out, int out_dtype, pcops_stream_t stream) {
  if (n < 0 || !dt_ok(score_dtype) || !dt_ok(out_dtype)) return PCOPS_ERR_INVALID;
  if (n == 0) return PCOPS_OK;
  if (!score || !a || !b || !out) return PCOPS_ERR_INVALID;
  if (n % 8) return PCOPS_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const long long n8 = n / 8;
  const dim3 grid(blend_grid(n8));
  switch (score_dtype * 2 + out_dtype) {
    case 0: hipLaunchKernelGGL((blend_fwd_kernel<0, 0>), grid, dim3(256), 0, s, score, a, b, out, n8); break;
    case 1: hipLaunchKernelGGL((blend_fwd_kernel<0, 1>), grid, dim3(256), 0, s, score, a, b, out, n8); break;
    case 2: hipLaunchKernelGGL((blend_fwd_kernel<1, 0>), grid, dim3(256), 0, s, score, a, b, out, n8); break;
    default: hipLaunchKernelGGL((blend_fwd_kernel<1, 1>), grid, dim3(256), 0, s, score, a, b, out, n8); break;
  }
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_blend_bwd(const void *g, int g_dtype, const void *score, int score_dtype, const float *a,
                               const float *b, long long n, float *da, float *db, void *dscore,
                               pcops_stream_t stream) {
  if (n < 0 || !dt_ok(score_dtype) || !dt_ok(g_dtype)) return PCOPS_ERR_INVALID;
  if (n == 0) return PCOPS_OK;
  if (!g || !score || !a || !b) return PCOPS_ERR_INVALID;
  if (n % 8) return PCOPS_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const long long n8 = n / 8;
  const dim3 grid(blend_grid(n8));
  switch (score_dtype * 2 + g_dtype) {
    case 0: hipLaunchKernelGGL((blend_bwd_kernel<0, 0>), grid, dim3(256), 0, s, g, score, a, b, da, db, dscore, n8); break;
    case 1: hipLaunchKernelGGL((blend_bwd_kernel<0, 1>), grid, dim3(256), 0, s, g, score, a, b, da, db, dscore, n8); break;
    case 2: hipLaunchKernelGGL((blend_bwd_kernel<1, 0>), grid, dim3(256), 0, s, g, score, a, b, da, db, dscore, n8); break;
    default: hipLaunchKernelGGL((blend_bwd_kernel<1, 1>), grid, dim3(256), 0, s, g, score, a, b, da, db, dscore, n8); break;
  }
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_transpose_add(const void *a, int a_dtype, const void *b, int b_dtype, void *out, int out_dtype,
                                   void *out2, int out2_dtype, int B, int R, int C, pcops_stream_t stream) {
  if (B < 0 || R < 0 || C < 0) return PCOPS_ERR_INVALID;
  if (B == 0 || R == 0 || C == 0) return PCOPS_OK;
  if (!a || !out || !dt_ok(a_dtype) || !dt_ok(out_dtype) || (b && !dt_ok(b_dtype)) || (out2 && !dt_ok(out2_dtype)))
    return PCOPS_ERR_INVALID;
  const dim3 grid((C + kT - 1) / kT, (R + kT - 1) / kT, B);
  hipLaunchKernelGGL(transpose_add_kernel, grid, dim3(256), 0, (hipStream_t)stream, a, a_dtype, b, b_dtype, out,
                     out_dtype, out2, out2_dtype, R, C);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_layernorm_fwd(const void *a, int a_dtype, const void *b, int b_dtype, const float *gamma,
                                   const float *beta, float eps, int rows, int C, float *y32, void *y16, float *mean,
                                   float *rstd, pcops_stream_t stream) {
  if (rows < 0 || C <= 0) return PCOPS_ERR_INVALID;
  if (rows == 0) return PCOPS_OK;
  if (C > 512 * kMaxCh || C % 8) return PCOPS_ERR_UNSUPPORTED;
  if (!a || !gamma || !beta || !mean || !rstd || (!y32 && !y16) || !dt_ok(a_dtype) || (b && !dt_ok(b_dtype)))
    return PCOPS_ERR_INVALID;
  LnArgs p{};
  p.a = a;
  p.b = b;
  p.gamma = gamma;
  p.beta = beta;
  p.mean = mean;
  p.rstd = rstd;
  p.eps = eps;
  p.rows = rows;
  p.C = C;
  p.y32 = y32;
  p.y16 = (__bf16 *)y16;
  p.s = (hipStream_t)stream;
  ln_dispatch<LnFwdF>(C <= 512 ? 1 : 2, a_dtype, b ? b_dtype : -1, p);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" unsigned long long pcops_layernorm_bwd_workspace_bytes(int rows, int C) {
  if (rows <= 0 || C <= 0) return 0;
  return (unsigned long long)ln_bwd_blocks(rows) * 2 * C * sizeof(float);
}

namespace {
int layernorm_bwd_impl(const float *dy32, const void *dy16, const void *a, int a_dtype, const void *b, int b_dtype,
                       const float *gamma, const float *mean, const float *rstd, int rows, int C, float *dx32,
                       void *dx16, float *dgamma, float *dbeta, void *dsum, int dsum_src, void *workspace,
                       unsigned long long workspace_bytes, unsigned long long need, hipStream_t s,
                       bool dy32_bf16 = false, const void *dyx = nullptr, long long ldg = 0) {
  if (rows < 0 || C <= 0) return PCOPS_ERR_INVALID;
  if (C > 512 * kMaxCh || C % 8) return PCOPS_ERR_UNSUPPORTED;
  if (!dgamma || !dbeta) return PCOPS_ERR_INVALID;
  if (dsum_src & ~3) return PCOPS_ERR_INVALID;
  const int dsum_dt = (dsum_src >> 1) & 1;   // bit 1: dsum stored bf16 (the consuming bias's dtype)
  dsum_src &= 1;
  if (dsum && ((dsum_src == 1 && !dx16) || (dsum_src == 0 && !dx32)))
    return PCOPS_ERR_INVALID;
  if (rows == 0) {
    if (pc_memset_async(dgamma, 0, sizeof(float) * C, s) != hipSuccess ||
        pc_memset_async(dbeta, 0, sizeof(float) * C, s) != hipSuccess ||
        (dsum && pc_memset_async(dsum, 0, (dsum_dt ? 2 : 4) * (size_t)C, s) != hipSuccess))
      return PCOPS_ERR_LAUNCH;
    return PCOPS_OK;
  }
  if (!a || !gamma || !mean || !rstd || (!dy32 && !dy16) || (!dx32 && !dx16) || !dt_ok(a_dtype) ||
      (b && !dt_ok(b_dtype)))
    return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < need) return PCOPS_ERR_WORKSPACE;
  const int blocks = ln_bwd_blocks(rows);
  float *part = (float *)workspace;
  LnArgs p{};
  p.a = a;
  p.b = b;
  p.g32 = dy32;
  p.g16 = (const __bf16 *)dy16;
  p.gx = (const __bf16 *)dyx;
  p.ldg = ldg > 0 ? ldg : C;
  p.gamma = gamma;
  p.mean = mean;
  p.rstd = rstd;
  p.rows = rows;
  p.C = C;
  p.y32 = dx32;
  p.y16 = (__bf16 *)dx16;
  p.part = part;
  p.cs = dsum != nullptr;
  p.sum16 = dsum_src == 1;
  p.s = s;
  ln_dispatch<LnBwdF>(C <= 512 ? 1 : 2, a_dtype, b ? b_dtype : -1, p,
                      (dy32 ? 1 : 0) | (dy16 ? 2 : 0) | (dy32_bf16 ? 4 : 0) | (dyx ? 8 : 0), blocks,
                      ln_bwd_rpw(rows));
  const int np = dsum ? 3 : 2;
  launch_colsum_final(part, blocks, np * C, (void *)dgamma, 0, C, (void *)dbeta, 2 * C, dsum, s, dsum_dt);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
}  // namespace

extern "C" int pcops_layernorm_bwd(const float *dy32, const void *dy16, const void *a, int a_dtype, const void *b,
                                   int b_dtype, const float *gamma, const float *mean, const float *rstd, int rows,
                                   int C, float *dx32, void *dx16, float *dgamma, float *dbeta, void *workspace,
                                   unsigned long long workspace_bytes, pcops_stream_t stream) {
  return layernorm_bwd_impl(dy32, dy16, a, a_dtype, b, b_dtype, gamma, mean, rstd, rows, C, dx32, dx16, dgamma, dbeta,
                            nullptr, 0, workspace, workspace_bytes, pcops_layernorm_bwd_workspace_bytes(rows, C),
                            (hipStream_t)stream);
}

extern "C" unsigned long long pcops_layernorm_bwd_colsum_workspace_bytes(int rows, int C) {
  if (rows <= 0 || C <= 0) return 0;
  return (unsigned long long)ln_bwd_blocks(rows) * 3 * C * sizeof(float);
}

extern "C" int pcops_layernorm_bwd_colsum(const float *dy32, const void *dy16, const void *a, int a_dtype,
                                          const void *b, int b_dtype, const float *gamma, const float *mean,
                                          const float *rstd, int rows, int C, float *dx32, void *dx16, float *dgamma,
                                          float *dbeta, void *dsum, int dsum_src, void *workspace,
                                          unsigned long long workspace_bytes, pcops_stream_t stream) {
  if (!dsum) return PCOPS_ERR_INVALID;
  return layernorm_bwd_impl(dy32, dy16, a, a_dtype, b, b_dtype, gamma, mean, rstd, rows, C, dx32, dx16, dgamma, dbeta,
                            dsum, dsum_src, workspace, workspace_bytes,
                            pcops_layernorm_bwd_colsum_workspace_bytes(rows, C), (hipStream_t)stream);
}

extern "C" int pcops_layernorm_bwd_bf16g(const void *dy_a, const void *dy16, const void *a, int a_dtype,
                                         const void *b, int b_dtype, const float *gamma, const float *mean,
                                         const float *rstd, int rows, int C, float *dx32, void *dx16, float *dgamma,
                                         float *dbeta, void *dsum, int dsum_src, void *workspace,
                                         unsigned long long workspace_bytes, pcops_stream_t stream) {
  if (!dy_a || !dy16) return PCOPS_ERR_INVALID;
  return layernorm_bwd_impl((const float *)dy_a, dy16, a, a_dtype, b, b_dtype, gamma, mean, rstd, rows, C, dx32, dx16,
                            dgamma, dbeta, dsum, dsum_src, workspace, workspace_bytes,
                            dsum ? pcops_layernorm_bwd_colsum_workspace_bytes(rows, C)
                                 : pcops_layernorm_bwd_workspace_bytes(rows, C),
                            (hipStream_t)stream, true);
}

extern "C" int pcops_layernorm_bwd_ex(const void *dy, int dy_dtype, long long ld_dy, const void *dy_x,
                                      const void *dy16, const void *a, int a_dtype, const void *b, int b_dtype,
                                      const float *gamma, const float *mean, const float *rstd, int rows, int C,
                                      float *dx32, void *dx16, float *dgamma, float *dbeta, void *dsum, int dsum_src,
                                      void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream) {
  if (!dy || !dt_ok(dy_dtype)) return PCOPS_ERR_INVALID;
  if (ld_dy < C || ld_dy % 8 || (reinterpret_cast<unsigned long long>(dy) & 15)) return PCOPS_ERR_INVALID;
  if (dy_x && dy_dtype != 0) return PCOPS_ERR_UNSUPPORTED;   // instantiated: fp32 dy + dy_x (+ dy16)
  return layernorm_bwd_impl((const float *)dy, dy16, a, a_dtype, b, b_dtype, gamma, mean, rstd, rows, C, dx32, dx16,
                            dgamma, dbeta, dsum, dsum_src, workspace, workspace_bytes,
                            dsum ? pcops_layernorm_bwd_colsum_workspace_bytes(rows, C)
                                 : pcops_layernorm_bwd_workspace_bytes(rows, C),
                            (hipStream_t)stream, dy_dtype == 1, dy_x, ld_dy);
}

extern "C" unsigned long long pcops_colsum_workspace_bytes(long long rows, int C) {
  if (rows <= 0 || C <= 0 || C % 8) return 0;
  int chunks;
  long long rpc;
  colsum_shape(rows, C, chunks, rpc);
  return (unsigned long long)chunks * C * sizeof(float);
}

extern "C" int pcops_gelu_bwd_colsum(const void *dy, const void *u, int dtype, long long rows, int C, void *du,
                                     void *dsum, int dsum_dtype, void *workspace, unsigned long long workspace_bytes,
                                     pcops_stream_t stream) {
  if (rows < 0 || C <= 0 || !dt_ok(dtype) || (dsum && !dt_ok(dsum_dtype))) return PCOPS_ERR_INVALID;
  if (C % 8) return PCOPS_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  if (rows == 0) {
    if (dsum && pc_memset_async(dsum, 0, (dsum_dtype == 0 ? 4 : 2) * (size_t)C, s) != hipSuccess) return PCOPS_ERR_LAUNCH;
    return PCOPS_OK;
  }
  if (!dy || !u || !du) return PCOPS_ERR_INVALID;
  if (dsum && (!workspace || workspace_bytes < pcops_colsum_workspace_bytes(rows, C))) return PCOPS_ERR_WORKSPACE;
  int chunks;
  long long rpc;
  colsum_shape(rows, C, chunks, rpc);
  const int V = colsum_v(C);
  const dim3 grid(chunks, C / 8 / V);
  float *part = (float *)workspace;
  if (dsum) {
    if (dtype == 0)
      hipLaunchKernelGGL((gelu_bwd_partial_kernel<0, true>), grid, dim3(256), 0, s, dy, u, du, rows, C, V, rpc, part);
    else
      hipLaunchKernelGGL((gelu_bwd_partial_kernel<1, true>), grid, dim3(256), 0, s, dy, u, du, rows, C, V, rpc, part);
    launch_colsum_final(part, chunks, C, dsum, dsum_dtype, C, nullptr, C, nullptr, s);
  } else {
    if (dtype == 0)
      hipLaunchKernelGGL((gelu_bwd_partial_kernel<0, false>), grid, dim3(256), 0, s, dy, u, du, rows, C, V, rpc,
                         nullptr);
    else
      hipLaunchKernelGGL((gelu_bwd_partial_kernel<1, false>), grid, dim3(256), 0, s, dy, u, du, rows, C, V, rpc,
                         nullptr);
  }
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_colsum(const void *g, int g_dtype, long long rows, int C, void *out, int out_dtype,
                            void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream) {
  return pcops_colsum_ld(g, g_dtype, rows, C, C, out, out_dtype, workspace, workspace_bytes, stream);
}

extern "C" int pcops_colsum_ld(const void *g, int g_dtype, long long rows, int C, long long ld, void *out,
                               int out_dtype, void *workspace, unsigned long long workspace_bytes,
                               pcops_stream_t stream) {
  if (rows < 0 || C <= 0 || ld < C || !dt_ok(g_dtype) || !dt_ok(out_dtype) || !out) return PCOPS_ERR_INVALID;
  if (C % 8 || ld % 8) return PCOPS_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  if (rows == 0) {
    if (pc_memset_async(out, 0, (size_t)C * (out_dtype == 0 ? 4 : 2), s) != hipSuccess) return PCOPS_ERR_LAUNCH;
    return PCOPS_OK;
  }
  if (!g) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_colsum_workspace_bytes(rows, C)) return PCOPS_ERR_WORKSPACE;
  int chunks;
  long long rpc;
  colsum_shape(rows, C, chunks, rpc);
  const int V = colsum_v(C);
  const dim3 grid(chunks, C / 8 / V);
  float *part = (float *)workspace;
  if (g_dtype == 0)
    hipLaunchKernelGGL(colsum_partial_kernel<0>, grid, dim3(256), 0, s, g, rows, C, V, rpc, part, ld);
  else
    hipLaunchKernelGGL(colsum_partial_kernel<1>, grid, dim3(256), 0, s, g, rows, C, V, rpc, part, ld);
  launch_colsum_final(part, chunks, C, out, out_dtype, C, nullptr, C, nullptr, s);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_sum_rows(const float *part, int S, long long N, void *out, int out_dtype, pcops_stream_t stream) {
  if (S <= 0 || N < 0 || !dt_ok(out_dtype)) return PCOPS_ERR_INVALID;
  if (N == 0) return PCOPS_OK;
  if (N % 4) return PCOPS_ERR_UNSUPPORTED;
  if (!part || !out) return PCOPS_ERR_INVALID;
  const long long n4 = N / 4;
  static const bool sliced = colsum_env("PCOPS_SUMROWS_SLICED", 1) != 0;
  if (S >= 32 && sliced)
    hipLaunchKernelGGL(sum_rows_sliced_kernel, dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0, (hipStream_t)stream,
                       part, S, n4, N, out, out_dtype);
  else
    hipLaunchKernelGGL(sum_rows_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, part,
                       S, n4, N, out, out_dtype);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

constexpr int kSkinnyBlocks = 512;

constexpr int kSkinnySplit = 32;

extern "C" unsigned long long pcops_wgrad_skinny_workspace_bytes(int Co, int Ci) {
  return (unsigned long long)(kSkinnyBlocks + kSkinnySplit) * Co * Ci * sizeof(float);
}

extern "C" int pcops_wgrad_skinny(const void *g, const void *x, long long T, int Co, int Ci, void *dw, int dw_dtype,
                                  void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream) {
  if (T < 0 || Co <= 0 || Ci <= 0 || !dw || !dt_ok(dw_dtype)) return PCOPS_ERR_INVALID;
  if (Ci != 6 || Co % 8 || Co > 64 || (Co * Ci) % 4) return PCOPS_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  if (T == 0) {
    if (pc_memset_async(dw, 0, (size_t)Co * Ci * (dw_dtype == 0 ? 4 : 2), s) != hipSuccess) return PCOPS_ERR_LAUNCH;
    return PCOPS_OK;
  }
  if (!g || !x) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_wgrad_skinny_workspace_bytes(Co, Ci)) return PCOPS_ERR_WORKSPACE;
  const long long rpb = (T + kSkinnyBlocks - 1) / kSkinnyBlocks;
  const int blocks = (int)((T + rpb - 1) / rpb);
  float *part = (float *)workspace;
  hipLaunchKernelGGL(wgrad_skinny_kernel<6>, dim3(blocks), dim3(256), 0, s, (const __bf16 *)g, (const __bf16 *)x, T, Co,
                     rpb, part);
  const long long N = (long long)Co * Ci, n4 = N / 4;
  float *part2 = part + (long long)kSkinnyBlocks * N;
  hipLaunchKernelGGL(sum_rows_split_kernel, dim3((unsigned)((n4 + 255) / 256), kSkinnySplit), dim3(256), 0, s, part,
                     blocks, n4, N, part2);
  hipLaunchKernelGGL(sum_rows_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, part2, kSkinnySplit, n4, N,
                     dw, dw_dtype);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
