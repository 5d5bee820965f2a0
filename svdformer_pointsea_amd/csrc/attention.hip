// Attention core of nn.MultiheadAttention as used by self_attention /
// cross_attention (models/model_utils.py:542-617): O = softmax(scale QK^T) V,
// flash-style on gfx950 MFMA.  Only the two contractions run on the matrix
// cores (32x32 tiles); softmax, masking and rescaling stay in VALU registers.
//
// Structure ("entity on the lane"): a wave owns 32 entities (queries for the
// forward / dQ pass, keys for the dK/dV pass) whose operand fragment stays in
// VGPRs; the other side streams through LDS in 32-row tiles.
//   product 1:  X(32 rows x 32 entities) = Rows(32 x D) . Ent(D x 32)
//   product 2:  Y(D x 32)             += Rows^T(D x 32) . X   (X used in place:
//               its rows are the MFMA k index, so no lane movement is needed;
//               the bf16 Rows^T fragment comes from ds_read_b64_tr_b16)
// forward : X = S^T (keys x queries), Y = O^T            (Rows = K, then V)
// dQ pass : X = S^T, dP^T; dS^T = P^T o (dP^T - delta);  Y = dQ^T (Rows = K)
// dKV pass: X = S, dP (queries x keys); Y1 = dV^T (Rows = dO), Y2 = dK^T (Rows = Q)
// Precision: bf16 operands (v_mfma_f32_32x32x16_bf16, fp32 accumulate) for
// speed, or fp32 operands (v_mfma_f32_32x32x2_f32, exact fp32 fma chain) for
// the parity build.
#include "common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWaves = 4;
constexpr int kThreads = kWaves * 64;
constexpr int kRows = 32;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ int lane_() { return threadIdx.x & 63; }

// accumulator row held by register r of lane half h (32x32 MFMA C/D map)
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ float other_half(float v) { return __shfl_xor(v, 32, 64); }

// ----------------------------------------------------------------- precisions
template <typename T, int D>
struct Prec;

template <int D>
struct Prec<__bf16, D> {
  static constexpr int kStride = D + 8;  // LDS row stride (elements): 16-B shift per row
  struct Frag {
    bf16x8 v[D / 16];
  };
  // entity fragment: lane l holds entity l&31, d = 16s + 8h + j
  __device__ static void load_frag(Frag &f, const __bf16 *row, bool valid) {
    const int h = lane_() >> 5;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      if (valid)
        f.v[s] = *reinterpret_cast<const bf16x8 *>(row + 16 * s + 8 * h);
      else
        f.v[s] = bf16x8{};
    }
  }
  __device__ static void product1(f32x16 &acc, const __bf16 *lds, const Frag &f) {
    const int l = lane_(), h = l >> 5;
    const __bf16 *rp = lds + (l & 31) * kStride + 8 * h;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      const bf16x8 a = *reinterpret_cast<const bf16x8 *>(rp + 16 * s);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, f.v[s], acc, 0, 0, 0);
    }
  }
  // Y[db] += Rows^T . X   (X fp32 accumulator, converted to bf16 in place)
  __device__ static void product2(f32x16 (&Y)[D / 32], const __bf16 *lds, const f32x16 &X) {
#if defined(__HIP_DEVICE_COMPILE__)
    const int l = lane_(), h = l >> 5, g = (l >> 4) & 1, i = l & 15, q = i >> 2, p = i & 3;
    typedef __attribute__((address_space(3))) short4v lds_s4;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 b;
#pragma unroll
      for (int e = 0; e < 8; ++e) b[e] = (__bf16)X[8 * s + e];
      const int row0 = 16 * s + 4 * h + q;
#pragma unroll
      for (int db = 0; db < D / 32; ++db) {
        const int col = db * 32 + 16 * g + 4 * p;
        const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(lds + row0 * kStride + col));
        const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(lds + (row0 + 8) * kStride + col));
        const bf16x8 a = __builtin_shufflevector(__builtin_bit_cast(bf16x4, lo), __builtin_bit_cast(bf16x4, hi), 0, 1,
                                                 2, 3, 4, 5, 6, 7);
        Y[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, Y[db], 0, 0, 0);
      }
    }
#endif
  }
  __device__ static float to_f(__bf16 v) { return (float)v; }
  __device__ static __bf16 from_f(float v) { return (__bf16)v; }
};

template <int D>
struct Prec<float, D> {
  static constexpr int kStride = D + 1;  // odd stride: column reads hit 32 banks
  struct Frag {
    float v[D / 2];
  };
  // lane l holds entity l&31, d = 2s + h
  __device__ static void load_frag(Frag &f, const float *row, bool valid) {
    const int h = lane_() >> 5;
#pragma unroll
    for (int s = 0; s < D / 2; ++s) f.v[s] = valid ? row[2 * s + h] : 0.f;
  }
  __device__ static void product1(f32x16 &acc, const float *lds, const Frag &f) {
    const int l = lane_(), h = l >> 5;
    const float *rp = lds + (l & 31) * kStride + h;
#pragma unroll
    for (int s = 0; s < D / 2; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(rp[2 * s], f.v[s], acc, 0, 0, 0);
  }
  __device__ static void product2(f32x16 (&Y)[D / 32], const float *lds, const f32x16 &X) {
    const int l = lane_(), h = l >> 5;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float *rp = lds + acc_row(r, h) * kStride + (l & 31);
#pragma unroll
      for (int db = 0; db < D / 32; ++db)
        Y[db] = __builtin_amdgcn_mfma_f32_32x32x2f32(rp[db * 32], X[r], Y[db], 0, 0, 0);
    }
  }
  __device__ static float to_f(float v) { return v; }
  __device__ static float from_f(float v) { return v; }
};

// stage rows [r0, r0+32) x D of a (bh-offset) tensor into LDS; rows >= L -> 0
template <typename T, int D>
__device__ __forceinline__ void stage_tile(T *lds, const T *base, long long s_row, int r0, int L) {
  constexpr int kStride = Prec<T, D>::kStride;
  if constexpr (sizeof(T) == 2) {
    constexpr int kChunks = D / 8;  // 16-byte chunks per row
    for (int c = threadIdx.x; c < kRows * kChunks; c += kThreads) {
      const int row = c / kChunks, ch = c - row * kChunks;
      bf16x8 v{};
      if (r0 + row < L) v = *reinterpret_cast<const bf16x8 *>(base + (long long)(r0 + row) * s_row + ch * 8);
      *reinterpret_cast<bf16x8 *>(lds + row * kStride + ch * 8) = v;
    }
  } else {
    constexpr int kChunks = D / 4;
    for (int c = threadIdx.x; c < kRows * kChunks; c += kThreads) {
      const int row = c / kChunks, ch = c - row * kChunks;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r0 + row < L) v = *reinterpret_cast<const float4 *>(base + (long long)(r0 + row) * s_row + ch * 4);
      T *dst = lds + row * kStride + ch * 4;
      dst[0] = v.x;
      dst[1] = v.y;
      dst[2] = v.z;
      dst[3] = v.w;
    }
  }
}

// store Y (D x 32 entities) as out[entity][d] (row = entity), times `mul`
template <typename T, int D>
__device__ __forceinline__ void store_Y(const f32x16 (&Y)[D / 32], T *base, long long s_row, int e0, int L,
                                        float mul) {
  const int l = lane_(), h = l >> 5, e = e0 + (l & 31);
  if (e >= L) return;
  T *row = base + (long long)e * s_row;
#pragma unroll
  for (int db = 0; db < D / 32; ++db)
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) {
      const int d = db * 32 + 8 * r4 + 4 * h;
      if constexpr (sizeof(T) == 2) {
        bf16x4 v;
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = (__bf16)(Y[db][4 * r4 + c] * mul);
        *reinterpret_cast<bf16x4 *>(row + d) = v;
      } else {
        *reinterpret_cast<float4 *>(row + d) =
            make_float4(Y[db][4 * r4] * mul, Y[db][4 * r4 + 1] * mul, Y[db][4 * r4 + 2] * mul, Y[db][4 * r4 + 3] * mul);
      }
    }
}

struct Strides {
  long long q_sbh, q_srow, k_sbh, k_srow, v_sbh, v_srow, o_sbh, o_srow;
};

// ----------------------------------------------------------------- forward
template <typename T, int D>
__global__ __launch_bounds__(kThreads) void attn_fwd_kernel(const T *__restrict__ Q, const T *__restrict__ K,
                                                            const T *__restrict__ V, T *__restrict__ O,
                                                            float *__restrict__ lse, int Lq, int Lk, float scale,
                                                            Strides st) {
  using P = Prec<T, D>;
  __shared__ __attribute__((aligned(16))) T sk[kRows * P::kStride];
  __shared__ __attribute__((aligned(16))) T sv[kRows * P::kStride];
  const int bh = blockIdx.y;
  const int l = lane_(), h = l >> 5, w = threadIdx.x >> 6;
  const int q0 = blockIdx.x * (kWaves * 32) + w * 32;
  const int qi = q0 + (l & 31);
  typename P::Frag qf;
  P::load_frag(qf, Q + bh * st.q_sbh + (long long)(qi < Lq ? qi : 0) * st.q_srow, qi < Lq);
  const T *Kb = K + bh * st.k_sbh;
  const T *Vb = V + bh * st.v_sbh;
  const float sl2 = scale * kLog2e;
  float m = -INFINITY, lsum = 0.f;
  f32x16 Y[D / 32];
#pragma unroll
  for (int db = 0; db < D / 32; ++db) Y[db] = f32x16{};

  for (int k0 = 0; k0 < Lk; k0 += kRows) {
    stage_tile<T, D>(sk, Kb, st.k_srow, k0, Lk);
    stage_tile<T, D>(sv, Vb, st.v_srow, k0, Lk);
    __syncthreads();
    f32x16 X = f32x16{};
    P::product1(X, sk, qf);
    float tmax = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float s = (k0 + acc_row(r, h) < Lk) ? X[r] * sl2 : -INFINITY;
      X[r] = s;
      tmax = fmaxf(tmax, s);
    }
    tmax = fmaxf(tmax, other_half(tmax));
    const float mn = fmaxf(m, tmax);
    const float alpha = exp2f(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float pv = exp2f(X[r] - mn);
      X[r] = pv;
      rs += pv;
    }
    rs += other_half(rs);
    lsum = lsum * alpha + rs;
    m = mn;
    if (alpha != 1.f) {
#pragma unroll
      for (int db = 0; db < D / 32; ++db) Y[db] *= alpha;
    }
    P::product2(Y, sv, X);
    __syncthreads();
  }
  store_Y<T, D>(Y, O + bh * st.o_sbh, st.o_srow, q0, Lq, 1.f / lsum);
  if (h == 0 && qi < Lq && lse) lse[(long long)bh * Lq + qi] = (m + log2f(lsum)) * kLn2;
}

// delta[bh][q] = sum_d dO[q][d] * O[q][d]  (one wave per row)
template <typename T>
__global__ void attn_delta_kernel(const T *__restrict__ O, const T *__restrict__ dO, float *__restrict__ delta,
                                  int BH, int Lq, int D, Strides st) {
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= BH * Lq) return;
  const int bh = row / Lq, q = row - bh * Lq;
  const T *o = O + bh * st.o_sbh + (long long)q * st.o_srow;
  const T *g = dO + bh * st.o_sbh + (long long)q * st.o_srow;
  float s = 0.f;
  for (int d = lane_(); d < D; d += 64) s += Prec<T, 32>::to_f(o[d]) * Prec<T, 32>::to_f(g[d]);
  s = wave_sum_f32(s);
  if (lane_() == 0) delta[row] = s;
}

// ----------------------------------------------------------------- dQ pass
template <typename T, int D>
__global__ __launch_bounds__(kThreads) void attn_dq_kernel(const T *__restrict__ Q, const T *__restrict__ K,
                                                           const T *__restrict__ V, const T *__restrict__ dO,
                                                           const float *__restrict__ lse,
                                                           const float *__restrict__ delta, T *__restrict__ dQ,
                                                           int Lq, int Lk, float scale, Strides st) {
  using P = Prec<T, D>;
  __shared__ __attribute__((aligned(16))) T sk[kRows * P::kStride];
  __shared__ __attribute__((aligned(16))) T sv[kRows * P::kStride];
  const int bh = blockIdx.y;
  const int l = lane_(), h = l >> 5, w = threadIdx.x >> 6;
  const int q0 = blockIdx.x * (kWaves * 32) + w * 32;
  const int qi = q0 + (l & 31);
  const bool qv = qi < Lq;
  typename P::Frag qf, gf;
  P::load_frag(qf, Q + bh * st.q_sbh + (long long)(qv ? qi : 0) * st.q_srow, qv);
  P::load_frag(gf, dO + bh * st.o_sbh + (long long)(qv ? qi : 0) * st.o_srow, qv);
  const float lse2 = qv ? lse[(long long)bh * Lq + qi] * kLog2e : INFINITY;
  const float dl = qv ? delta[(long long)bh * Lq + qi] : 0.f;
  const T *Kb = K + bh * st.k_sbh;
  const T *Vb = V + bh * st.v_sbh;
  const float sl2 = scale * kLog2e;
  f32x16 Y[D / 32];
#pragma unroll
  for (int db = 0; db < D / 32; ++db) Y[db] = f32x16{};
  for (int k0 = 0; k0 < Lk; k0 += kRows) {
    stage_tile<T, D>(sk, Kb, st.k_srow, k0, Lk);
    stage_tile<T, D>(sv, Vb, st.v_srow, k0, Lk);
    __syncthreads();
    f32x16 S = f32x16{}, G = f32x16{};
    P::product1(S, sk, qf);  // S^T
    P::product1(G, sv, gf);  // dP^T
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float pv = (k0 + acc_row(r, h) < Lk) ? exp2f(S[r] * sl2 - lse2) : 0.f;
      S[r] = pv * (G[r] - dl);  // dS^T (without the softmax scale)
    }
    P::product2(Y, sk, S);
    __syncthreads();
  }
  store_Y<T, D>(Y, dQ + bh * st.q_sbh, st.q_srow, q0, Lq, scale);
}

// ----------------------------------------------------------------- dK/dV pass
template <typename T, int D>
__global__ __launch_bounds__(kThreads) void attn_dkv_kernel(const T *__restrict__ Q, const T *__restrict__ K,
                                                            const T *__restrict__ V, const T *__restrict__ dO,
                                                            const float *__restrict__ lse,
                                                            const float *__restrict__ delta, T *__restrict__ dK,
                                                            T *__restrict__ dV, int Lq, int Lk, float scale,
                                                            Strides st) {
  using P = Prec<T, D>;
  __shared__ __attribute__((aligned(16))) T sq[kRows * P::kStride];
  __shared__ __attribute__((aligned(16))) T sg[kRows * P::kStride];
  __shared__ float slse[kRows], sdl[kRows];
  const int bh = blockIdx.y;
  const int l = lane_(), h = l >> 5, w = threadIdx.x >> 6;
  const int k0w = blockIdx.x * (kWaves * 32) + w * 32;
  const int ki = k0w + (l & 31);
  const bool kv = ki < Lk;
  typename P::Frag kf, vf;
  P::load_frag(kf, K + bh * st.k_sbh + (long long)(kv ? ki : 0) * st.k_srow, kv);
  P::load_frag(vf, V + bh * st.v_sbh + (long long)(kv ? ki : 0) * st.v_srow, kv);
  const T *Qb = Q + bh * st.q_sbh;
  const T *Gb = dO + bh * st.o_sbh;
  const float sl2 = scale * kLog2e;
  f32x16 Y1[D / 32], Y2[D / 32];
#pragma unroll
  for (int db = 0; db < D / 32; ++db) {
    Y1[db] = f32x16{};
    Y2[db] = f32x16{};
  }
  for (int r0 = 0; r0 < Lq; r0 += kRows) {
    stage_tile<T, D>(sq, Qb, st.q_srow, r0, Lq);
    stage_tile<T, D>(sg, Gb, st.o_srow, r0, Lq);
    if (threadIdx.x < kRows) {
      const int q = r0 + threadIdx.x;
      slse[threadIdx.x] = q < Lq ? lse[(long long)bh * Lq + q] * kLog2e : INFINITY;
      sdl[threadIdx.x] = q < Lq ? delta[(long long)bh * Lq + q] : 0.f;
    }
    __syncthreads();
    f32x16 S = f32x16{}, G = f32x16{};
    P::product1(S, sq, kf);  // S  (queries x keys)
    P::product1(G, sg, vf);  // dP (queries x keys)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = acc_row(r, h);
      const float pv = exp2f(S[r] * sl2 - slse[row]);  // 0 for rows beyond Lq (lse = +inf)
      S[r] = pv;
      G[r] = pv * (G[r] - sdl[row]);
    }
    P::product2(Y1, sg, S);  // dV^T += dO^T P
    P::product2(Y2, sq, G);  // dK^T += Q^T dS
    __syncthreads();
  }
  store_Y<T, D>(Y1, dV + bh * st.v_sbh, st.v_srow, k0w, Lk, 1.f);
  store_Y<T, D>(Y2, dK + bh * st.k_sbh, st.k_srow, k0w, Lk, scale);
}

bool aligned_ok(const void *p, long long s_bh, long long s_row, int esize) {
  const int vec = 16 / esize;
  return ((uintptr_t)p % 16 == 0) && (s_bh % vec == 0) && (s_row % vec == 0);
}

template <typename T>
int launch_fwd(const void *q, const void *k, const void *v, void *o, float *lse, int BH, int Lq, int Lk, int D,
               float scale, const Strides &st, hipStream_t s) {
  const dim3 grid((Lq + kWaves * 32 - 1) / (kWaves * 32), BH);
#define ATT_FWD(DD)                                                                                           \
  case DD:                                                                                                    \
    hipLaunchKernelGGL((attn_fwd_kernel<T, DD>), grid, dim3(kThreads), 0, s, (const T *)q, (const T *)k,     \
                       (const T *)v, (T *)o, lse, Lq, Lk, scale, st);                                         \
    break;
  switch (D) {
    ATT_FWD(32)
    ATT_FWD(64)
    ATT_FWD(96)
    ATT_FWD(128)
    default:
      return PCOPS_ERR_UNSUPPORTED;
  }
#undef ATT_FWD
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

template <typename T>
int launch_delta(const void *o, const void *dout, float *delta, int BH, int Lq, int D, const Strides &st,
                 hipStream_t s) {
  const int rows = BH * Lq;
  hipLaunchKernelGGL((attn_delta_kernel<T>), dim3((rows + 3) / 4), dim3(256), 0, s, (const T *)o, (const T *)dout,
                     delta, BH, Lq, D, st);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

template <typename T>
int launch_dq(const void *q, const void *k, const void *v, const void *dout, const float *lse, const float *delta,
              void *dq, int BH, int Lq, int Lk, int D, float scale, const Strides &st, hipStream_t s) {
  const dim3 gq((Lq + kWaves * 32 - 1) / (kWaves * 32), BH);
#define ATT_DQ(DD)                                                                                              \
  case DD:                                                                                                      \
    hipLaunchKernelGGL((attn_dq_kernel<T, DD>), gq, dim3(kThreads), 0, s, (const T *)q, (const T *)k,           \
                       (const T *)v, (const T *)dout, lse, delta, (T *)dq, Lq, Lk, scale, st);                  \
    break;
  switch (D) {
    ATT_DQ(32)
    ATT_DQ(64)
    ATT_DQ(96)
    ATT_DQ(128)
    default:
      return PCOPS_ERR_UNSUPPORTED;
  }
#undef ATT_DQ
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

template <typename T>
int launch_dkv(const void *q, const void *k, const void *v, const void *dout, const float *lse, const float *delta,
               void *dk, void *dv, int BH, int Lq, int Lk, int D, float scale, const Strides &st, hipStream_t s) {
  const dim3 gk((Lk + kWaves * 32 - 1) / (kWaves * 32), BH);
#define ATT_DKV(DD)                                                                                             \
  case DD:                                                                                                      \
    hipLaunchKernelGGL((attn_dkv_kernel<T, DD>), gk, dim3(kThreads), 0, s, (const T *)q, (const T *)k,          \
                       (const T *)v, (const T *)dout, lse, delta, (T *)dk, (T *)dv, Lq, Lk, scale, st);         \
    break;
  switch (D) {
    ATT_DKV(32)
    ATT_DKV(64)
    ATT_DKV(96)
    ATT_DKV(128)
    default:
      return PCOPS_ERR_UNSUPPORTED;
  }
#undef ATT_DKV
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

int check_common(int BH, int Lq, int Lk, int D, int dtype) {
  if (BH < 0 || Lq < 0 || Lk < 0) return PCOPS_ERR_INVALID;
  if (D % 32 != 0 || D <= 0 || D > 128 || (dtype != 0 && dtype != 1)) return PCOPS_ERR_UNSUPPORTED;
  return PCOPS_OK;
}

}  // namespace

extern "C" int pcops_attention_forward(const void *q, const void *k, const void *v, void *o, float *lse, int BH,
                                       int Lq, int Lk, int D, float scale, int dtype, long long q_sbh,
                                       long long q_srow, long long k_sbh, long long k_srow, long long v_sbh,
                                       long long v_srow, long long o_sbh, long long o_srow, pcops_stream_t stream) {
  if (BH < 0 || Lq < 0 || Lk < 0) return PCOPS_ERR_INVALID;
  if (BH == 0 || Lq == 0) return PCOPS_OK;
  if (Lk <= 0 || !q || !k || !v || !o) return PCOPS_ERR_INVALID;
  if (D % 32 != 0 || D > 128 || (dtype != 0 && dtype != 1)) return PCOPS_ERR_UNSUPPORTED;
  const int es = dtype == 0 ? 4 : 2;
  if (!aligned_ok(q, q_sbh, q_srow, es) || !aligned_ok(k, k_sbh, k_srow, es) || !aligned_ok(v, v_sbh, v_srow, es) ||
      !aligned_ok(o, o_sbh, o_srow, es))
    return PCOPS_ERR_UNSUPPORTED;
  const Strides st{q_sbh, q_srow, k_sbh, k_srow, v_sbh, v_srow, o_sbh, o_srow};
  hipStream_t s = (hipStream_t)stream;
  return dtype == 0 ? launch_fwd<float>(q, k, v, o, lse, BH, Lq, Lk, D, scale, st, s)
                    : launch_fwd<__bf16>(q, k, v, o, lse, BH, Lq, Lk, D, scale, st, s);
}

extern "C" unsigned long long pcops_attention_bwd_workspace_bytes(int BH, int Lq, int Lk, int D) {
  (void)Lk;
  (void)D;
  if (BH <= 0 || Lq <= 0) return 0;
  return (unsigned long long)BH * Lq * sizeof(float);
}

extern "C" int pcops_attention_bwd_preprocess(const void *o, const void *dout, int BH, int Lq, int D, int dtype,
                                              long long o_sbh, long long o_srow, void *workspace,
                                              unsigned long long workspace_bytes, pcops_stream_t stream) {
  int rc = check_common(BH, Lq, 1, D, dtype);
  if (rc) return rc;
  if (BH == 0 || Lq == 0) return PCOPS_OK;
  if (!o || !dout) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_attention_bwd_workspace_bytes(BH, Lq, 1, D)) return PCOPS_ERR_WORKSPACE;
  const Strides st{0, 0, 0, 0, 0, 0, o_sbh, o_srow};
  hipStream_t s = (hipStream_t)stream;
  return dtype == 0 ? launch_delta<float>(o, dout, (float *)workspace, BH, Lq, D, st, s)
                    : launch_delta<__bf16>(o, dout, (float *)workspace, BH, Lq, D, st, s);
}

extern "C" int pcops_attention_bwd_dq(const void *q, const void *k, const void *v, const void *dout, const float *lse,
                                      void *dq, int BH, int Lq, int Lk, int D, float scale, int dtype,
                                      long long q_sbh, long long q_srow, long long k_sbh, long long k_srow,
                                      long long v_sbh, long long v_srow, long long o_sbh, long long o_srow,
                                      const void *workspace, unsigned long long workspace_bytes,
                                      pcops_stream_t stream) {
  int rc = check_common(BH, Lq, Lk, D, dtype);
  if (rc) return rc;
  if (BH == 0 || Lq == 0) return PCOPS_OK;
  if (!q || !k || !v || !dout || !lse || !dq || Lk <= 0) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_attention_bwd_workspace_bytes(BH, Lq, Lk, D)) return PCOPS_ERR_WORKSPACE;
  const int es = dtype == 0 ? 4 : 2;
  if (!aligned_ok(q, q_sbh, q_srow, es) || !aligned_ok(k, k_sbh, k_srow, es) || !aligned_ok(v, v_sbh, v_srow, es) ||
      !aligned_ok(dout, o_sbh, o_srow, es) || !aligned_ok(dq, q_sbh, q_srow, es))
    return PCOPS_ERR_UNSUPPORTED;
  const Strides st{q_sbh, q_srow, k_sbh, k_srow, v_sbh, v_srow, o_sbh, o_srow};
  hipStream_t s = (hipStream_t)stream;
  const float *delta = (const float *)workspace;
  return dtype == 0 ? launch_dq<float>(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, D, scale, st, s)
                    : launch_dq<__bf16>(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, D, scale, st, s);
}

extern "C" int pcops_attention_bwd_dkv(const void *q, const void *k, const void *v, const void *dout,
                                       const float *lse, void *dk, void *dv, int BH, int Lq, int Lk, int D,
                                       float scale, int dtype, long long q_sbh, long long q_srow, long long k_sbh,
                                       long long k_srow, long long v_sbh, long long v_srow, long long o_sbh,
                                       long long o_srow, const void *workspace, unsigned long long workspace_bytes,
                                       pcops_stream_t stream) {
  int rc = check_common(BH, Lq, Lk, D, dtype);
  if (rc) return rc;
  if (BH == 0 || Lk == 0) return PCOPS_OK;
  if (!q || !k || !v || !dout || !lse || !dk || !dv || Lq <= 0) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_attention_bwd_workspace_bytes(BH, Lq, Lk, D)) return PCOPS_ERR_WORKSPACE;
  const int es = dtype == 0 ? 4 : 2;
  if (!aligned_ok(q, q_sbh, q_srow, es) || !aligned_ok(k, k_sbh, k_srow, es) || !aligned_ok(v, v_sbh, v_srow, es) ||
      !aligned_ok(dout, o_sbh, o_srow, es) || !aligned_ok(dk, k_sbh, k_srow, es) || !aligned_ok(dv, v_sbh, v_srow, es))
    return PCOPS_ERR_UNSUPPORTED;
  const Strides st{q_sbh, q_srow, k_sbh, k_srow, v_sbh, v_srow, o_sbh, o_srow};
  hipStream_t s = (hipStream_t)stream;
  const float *delta = (const float *)workspace;
  return dtype == 0 ? launch_dkv<float>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, D, scale, st, s)
                    : launch_dkv<__bf16>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, D, scale, st, s);
}

// dq/dk/dv use the q/k/v strides; dout uses the o strides.
extern "C" int pcops_attention_backward(const void *q, const void *k, const void *v, const void *o, const void *dout,
                                        const float *lse, void *dq, void *dk, void *dv, int BH, int Lq, int Lk, int D,
                                        float scale, int dtype, long long q_sbh, long long q_srow, long long k_sbh,
                                        long long k_srow, long long v_sbh, long long v_srow, long long o_sbh,
                                        long long o_srow, void *workspace, unsigned long long workspace_bytes,
                                        pcops_stream_t stream) {
  if (BH == 0 || Lq == 0 || Lk == 0) return check_common(BH, Lq, Lk, D, dtype);
  const int es = dtype == 0 ? 4 : 2;
  if (o && !aligned_ok(o, o_sbh, o_srow, es)) return PCOPS_ERR_UNSUPPORTED;
  int rc = pcops_attention_bwd_preprocess(o, dout, BH, Lq, D, dtype, o_sbh, o_srow, workspace, workspace_bytes, stream);
  if (rc) return rc;
  rc = pcops_attention_bwd_dq(q, k, v, dout, lse, dq, BH, Lq, Lk, D, scale, dtype, q_sbh, q_srow, k_sbh, k_srow, v_sbh,
                              v_srow, o_sbh, o_srow, workspace, workspace_bytes, stream);
  if (rc) return rc;
  return pcops_attention_bwd_dkv(q, k, v, dout, lse, dk, dv, BH, Lq, Lk, D, scale, dtype, q_sbh, q_srow, k_sbh, k_srow,
                                 v_sbh, v_srow, o_sbh, o_srow, workspace, workspace_bytes, stream);
}
