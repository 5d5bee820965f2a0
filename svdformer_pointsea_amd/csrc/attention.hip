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
#include <cstdlib>

#include <type_traits>

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

// Column sums of a wave's stored tile Y (D x 32 entities) over its entities, as
// stored (bf16(Y * mul)), entities >= L counting 0: the in_proj bias gradient of
// the projection whose output this gradient is (its column sums over all rows),
// formed here instead of by a separate pass over the packed q/k/v gradient.
// Reduce-scatter over the 32 entity lanes of each half: every step halves the
// values a lane holds and pairs it with a lane differing in one more bit --
// v_permlane16_swap (bit 4: one swap + one add per two values), then DPP
// row_ror:8 (bit 3), row_half_mirror (bit 2, pairs l with l ^ 7), quad_perm
// xor 2 (bit 1), each keeping the half selected by the lane's own bit, and
// quad_perm xor 1 for the last value: 38 VALU ops per 16 values instead of a
// 6-op wave sum for each.  Lane l ends with value j = 8 b4 + 4 b3 + 2 b2 + b1
// (its bits), summed over its half's 32 entities; the even lanes write it.
template <int CTRL>
__device__ __forceinline__ float dpp_(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ float keep_send_(float lo, float hi, bool bit) {
  const float keep = bit ? hi : lo, send = bit ? lo : hi;
  return keep + dpp_<CTRL>(send);
}
template <int D>
__device__ __forceinline__ void colsum_wave(const f32x16 (&Y)[D / 32], float mul, bool valid, float *sc, int w) {
  const int l = lane_(), h = l >> 5;
  const bool b3 = l & 8, b2 = l & 4, b1 = l & 2;
  float r[D / 32];
#pragma unroll
  for (int db = 0; db < D / 32; ++db) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = valid ? (float)(__bf16)(Y[db][j] * mul) : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // bit 4: rows 0/2 keep v[j], rows 1/3 keep v[j + 8]
      const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[j]), __float_as_uint(v[j + 8]), false, false);
      v[j] = __uint_as_float(p[0]) + __uint_as_float(p[1]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = keep_send_<0x128>(v[j], v[j + 4], b3);
#pragma unroll
    for (int j = 0; j < 2; ++j) v[j] = keep_send_<0x141>(v[j], v[j + 2], b2);
    v[0] = keep_send_<0x4E>(v[0], v[1], b1);
    r[db] = v[0] + dpp_<0xB1>(v[0]);
  }
  if ((l & 1) == 0) {
    const int j = ((l >> 4) & 1) * 8 + (b3 ? 4 : 0) + (b2 ? 2 : 0) + (b1 ? 1 : 0);
    const int d0 = 8 * (j >> 2) + 4 * h + (j & 3);
#pragma unroll
    for (int db = 0; db < D / 32; ++db) sc[w * D + db * 32 + d0] = r[db];
  }
}

// the partial row of block (bh, rb): row b * nrb + rb, columns h * D .. h * D + D - 1 of a
// (B * nrb, H * D) array, so the final sum is a plain column sum over its rows
__device__ __forceinline__ long long colsum_row(int bh, int rb, int H, int D) {
  const int b = bh / H, h = bh - b * H;
  return ((long long)(b * (int)gridDim.x + rb) * H + h) * D;
}

// after colsum_wave in every wave and a barrier: part_row[d] = sum over the NW waves in order
template <int D, int NW>
__device__ __forceinline__ void colsum_block(const float *sc, float *part_row) {
  for (int d = threadIdx.x; d < D; d += NW * 64) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += sc[w * D + d];
    part_row[d] = t;
  }
}

// Element (b, h, row, d) of a tensor lives at b*sb + h*sh + row*srow + d, so
// seq-first (L, B, H*hd) [sb = H*hd, sh = hd, srow = B*H*hd] and batch-first
// (B, L, H*hd) [sb = L*H*hd, sh = hd, srow = H*hd] layouts are both read in place.
struct Strides {
  long long q_sb, q_sh, q_srow, k_sb, k_sh, k_srow, v_sb, v_sh, v_srow, o_sb, o_sh, o_srow;
  int H;
  __device__ __forceinline__ long long q_off(int bh) const { return (long long)(bh / H) * q_sb + (long long)(bh % H) * q_sh; }
  __device__ __forceinline__ long long k_off(int bh) const { return (long long)(bh / H) * k_sb + (long long)(bh % H) * k_sh; }
  __device__ __forceinline__ long long v_off(int bh) const { return (long long)(bh / H) * v_sb + (long long)(bh % H) * v_sh; }
  __device__ __forceinline__ long long o_off(int bh) const { return (long long)(bh / H) * o_sb + (long long)(bh % H) * o_sh; }
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
  P::load_frag(qf, Q + st.q_off(bh) + (long long)(qi < Lq ? qi : 0) * st.q_srow, qi < Lq);
  const T *Kb = K + st.k_off(bh);
  const T *Vb = V + st.v_off(bh);
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
  store_Y<T, D>(Y, O + st.o_off(bh), st.o_srow, q0, Lq, 1.f / lsum);
  if (h == 0 && qi < Lq && lse) lse[(long long)bh * Lq + qi] = (m + log2f(lsum)) * kLn2;
}

// delta[bh][q] = sum_d dO[q][d] * O[q][d]  (one wave per row)
template <typename T>
__global__ void attn_delta_kernel(const T *__restrict__ O, const T *__restrict__ dO, float *__restrict__ delta,
                                  int BH, int Lq, int D, Strides st) {
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= BH * Lq) return;
  const int bh = row / Lq, q = row - bh * Lq;
  const T *o = O + st.o_off(bh) + (long long)q * st.o_srow;
  const T *g = dO + st.o_off(bh) + (long long)q * st.o_srow;
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
  P::load_frag(qf, Q + st.q_off(bh) + (long long)(qv ? qi : 0) * st.q_srow, qv);
  P::load_frag(gf, dO + st.o_off(bh) + (long long)(qv ? qi : 0) * st.o_srow, qv);
  const float lse2 = qv ? lse[(long long)bh * Lq + qi] * kLog2e : INFINITY;
  const float dl = qv ? delta[(long long)bh * Lq + qi] : 0.f;
  const T *Kb = K + st.k_off(bh);
  const T *Vb = V + st.v_off(bh);
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
  store_Y<T, D>(Y, dQ + st.q_off(bh), st.q_srow, q0, Lq, scale);
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
  P::load_frag(kf, K + st.k_off(bh) + (long long)(kv ? ki : 0) * st.k_srow, kv);
  P::load_frag(vf, V + st.v_off(bh) + (long long)(kv ? ki : 0) * st.v_srow, kv);
  const T *Qb = Q + st.q_off(bh);
  const T *Gb = dO + st.o_off(bh);
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
  store_Y<T, D>(Y1, dV + st.v_off(bh), st.v_srow, k0w, Lk, 1.f);
  store_Y<T, D>(Y2, dK + st.k_off(bh), st.k_srow, k0w, Lk, scale);
}

// ----------------------------------------------------------------- forward, bf16 (v2)
// NW waves x 32 queries per block; 64-key K/V tiles double-buffered in LDS
// (dynamic), the next tile prefetched into registers while the current one
// is on the matrix cores; one barrier per tile.  Half-wave exchange by
// v_permlane32_swap; the softmax scale folded into the exp2 argument (fma).
constexpr int kKT = 64;  // keys per tile
#ifndef PCOPS_SCHED_DS
#define PCOPS_SCHED_DS 1
#endif
constexpr bool kSchedDs = PCOPS_SCHED_DS;  // 0: compiler's own LDS/MFMA order (A/B builds)
#ifndef PCOPS_DQ_A
#define PCOPS_DQ_A 2  // dQ pass (two-half form): LDS reads issued this many MFMAs ahead; 0 = plain chains (A/B)
#endif
#ifndef PCOPS_DEFER_LOG2
#define PCOPS_DEFER_LOG2 8.f  // 0 = rescale on every max increase (A/B builds)
#endif
constexpr float kDeferLog2 = PCOPS_DEFER_LOG2;  // forward: rescale only when a row max grows by > 2^8

// v_exp_f32 directly: exp2f's library form wraps it in a denormal-range
// rescale (cmp + 2 cndmask + add + ldexp: 6 VALU per probability, 40 % of the
// forward loop's VALU).  A probability below 2^-126 of its row maximum is
// flushed to 0 instead -- invisible in bf16 P (and in any fp32 sum of them).
__device__ __forceinline__ float exp2_ftz(float x) { return __builtin_amdgcn_exp2f(x); }

// Row max of two 32x32 accumulator tiles as 8 + 7 v_max3_f32 (fmaxf on MFMA
// results makes the compiler canonicalise each operand first: a v_max x, x
// per score, IEEE mode).  The operands are MFMA results, and the hazard
// recognizer does not look inside inline asm: a VALU read of a VGPR written
// by a 16-pass XDL op needs ~18 wait states on gfx950 that nothing would
// insert.  Without them v_max3 read accumulators the MFMA had not finished
// writing (round 3: the 8-wave forward's output differed run to run in the
// last bf16 bit -- the stale max only shifts the exp reference -- and a max
// read far too low can overflow exp2 to inf).  Three s_nop 7 (24 wait states)
// open the first block; the second follows it (volatile order, data chain).
__device__ __forceinline__ float tile_max16(const f32x16 &a, const f32x16 &b) {
  float r;
  asm volatile(
      "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"
      "v_max3_f32 %0, %1, %2, %3\n\t"
      "v_max3_f32 %0, %0, %4, %5\n\t"
      "v_max3_f32 %0, %0, %6, %7\n\t"
      "v_max3_f32 %0, %0, %8, %9\n\t"
      "v_max3_f32 %0, %0, %10, %11\n\t"
      "v_max3_f32 %0, %0, %12, %13\n\t"
      "v_max3_f32 %0, %0, %14, %15\n\t"
      "v_max_f32 %0, %0, %16"
      : "=&v"(r)
      : "v"(a[0]), "v"(b[0]), "v"(a[1]), "v"(b[1]), "v"(a[2]), "v"(b[2]), "v"(a[3]), "v"(b[3]), "v"(a[4]), "v"(b[4]),
        "v"(a[5]), "v"(b[5]), "v"(a[6]), "v"(b[6]), "v"(a[7]), "v"(b[7]));
  asm volatile(
      "v_max3_f32 %0, %0, %1, %2\n\t"
      "v_max3_f32 %0, %0, %3, %4\n\t"
      "v_max3_f32 %0, %0, %5, %6\n\t"
      "v_max3_f32 %0, %0, %7, %8\n\t"
      "v_max3_f32 %0, %0, %9, %10\n\t"
      "v_max3_f32 %0, %0, %11, %12\n\t"
      "v_max3_f32 %0, %0, %13, %14\n\t"
      "v_max3_f32 %0, %0, %15, %16"
      : "+v"(r)
      : "v"(a[8]), "v"(b[8]), "v"(a[9]), "v"(b[9]), "v"(a[10]), "v"(b[10]), "v"(a[11]), "v"(b[11]), "v"(a[12]),
        "v"(b[12]), "v"(a[13]), "v"(b[13]), "v"(a[14]), "v"(b[14]), "v"(a[15]), "v"(b[15]));
  return r;
}

__device__ __forceinline__ float swap_halves_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float swap_halves_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// LDS tile image of the v2 kernels: rows of RS bf16 whose 16-B chunks are
// XOR-permuted per row (chunk ch of row r sits at chunk ch ^ f(r)), so that
// BOTH reads of a tile are bank-conflict free on gfx950: the row reads of
// k_product (ds_read_b128, 4 x 16-lane groups) and the transposed reads of
// v_product (ds_read_b64_tr_b16, 2 x 32-lane groups).  f depends on row bits
// 0..3 only, so a tile's second 32-row half uses the same f.  The maps were
// found and are checked by tools/lds_banks.py (a plain D+8 pad made the
// transposed reads 2-4 way conflicted: 14 % of dK/dV wave cycles).
template <int D>
struct Img;
template <>
struct Img<32> {
  static constexpr int RS = 40;
  __device__ static constexpr int f(int) { return 0; }
};
template <>
struct Img<64> {
  static constexpr int RS = 64;
  __device__ static constexpr int f(int r) { return ((r & 3) << 1) ^ ((r >> 2) & 3); }
};
template <>
struct Img<96> {
  static constexpr int RS = 96;
  __device__ static constexpr int f(int r) { return (r & 1) ^ ((r >> 2) & 3); }
};
template <>
struct Img<128> {
  static constexpr int RS = 128;
  __device__ static constexpr int f(int r) { return ((r & 3) << 2) ^ ((r >> 2) & 3); }
};

// element (row, 8*ch + e) of an Img<D> tile
template <int D>
__device__ __forceinline__ int img_off(int row, int ch) {
  return row * Img<D>::RS + 8 * (ch ^ Img<D>::f(row));
}

// acc += Rows(32 x D, Img<D> tile) . Ent   (entity fragment f)
template <int D>
__device__ __forceinline__ void k_product(f32x16 &acc, const __bf16 *lds, const bf16x8 (&f)[D / 16]) {
  const int l = lane_(), h = l >> 5, row = l & 31;
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    const bf16x8 a = *reinterpret_cast<const bf16x8 *>(lds + img_off<D>(row, 2 * s + h));
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, f[s], acc, 0, 0, 0);
  }
}

// two independent chains interleaved (acc0 over lds0 . f0, acc1 over lds1 . f1):
// consecutive MFMAs never wait on each other; each accumulator's order is
// k_product's
template <int D>
__device__ __forceinline__ void k_product2(f32x16 &acc0, const __bf16 *lds0, const bf16x8 (&f0)[D / 16],
                                           f32x16 &acc1, const __bf16 *lds1, const bf16x8 (&f1)[D / 16]) {
  const int l = lane_(), h = l >> 5, row = l & 31;
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    const bf16x8 a0 = *reinterpret_cast<const bf16x8 *>(lds0 + img_off<D>(row, 2 * s + h));
    const bf16x8 a1 = *reinterpret_cast<const bf16x8 *>(lds1 + img_off<D>(row, 2 * s + h));
    acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, f0[s], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, f1[s], acc1, 0, 0, 0);
  }
}

// Scheduling shape of an LDS-fed MFMA sequence of N MFMAs with R ds_reads
// each: the first A MFMAs' reads go out first, then every MFMA is followed by
// the reads of the MFMA A places later -- each read has A MFMAs (>= 64
// cycles) to land instead of the compiler's read-wait-MFMA (lgkmcnt(0)
// before every MFMA: the LDS latency exposed once per MFMA).
template <int N, int R, int A>
__device__ __forceinline__ void sched_ds_mfma() {
  __builtin_amdgcn_sched_group_barrier(0x100, A * R, 0);
#pragma unroll
  for (int i = 0; i < N - A; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, R, 0);
  }
  __builtin_amdgcn_sched_group_barrier(0x008, A, 0);
}

// Y[db] += Rows^T(D x 32, Img<D> tile) . X   (X = fp32 accumulator of 32 rows)
template <int D>
__device__ __forceinline__ void v_product(f32x16 (&Y)[D / 32], const __bf16 *lds, const f32x16 &X) {
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
      const int ch = 4 * db + 2 * g + (p >> 1), e = 4 * (p & 1);
      const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(lds + img_off<D>(row0, ch) + e));
      const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(lds + img_off<D>(row0 + 8, ch) + e));
      const bf16x8 a = __builtin_shufflevector(__builtin_bit_cast(bf16x4, lo), __builtin_bit_cast(bf16x4, hi), 0, 1,
                                               2, 3, 4, 5, 6, 7);
      Y[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, Y[db], 0, 0, 0);
    }
  }
#endif
}

// XCD-aware block order: the hardware hands consecutive workgroups to the 8
// XCDs round-robin, so the row blocks of one (batch, head) would land on 8
// different L2s and fetch that head's K/V (or Q/dO) 8 times.  Remap the
// linear id so each XCD gets a contiguous range of (head, row-block) pairs.
__device__ __forceinline__ void xcd_block(int &rb, int &bh) {
  const int nrb = gridDim.x, total = gridDim.x * gridDim.y;
  int L = blockIdx.x + nrb * blockIdx.y;
  if ((total & 7) == 0) L = (L & 7) * (total >> 3) + (L >> 3);
  rb = L % nrb;
  bh = L / nrb;
}

// Occupancy of the backward passes.  dQ (template OCC): 2 waves per SIMD for
// D <= 96 (D=96 0.093 -> 0.060 ms at the PCN shapes), 1 for D = 128 (its
// 256-register form spills).  dK/dV: see attn_dkv2_kernel's MODE.

template <int D, int NW>
struct Fwd2Cfg {
  static constexpr int kThr = NW * 64;
  static constexpr int kKS = Img<D>::RS;            // tile row stride (both tiles: Img<D>)
  static constexpr int kVS = Img<D>::RS;
  static constexpr int kChunks = kKT * D / 8;       // 16-B chunks per tile
  static constexpr int kCPT = (kChunks + kThr - 1) / kThr;
  static constexpr int kKBuf = kKT * kKS, kVBuf = kKT * kVS;
  static constexpr size_t kLds = 2ull * (kKBuf + kVBuf) * sizeof(__bf16);
  typedef bf16x8 Regs[kCPT];
};

// FAST: the full-tile form with one 32-bit offset per tensor (fewer VALU per load, but its
// loop-invariant offsets cost registers): measured per kernel (profiles/r6_attn_lib_ab.txt) --
// 1.5 % faster for the dK/dV pass (dkv2), slower for the hd-128 forward (+13 %) and dQ, a
// wash for the hd-64 forward (which then reloaded two spilled offsets from scratch per tile)
template <int D, int NW, bool FAST = false>
__device__ __forceinline__ void fwd2_load(typename Fwd2Cfg<D, NW>::Regs &kr, typename Fwd2Cfg<D, NW>::Regs &vr,
                                          const __bf16 *Kb, long long ks, const __bf16 *Vb, long long vs, int k0,
                                          int Lk) {
  using C = Fwd2Cfg<D, NW>;
  constexpr int RB = C::kThr % (D / 8) == 0 ? C::kThr / (D / 8) : 0;  // rows per pass of the block
  if (FAST && RB && C::kChunks % C::kThr == 0 && k0 + kKT <= Lk) {
    // a full tile: chunk t of the thread is row row0 + t RB at one column -- one unsigned 32-bit
    // offset per tensor and a wave-uniform 64-bit row base per chunk (the per-chunk 64-bit multiply
    // of the general form below cost ~10 VALU per load)
    const unsigned tid = threadIdx.x, row0 = tid / (D / 8), col = (tid % (D / 8)) * 8;
    const unsigned ok_ = row0 * (unsigned)ks + col, ov = row0 * (unsigned)vs + col;
#pragma unroll
    for (int t = 0; t < C::kCPT; ++t) {
      kr[t] = *reinterpret_cast<const bf16x8 *>(Kb + (long long)(k0 + t * RB) * ks + ok_);
      vr[t] = *reinterpret_cast<const bf16x8 *>(Vb + (long long)(k0 + t * RB) * vs + ov);
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < C::kCPT; ++t) {
    const int c = threadIdx.x + t * C::kThr;
    const int row = c / (D / 8), ch = c % (D / 8);
    const bool ok = (C::kChunks % C::kThr == 0 || c < C::kChunks) && k0 + row < Lk;
    kr[t] = ok ? *reinterpret_cast<const bf16x8 *>(Kb + (long long)(k0 + row) * ks + ch * 8) : bf16x8{};
    vr[t] = ok ? *reinterpret_cast<const bf16x8 *>(Vb + (long long)(k0 + row) * vs + ch * 8) : bf16x8{};
  }
}

template <int D, int NW, bool FAST = false>
__device__ __forceinline__ void fwd2_store(__bf16 *sk, __bf16 *sv, const typename Fwd2Cfg<D, NW>::Regs &kr,
                                           const typename Fwd2Cfg<D, NW>::Regs &vr) {
  using C = Fwd2Cfg<D, NW>;
  constexpr int RB = C::kThr % (D / 8) == 0 ? C::kThr / (D / 8) : 0;
  if constexpr (FAST && RB && RB % 16 == 0 && C::kChunks % C::kThr == 0) {
    // Img<D>'s permutation reads row bits 0..3: rows row0 + t RB share it (immediate offsets)
    const unsigned tid = threadIdx.x, row0 = tid / (D / 8), ch = tid % (D / 8);
    const unsigned so = (unsigned)img_off<D>((int)row0, (int)ch);
#pragma unroll
    for (int t = 0; t < C::kCPT; ++t) {
      *reinterpret_cast<bf16x8 *>(sk + so + t * RB * C::kKS) = kr[t];
      *reinterpret_cast<bf16x8 *>(sv + so + t * RB * C::kVS) = vr[t];
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < C::kCPT; ++t) {
    const int c = threadIdx.x + t * C::kThr;
    if (C::kChunks % C::kThr != 0 && c >= C::kChunks) continue;
    const int row = c / (D / 8), ch = c % (D / 8);
    *reinterpret_cast<bf16x8 *>(sk + img_off<D>(row, ch)) = kr[t];
    *reinterpret_cast<bf16x8 *>(sv + img_off<D>(row, ch)) = vr[t];
  }
}

template <int D, int NW, int OCC>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(OCC))) void attn_fwd2_kernel(const __bf16 *__restrict__ Q, const __bf16 *__restrict__ K,
                                                            const __bf16 *__restrict__ V, __bf16 *__restrict__ O,
                                                            float *__restrict__ lse, int Lq, int Lk, float scale,
                                                            Strides st) {
  using C = Fwd2Cfg<D, NW>;
  extern __shared__ __attribute__((aligned(16))) unsigned char fwd2_smem[];
  __bf16 *sk = reinterpret_cast<__bf16 *>(fwd2_smem);
  __bf16 *sv = sk + 2 * C::kKBuf;
  int rb, bh;
  xcd_block(rb, bh);
  const int l = lane_(), h = l >> 5, w = threadIdx.x >> 6;
  const int q0 = rb * (NW * 32) + w * 32;
  const int qi = q0 + (l & 31);
  bf16x8 qf[D / 16];
  {
    const __bf16 *row = Q + st.q_off(bh) + (long long)(qi < Lq ? qi : 0) * st.q_srow + 8 * h;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) qf[s] = qi < Lq ? *reinterpret_cast<const bf16x8 *>(row + 16 * s) : bf16x8{};
  }
  const __bf16 *Kb = K + st.k_off(bh);
  const __bf16 *Vb = V + st.v_off(bh);
  const float sl2 = scale * kLog2e;
  float m = -INFINITY, lsum = 0.f;
  f32x16 Y[D / 32];
#pragma unroll
  for (int db = 0; db < D / 32; ++db) Y[db] = f32x16{};
  typename C::Regs kr, vr;
  fwd2_load<D, NW>(kr, vr, Kb, st.k_srow, Vb, st.v_srow, 0, Lk);
  fwd2_store<D, NW>(sk, sv, kr, vr);
  lds_barrier();
  const int ntiles = (Lk + kKT - 1) / kKT;
  // one tile; EDGE: the last, partial tile (key masking), compiled separately
  // so full tiles carry no per-score mask selects
  auto tile = [&](int t, auto edge_c) {
    constexpr bool EDGE = decltype(edge_c)::value;
    const int cur = t & 1;
    const int k0 = t * kKT;
    if (t + 1 < ntiles) fwd2_load<D, NW>(kr, vr, Kb, st.k_srow, Vb, st.v_srow, k0 + kKT, Lk);
    const __bf16 *ck = sk + cur * C::kKBuf;
    const __bf16 *cv = sv + cur * C::kVBuf;
    f32x16 X0 = f32x16{}, X1 = f32x16{};
    k_product2<D>(X0, ck, qf, X1, ck + 32 * C::kKS, qf);
    if constexpr (kSchedDs) sched_ds_mfma<D / 8, 1, 2>();
    if constexpr (EDGE) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (k0 + acc_row(r, h) >= Lk) X0[r] = -INFINITY;
        if (k0 + 32 + acc_row(r, h) >= Lk) X1[r] = -INFINITY;
      }
    }
    float tmax = tile_max16(X0, X1);
    tmax = swap_halves_max(tmax);
    // deferred max (guide T13): while no row's tile max exceeds its running
    // max by more than kDeferLog2 (P <= 2^8), keep m and skip the O rescale;
    // the decision is wave-uniform and taken before this tile's P exists
    const float pm = tmax * sl2;
    const bool keep = __all(pm - m <= kDeferLog2);
    const float mn = keep ? m : fmaxf(m, pm);
    const float alpha = keep ? 1.f : exp2_ftz(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      X0[r] = exp2_ftz(__builtin_fmaf(X0[r], sl2, -mn));
      X1[r] = exp2_ftz(__builtin_fmaf(X1[r], sl2, -mn));
      rs += X0[r] + X1[r];
    }
    rs = swap_halves_sum(rs);
    lsum = lsum * alpha + rs;
    m = mn;
    if (!keep) {
#pragma unroll
      for (int db = 0; db < D / 32; ++db) Y[db] *= alpha;
    }
    v_product<D>(Y, cv, X0);
    v_product<D>(Y, cv + 32 * C::kVS, X1);
    if constexpr (kSchedDs) sched_ds_mfma<D / 8, 2, (OCC >= 4 ? 1 : 2)>();
    if (t + 1 < ntiles) fwd2_store<D, NW>(sk + (cur ^ 1) * C::kKBuf, sv + (cur ^ 1) * C::kVBuf, kr, vr);
    lds_barrier();
  };
  const int nfull = Lk / kKT;
  for (int t = 0; t < nfull; ++t) tile(t, std::false_type{});
  if (nfull < ntiles) tile(nfull, std::true_type{});
  store_Y<__bf16, D>(Y, O + st.o_off(bh), st.o_srow, q0, Lq, 1.f / lsum);
  if (h == 0 && qi < Lq && lse) lse[(long long)bh * Lq + qi] = (m + log2f(lsum)) * kLn2;
}

int env_int(const char *name, int dflt) {
  const char *e = getenv(name);
  return e ? atoi(e) : dflt;
}

template <int D, int NW, int OCC>
int launch_fwd2_occ(const void *q, const void *k, const void *v, void *o, float *lse, int BH, int Lq, int Lk,
                    float scale, const Strides &st, hipStream_t s) {
  using C = Fwd2Cfg<D, NW>;
  static const hipError_t attr = hipFuncSetAttribute((const void *)attn_fwd2_kernel<D, NW, OCC>,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)C::kLds);
  if (attr != hipSuccess) return PCOPS_ERR_LAUNCH;
  const dim3 grid((Lq + NW * 32 - 1) / (NW * 32), BH);
  hipLaunchKernelGGL((attn_fwd2_kernel<D, NW, OCC>), grid, dim3(C::kThr), C::kLds, s, (const __bf16 *)q,
                     (const __bf16 *)k, (const __bf16 *)v, (__bf16 *)o, lse, Lq, Lk, scale, st);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

// Occupancy: 8-wave blocks at <= 128 VGPRs run 2 blocks per CU instead of
// one (130 -> 128 for D = 64: 0.466 -> 0.379 ms at (2048, 2048, B*H = 256)).
// D = 128 needs ~200 (Y alone is 64).  PCOPS_FWD_OCC=1 lifts the cap (A/B).
// 4-wave blocks (short sequences) are capped at 2 waves per SIMD: left
// alone the compiler gives them 400+ registers (one wave per SIMD).
template <int D, int NW>
int launch_fwd2(const void *q, const void *k, const void *v, void *o, float *lse, int BH, int Lq, int Lk, float scale,
                const Strides &st, hipStream_t s) {
  static const int occ = env_int("PCOPS_FWD_OCC", 4);
  if constexpr (D <= 64 && NW == 8) {
    if (occ == 4) return launch_fwd2_occ<D, NW, 4>(q, k, v, o, lse, BH, Lq, Lk, scale, st, s);
  }
  // D = 96 runs 4-wave blocks at any length (201 VGPRs: two independent
  // blocks per CU beat one 8-wave block at 185, 512^2 0.052 -> 0.047 ms);
  // D = 128 does not (2048^2 0.644 -> 0.719 ms)
  if constexpr (NW == 4 || D == 96) {
    return launch_fwd2_occ<D, 4, 2>(q, k, v, o, lse, BH, Lq, Lk, scale, st, s);
  } else {
    return launch_fwd2_occ<D, NW, 1>(q, k, v, o, lse, BH, Lq, Lk, scale, st, s);
  }
}

// ----------------------------------------------------------------- backward, bf16 (v2)
// dQ pass: queries on the lane, K/V 64-row tiles double-buffered (as forward).
// FD (fused delta): the lane's delta = rowsum(dO * O) is formed from the dO
// fragment it already holds and the same chunks of O (the two lane halves
// hold the two halves of the row: one permlane32 swap adds them) and written
// to delta_out for the dK/dV pass -- no separate preprocess launch, no second
// read of dO.
template <int D, int NW, int OCC, bool FD, bool HS, bool CS>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void attn_dq2_kernel(const __bf16 *__restrict__ Q, const __bf16 *__restrict__ K,
                                                           const __bf16 *__restrict__ V, const __bf16 *__restrict__ dO,
                                                           const float *__restrict__ lse,
                                                           const float *__restrict__ delta, __bf16 *__restrict__ dQ,
                                                           int Lq, int Lk, float scale, Strides st,
                                                           const __bf16 *__restrict__ O, float *__restrict__ delta_out,
                                                           float *__restrict__ cpart) {
  using C = Fwd2Cfg<D, NW>;
  extern __shared__ __attribute__((aligned(16))) unsigned char bwd2_smem[];
  __bf16 *sk = reinterpret_cast<__bf16 *>(bwd2_smem);
  __bf16 *sv = sk + 2 * C::kKBuf;
  int rb, bh;
  xcd_block(rb, bh);
  const int l = lane_(), h = l >> 5, w = threadIdx.x >> 6;
  const int q0 = rb * (NW * 32) + w * 32;
  const int qi = q0 + (l & 31);
  const bool qv = qi < Lq;
  bf16x8 qf[D / 16], gf[D / 16];
  {
    const __bf16 *qr = Q + st.q_off(bh) + (long long)(qv ? qi : 0) * st.q_srow + 8 * h;
    const __bf16 *gr = dO + st.o_off(bh) + (long long)(qv ? qi : 0) * st.o_srow + 8 * h;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      qf[s] = qv ? *reinterpret_cast<const bf16x8 *>(qr + 16 * s) : bf16x8{};
      gf[s] = qv ? *reinterpret_cast<const bf16x8 *>(gr + 16 * s) : bf16x8{};
    }
  }
  const float lse2 = qv ? lse[(long long)bh * Lq + qi] * kLog2e : INFINITY;
  float dl;
  if constexpr (FD) {
    const __bf16 *orow = O + st.o_off(bh) + (long long)(qv ? qi : 0) * st.o_srow + 8 * h;
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      const bf16x8 of = qv ? *reinterpret_cast<const bf16x8 *>(orow + 16 * s) : bf16x8{};
#pragma unroll
      for (int e = 0; e < 8; ++e) part = __builtin_fmaf((float)of[e], (float)gf[s][e], part);
    }
    dl = swap_halves_sum(part);
    if (h == 0 && qv) delta_out[(long long)bh * Lq + qi] = dl;
  } else {
    dl = qv ? delta[(long long)bh * Lq + qi] : 0.f;
  }
  const __bf16 *Kb = K + st.k_off(bh);
  const __bf16 *Vb = V + st.v_off(bh);
  const float sl2 = scale * kLog2e;
  f32x16 Y[D / 32];
#pragma unroll
  for (int db = 0; db < D / 32; ++db) Y[db] = f32x16{};
  typename C::Regs kr, vr;
  fwd2_load<D, NW>(kr, vr, Kb, st.k_srow, Vb, st.v_srow, 0, Lk);
  fwd2_store<D, NW>(sk, sv, kr, vr);
  lds_barrier();
  const int ntiles = (Lk + kKT - 1) / kKT;
  auto tile = [&](int t, auto edge_c) {
    constexpr bool EDGE = decltype(edge_c)::value;
    const int cur = t & 1;
    const int k0 = t * kKT;
    if (t + 1 < ntiles) fwd2_load<D, NW>(kr, vr, Kb, st.k_srow, Vb, st.v_srow, k0 + kKT, Lk);
    const __bf16 *ck = sk + cur * C::kKBuf;
    const __bf16 *cv = sv + cur * C::kVBuf;
    if constexpr (HS) {
      // one 32-key half at a time: half the live S / dP registers (the
      // accumulation order of Y is unchanged)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        f32x16 S = f32x16{}, G = f32x16{};
        k_product<D>(S, ck + 32 * hf * C::kKS, qf);
        k_product<D>(G, cv + 32 * hf * C::kVS, gf);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float p = exp2_ftz(__builtin_fmaf(S[r], sl2, -lse2));
          if constexpr (EDGE) {
            if (k0 + 32 * hf + acc_row(r, h) >= Lk) p = 0.f;
          }
          S[r] = p * (G[r] - dl);  // dS^T without the softmax scale
        }
        v_product<D>(Y, ck + 32 * hf * C::kKS, S);
      }
    } else {
      f32x16 S0 = f32x16{}, S1 = f32x16{}, G0 = f32x16{}, G1 = f32x16{};
#if PCOPS_DQ_A > 0
      // the two key halves' chains interleaved, each LDS read issued PCOPS_DQ_A MFMAs ahead
      // (the plain chains waited lgkmcnt(0) before every MFMA: the read latency exposed 32 times
      // a tile); per accumulator the MFMA order is k_product's, so dQ is bitwise unchanged
      k_product2<D>(S0, ck, qf, S1, ck + 32 * C::kKS, qf);
      sched_ds_mfma<D / 8, 1, PCOPS_DQ_A>();
      k_product2<D>(G0, cv, gf, G1, cv + 32 * C::kVS, gf);
      sched_ds_mfma<D / 8, 1, PCOPS_DQ_A>();
#else
      k_product<D>(S0, ck, qf);
      k_product<D>(S1, ck + 32 * C::kKS, qf);
      k_product<D>(G0, cv, gf);
      k_product<D>(G1, cv + 32 * C::kVS, gf);
#endif
  #pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p0 = exp2_ftz(__builtin_fmaf(S0[r], sl2, -lse2));
        float p1 = exp2_ftz(__builtin_fmaf(S1[r], sl2, -lse2));
        if constexpr (EDGE) {
          if (k0 + acc_row(r, h) >= Lk) p0 = 0.f;
          if (k0 + 32 + acc_row(r, h) >= Lk) p1 = 0.f;
        }
        S0[r] = p0 * (G0[r] - dl);  // dS^T without the softmax scale
        S1[r] = p1 * (G1[r] - dl);
      }
      v_product<D>(Y, ck, S0);
      v_product<D>(Y, ck + 32 * C::kKS, S1);
    }
    if (t + 1 < ntiles) fwd2_store<D, NW>(sk + (cur ^ 1) * C::kKBuf, sv + (cur ^ 1) * C::kVBuf, kr, vr);
    lds_barrier();
  };
  const int nfull = Lk / kKT;
  for (int t = 0; t < nfull; ++t) tile(t, std::false_type{});
  if (nfull < ntiles) tile(nfull, std::true_type{});
  store_Y<__bf16, D>(Y, dQ + st.q_off(bh), st.q_srow, q0, Lq, scale);
  if constexpr (CS) {  // the tiles' LDS is free: the last tile ended with a barrier
    float *sc = reinterpret_cast<float *>(bwd2_smem);
    colsum_wave<D>(Y, scale, qi < Lq, sc, w);
    lds_barrier();
    colsum_block<D, NW>(sc, cpart + colsum_row(bh, rb, st.H, D));
  }
}

// dK/dV pass: keys on the lane, Q/dO 64-row tiles (+ their lse/delta) double-buffered.
// MODE 0: dK and dV in one pass (one wave per SIMD: both D x 32 accumulators
// live).  MODE 1: dV only, MODE 2: dK only -- half the accumulators, so OCC = 2
// waves per SIMD fit; the split pays one extra S recompute (5 instead of 4
// GEMM units per key) for the second wave's latency hiding.
template <int D, int NW, int MODE, int OCC, bool CS>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void attn_dkv2_kernel(const __bf16 *__restrict__ Q,
                                                            const __bf16 *__restrict__ K,
                                                            const __bf16 *__restrict__ V,
                                                            const __bf16 *__restrict__ dO,
                                                            const float *__restrict__ lse,
                                                            const float *__restrict__ delta, __bf16 *__restrict__ dK,
                                                            __bf16 *__restrict__ dV, int Lq, int Lk, float scale,
                                                            Strides st, float *__restrict__ cpart_k,
                                                            float *__restrict__ cpart_v) {
  using C = Fwd2Cfg<D, NW>;
  extern __shared__ __attribute__((aligned(16))) unsigned char bwd2_smem[];
  __bf16 *sq = reinterpret_cast<__bf16 *>(bwd2_smem);
  __bf16 *sg = sq + 2 * C::kKBuf;
  float *slse = reinterpret_cast<float *>(sg + 2 * C::kVBuf);  // [2][64]
  float *sdl = slse + 2 * kKT;                                  // [2][64]
  int rb, bh;
  xcd_block(rb, bh);
  const int l = lane_(), h = l >> 5, w = threadIdx.x >> 6;
  const int k0w = rb * (NW * 32) + w * 32;
  const int ki = k0w + (l & 31);
  const bool kv = ki < Lk;
  bf16x8 kf[D / 16], vf[D / 16];
  {
    const __bf16 *kr0 = K + st.k_off(bh) + (long long)(kv ? ki : 0) * st.k_srow + 8 * h;
    const __bf16 *vr0 = V + st.v_off(bh) + (long long)(kv ? ki : 0) * st.v_srow + 8 * h;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      kf[s] = kv ? *reinterpret_cast<const bf16x8 *>(kr0 + 16 * s) : bf16x8{};
      vf[s] = (kv && MODE != 1) ? *reinterpret_cast<const bf16x8 *>(vr0 + 16 * s) : bf16x8{};
    }
  }
  const __bf16 *Qb = Q + st.q_off(bh);
  const __bf16 *Gb = dO + st.o_off(bh);
  const float *lse_b = lse + (long long)bh * Lq;
  const float *dl_b = delta + (long long)bh * Lq;
  const float sl2 = scale * kLog2e;
  f32x16 Y1[D / 32], Y2[D / 32];
#pragma unroll
  for (int db = 0; db < D / 32; ++db) {
    Y1[db] = f32x16{};
    Y2[db] = f32x16{};
  }
  typename C::Regs qr, gr;
  float lr = INFINITY, dr = 0.f;
  fwd2_load<D, NW, true>(qr, gr, Qb, st.q_srow, Gb, st.o_srow, 0, Lq);
  if (threadIdx.x < kKT) {
    lr = threadIdx.x < Lq ? lse_b[threadIdx.x] * kLog2e : INFINITY;
    dr = threadIdx.x < Lq ? dl_b[threadIdx.x] : 0.f;
  }
  fwd2_store<D, NW, true>(sq, sg, qr, gr);
  if (threadIdx.x < kKT) {
    slse[threadIdx.x] = lr;
    sdl[threadIdx.x] = dr;
  }
  lds_barrier();
  const int ntiles = (Lq + kKT - 1) / kKT;
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const int r0 = t * kKT;
    if (t + 1 < ntiles) {
      fwd2_load<D, NW, true>(qr, gr, Qb, st.q_srow, Gb, st.o_srow, r0 + kKT, Lq);
      if (threadIdx.x < kKT) {
        const int q = r0 + kKT + threadIdx.x;
        lr = q < Lq ? lse_b[q] * kLog2e : INFINITY;
        dr = q < Lq ? dl_b[q] : 0.f;
      }
    }
    const __bf16 *cq = sq + cur * C::kKBuf;
    const __bf16 *cg = sg + cur * C::kVBuf;
    const float *cl = slse + cur * kKT;
    const float *cd = sdl + cur * kKT;
    if constexpr (MODE == 0) {
      f32x16 S0 = f32x16{}, S1 = f32x16{}, G0 = f32x16{}, G1 = f32x16{};
      k_product<D>(S0, cq, kf);  // S  (queries x keys)
      k_product<D>(S1, cq + 32 * C::kKS, kf);
      k_product<D>(G0, cg, vf);  // dP (queries x keys)
      k_product<D>(G1, cg + 32 * C::kVS, vf);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = acc_row(r, h);
        const float p0 = exp2_ftz(__builtin_fmaf(S0[r], sl2, -cl[row]));  // 0 for rows beyond Lq (lse = +inf)
        const float p1 = exp2_ftz(__builtin_fmaf(S1[r], sl2, -cl[row + 32]));
        S0[r] = p0;
        S1[r] = p1;
        G0[r] = p0 * (G0[r] - cd[row]);
        G1[r] = p1 * (G1[r] - cd[row + 32]);
      }
      v_product<D>(Y1, cg, S0);  // dV^T += dO^T P
      v_product<D>(Y1, cg + 32 * C::kVS, S1);
      v_product<D>(Y2, cq, G0);  // dK^T += Q^T dS
      v_product<D>(Y2, cq + 32 * C::kKS, G1);
    } else {
      // one 32-query half at a time: half the live S / dP registers (the
      // per-accumulator order -- half 0 then half 1 -- is unchanged)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        f32x16 S = f32x16{}, G = f32x16{};
        k_product<D>(S, cq + 32 * hf * C::kKS, kf);
        if (MODE != 1) k_product<D>(G, cg + 32 * hf * C::kVS, vf);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = acc_row(r, h) + 32 * hf;
          const float p = exp2_ftz(__builtin_fmaf(S[r], sl2, -cl[row]));
          S[r] = p;
          if (MODE != 1) G[r] = p * (G[r] - cd[row]);
        }
        if (MODE != 2) v_product<D>(Y1, cg + 32 * hf * C::kVS, S);
        if (MODE != 1) v_product<D>(Y2, cq + 32 * hf * C::kKS, G);
      }
    }
    if (t + 1 < ntiles) {
      fwd2_store<D, NW, true>(sq + (cur ^ 1) * C::kKBuf, sg + (cur ^ 1) * C::kVBuf, qr, gr);
      if (threadIdx.x < kKT) {
        slse[(cur ^ 1) * kKT + threadIdx.x] = lr;
        sdl[(cur ^ 1) * kKT + threadIdx.x] = dr;
      }
    }
    lds_barrier();
  }
  if (MODE != 2) store_Y<__bf16, D>(Y1, dV + st.v_off(bh), st.v_srow, k0w, Lk, 1.f);
  if (MODE != 1) store_Y<__bf16, D>(Y2, dK + st.k_off(bh), st.k_srow, k0w, Lk, scale);
  if constexpr (CS) {  // the tiles' LDS is free: the last tile ended with a barrier
    float *sc = reinterpret_cast<float *>(bwd2_smem);
    const long long row = colsum_row(bh, rb, st.H, D);
    if (MODE != 2) colsum_wave<D>(Y1, 1.f, ki < Lk, sc, w);
    if (MODE != 1) colsum_wave<D>(Y2, scale, ki < Lk, sc + NW * D, w);
    lds_barrier();
    if (MODE != 2) colsum_block<D, NW>(sc, cpart_v + row);
    if (MODE != 1) colsum_block<D, NW>(sc + NW * D, cpart_k + row);
  }
}

// ----------------------------------------------------------------- dK/dV, one pass, software-pipelined (v3)
// 4 waves x 32 keys per block at one wave per SIMD (D = 128 keeps dK^T, dV^T,
// the K / V fragments and two half tiles' S / dP live: > 256 registers).  The
// query stream runs in 32-row half tiles j = 0, 1, 2, ...:
//   A(j)  S = Q_j K^T, dP = dO_j V^T              (2 D/16 MFMA, rows from LDS)
//   B(j)  P = exp2(S sl2 - lse2), dS = P (dP - delta), both rounded to bf16 (VALU)
//   C(j)  dV^T += dO_j^T P,  dK^T += Q_j^T dS      (2 D/16 MFMA, transposed reads)
// issued as [A(j+1) interleaved with B(j)] then [C(j)]: with no partner wave
// on the SIMD, the softmax-side VALU of one half fills the MFMA gaps of the
// next half's products.  The 64-row Q / dO tiles (with their lse / delta)
// rotate through a 3-slot LDS ring, so one barrier per tile suffices: the slot
// written before barrier t was last read before barrier t-1.  Per accumulator
// the MFMA order equals attn_dkv2_kernel MODE 0's, so dK / dV are bitwise the
// same as that kernel's.
template <int D>
__device__ __forceinline__ void v_product_b(f32x16 (&Y)[D / 32], const __bf16 *lds, const bf16x8 (&b)[2]) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int l = lane_(), h = l >> 5, g = (l >> 4) & 1, i = l & 15, q = i >> 2, p = i & 3;
  typedef __attribute__((address_space(3))) short4v lds_s4;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int row0 = 16 * s + 4 * h + q;
#pragma unroll
    for (int db = 0; db < D / 32; ++db) {
      const int ch = 4 * db + 2 * g + (p >> 1), e = 4 * (p & 1);
      const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(lds + img_off<D>(row0, ch) + e));
      const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(lds + img_off<D>(row0 + 8, ch) + e));
      const bf16x8 a = __builtin_shufflevector(__builtin_bit_cast(bf16x4, lo), __builtin_bit_cast(bf16x4, hi), 0, 1,
                                               2, 3, 4, 5, 6, 7);
      Y[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[s], Y[db], 0, 0, 0);
    }
  }
#endif
}

// B(j): the lane's 16 rows are acc_row(r, h) = 8g + 4h + i (r = 4g + i): four
// float4 LDS reads each of lse2 and delta (cl / cd point at the half's 32 rows),
// issued in a scheduling region of their own so the VALU groups of the
// interleaved [A | B] region find their operands ready
struct RowConsts {
  float4 l[4], d[4];
};
__device__ __forceinline__ void dkv3_rows(RowConsts &rc, const float *cl, const float *cd) {
  const int h = lane_() >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    rc.l[g] = *reinterpret_cast<const float4 *>(cl + 8 * g + 4 * h);
    rc.d[g] = *reinterpret_cast<const float4 *>(cd + 8 * g + 4 * h);
  }
}

// Instruction order inside the half step.  sched_barrier / sched_group_barrier
// do not hold here: they are side-effect intrinsics without memory operands,
// so the IR optimiser moves the (pure) MFMA and VALU work across them (all the
// fences of a half step ended up together after its last chunk).  An empty
// volatile asm with "+v" operands does hold: volatile asms keep their order,
// and an operand redefined by one can only be used after it.  pin() marks the
// start of a chunk; the chunk's inputs pass through it and its outputs
// through the next one, so each chunk's VALU and MFMA stay between the two.
// Diagnostic ablations of the dK/dV v3 loop (tools/dkv3_probe.hip builds; 0 in the
// product): 1 = B without exp / row constants, 2 = no C MFMAs, 4 = no A MFMAs
#ifndef PCOPS_DKV3_ABL
#define PCOPS_DKV3_ABL 0
#endif
#ifndef PCOPS_DS_NT
#define PCOPS_DS_NT 1
#endif
// Register pressure (round 6): the D = 128 body holds the next half's row fragments (64 VGPRs)
// and C's transposed fragments (64) from early in the half, and the compiler moves ~64-87
// values per tile between AGPRs and VGPRs to fit.  Reading them just in time instead
// (PCOPS_DKV3_LA / _LAC = chunks of read-ahead) removes ~23 of those moves but exposes the LDS
// latency: 1.43-1.47 -> 1.55-1.61 ms at 2048^2 (profiles/r6_dkv3_regpressure_ab.txt), so the
// early reads stay (0 = the whole half's fragments at once).  S / dP as VGPR-form inline-asm
// MFMAs (no v_accvgpr_read per score) did not fit either: the compiler spilled others instead.
#ifndef PCOPS_DKV3_LA
#define PCOPS_DKV3_LA 0
#endif
#ifndef PCOPS_DKV3_LAC
#define PCOPS_DKV3_LAC 0
#endif

template <typename T>
__device__ __forceinline__ void pin(T &x) {
  asm volatile("" : "+v"(x));
}

// the D/16 row fragments of a 32-row half (k_product's A operands), issued together
template <int D>
__device__ __forceinline__ void rows_frag(bf16x8 (&a)[D / 16], const __bf16 *lds) {
  const int l = lane_(), h = l >> 5, row = l & 31;
#pragma unroll
  for (int s = 0; s < D / 16; ++s) a[s] = *reinterpret_cast<const bf16x8 *>(lds + img_off<D>(row, 2 * s + h));
}

// fragment f = s (D/32) + db of tr_frag (two ds_read_b64_tr_b16)
template <int D>
__device__ __forceinline__ bf16x8 tr_frag1(const __bf16 *lds, int f) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int l = lane_(), h = l >> 5, g = (l >> 4) & 1, i = l & 15, q = i >> 2, p = i & 3;
  const int s = f / (D / 32), db = f % (D / 32);
  typedef __attribute__((address_space(3))) short4v lds_s4;
  const int row0 = 16 * s + 4 * h + q;
  const int ch = 4 * db + 2 * g + (p >> 1), e = 4 * (p & 1);
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(lds + img_off<D>(row0, ch) + e));
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(lds + img_off<D>(row0 + 8, ch) + e));
  return __builtin_shufflevector(__builtin_bit_cast(bf16x4, lo), __builtin_bit_cast(bf16x4, hi), 0, 1, 2, 3, 4, 5, 6, 7);
#else
  return bf16x8{};
#endif
}

// fragment s of rows_frag (one ds_read_b128)
template <int D>
__device__ __forceinline__ bf16x8 row_frag1(const __bf16 *lds, int s) {
  const int l = lane_(), h = l >> 5, row = l & 31;
  return *reinterpret_cast<const bf16x8 *>(lds + img_off<D>(row, 2 * s + h));
}

// the D/16 transposed fragments of a 32-row half (v_product's A operands, [s][db])
template <int D>
__device__ __forceinline__ void tr_frag(bf16x8 (&a)[D / 16], const __bf16 *lds) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int l = lane_(), h = l >> 5, g = (l >> 4) & 1, i = l & 15, q = i >> 2, p = i & 3;
  typedef __attribute__((address_space(3))) short4v lds_s4;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int row0 = 16 * s + 4 * h + q;
#pragma unroll
    for (int db = 0; db < D / 32; ++db) {
      const int ch = 4 * db + 2 * g + (p >> 1), e = 4 * (p & 1);
      const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(lds + img_off<D>(row0, ch) + e));
      const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(lds + img_off<D>(row0 + 8, ch) + e));
      a[s * (D / 32) + db] =
          __builtin_shufflevector(__builtin_bit_cast(bf16x4, lo), __builtin_bit_cast(bf16x4, hi), 0, 1, 2, 3, 4, 5, 6, 7);
    }
  }
#endif
}

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float f4_at(const float4 &v, int i) {
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}

// [A(j+1) | B(j)] in D/16 chunks: chunk I = MFMA I of the S chain and of the dP
// chain, plus B's rows [16 I / (D/16), 16 (I+1) / (D/16)) (whole bf16 pairs:
// packed words pw / gw[r / 2]).  NEXT = false: B only.  The transposed reads of
// C(j) are issued after chunk TRI so they land before C starts.
template <int D, bool NEXT, int I = 0>
__device__ __forceinline__ void dkv3_ab(f32x16 &Sn, f32x16 &Gn, bf16x8 (&qa)[D / 16], bf16x8 (&ga)[D / 16],
                                        bf16x8 (&kf)[D / 16], bf16x8 (&vf)[D / 16], const f32x16 &S,
                                        const f32x16 &G, const RowConsts &rc, float sl2, unsigned (&pw)[8],
                                        unsigned (&gw)[8], bf16x8 (&va)[D / 16], bf16x8 (&ka)[D / 16],
                                        const __bf16 *hq, const __bf16 *hg, const __bf16 *nq,
                                        const __bf16 *ng) {
  if constexpr (I < D / 16) {
    constexpr int R0 = 2 * (8 * I / (D / 16)), R1 = 2 * (8 * (I + 1) / (D / 16));
    float la[16], da[16];
#pragma unroll
    for (int r = R0; r < R1; ++r) {
      la[r] = f4_at(rc.l[r >> 2], r & 3);
      da[r] = f4_at(rc.d[r >> 2], r & 3);
      pin(la[r]);
      pin(da[r]);
    }
    if constexpr (NEXT && PCOPS_DKV3_LA > 0 && I + PCOPS_DKV3_LA < D / 16) {
      // the row fragments PCOPS_DKV3_LA chunks ahead (not all D/16 at the half's start: the
      // 512-register body then spilled ~90 registers per tile through v_accvgpr moves)
      qa[I + PCOPS_DKV3_LA] = row_frag1<D>(nq, I + PCOPS_DKV3_LA);
      ga[I + PCOPS_DKV3_LA] = row_frag1<D>(ng, I + PCOPS_DKV3_LA);
    }
    if constexpr (NEXT && !(PCOPS_DKV3_ABL & 4)) {
      pin(kf[I]);
      pin(vf[I]);
      Sn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa[I], kf[I], Sn, 0, 0, 0);
      Gn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[I], vf[I], Gn, 0, 0, 0);
    }
#pragma unroll
    for (int r = R0; r < R1; r += 2) {
#if PCOPS_DKV3_ABL & 1
      const bf16x2 pp = {(__bf16)S[r], (__bf16)S[r + 1]};
      const bf16x2 gg = {(__bf16)G[r], (__bf16)G[r + 1]};
#else
      const float p0 = exp2_ftz(__builtin_fmaf(S[r], sl2, -la[r]));  // 0 for rows beyond Lq (lse = +inf)
      const float p1 = exp2_ftz(__builtin_fmaf(S[r + 1], sl2, -la[r + 1]));
      const bf16x2 pp = {(__bf16)p0, (__bf16)p1};
      const bf16x2 gg = {(__bf16)(p0 * (G[r] - da[r])), (__bf16)(p1 * (G[r + 1] - da[r + 1]))};
#endif
      pw[r / 2] = __builtin_bit_cast(unsigned, pp);
      gw[r / 2] = __builtin_bit_cast(unsigned, gg);
      pin(pw[r / 2]);
      pin(gw[r / 2]);
    }
    if constexpr (PCOPS_DKV3_LAC > 0) {
      // C's first transposed fragments, issued in the last chunks so they land before C
      if constexpr (I == D / 16 - 1) {
#pragma unroll
        for (int f = 0; f < PCOPS_DKV3_LAC; ++f) {
          va[f] = tr_frag1<D>(hg, f);
          ka[f] = tr_frag1<D>(hq, f);
        }
      }
    } else if constexpr (I == D / 32) {
      tr_frag<D>(va, hg);
      tr_frag<D>(ka, hq);
    }
    dkv3_ab<D, NEXT, I + 1>(Sn, Gn, qa, ga, kf, vf, S, G, rc, sl2, pw, gw, va, ka, hq, hg, nq, ng);
  }
}

// C(j): dV^T += dO^T P (va), dK^T += Q^T dS (ka), per accumulator in v_product's order
template <int D>
__device__ __forceinline__ void dkv3_c(f32x16 (&Y1)[D / 32], f32x16 (&Y2)[D / 32], bf16x8 (&va)[D / 16],
                                       bf16x8 (&ka)[D / 16], const unsigned (&pw)[8], const unsigned (&gw)[8],
                                       const __bf16 *hq, const __bf16 *hg) {
  bf16x8 pb[2], gb[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    pb[s] = __builtin_bit_cast(bf16x8, (u32x4){pw[4 * s], pw[4 * s + 1], pw[4 * s + 2], pw[4 * s + 3]});
    gb[s] = __builtin_bit_cast(bf16x8, (u32x4){gw[4 * s], gw[4 * s + 1], gw[4 * s + 2], gw[4 * s + 3]});
  }
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int db = 0; db < D / 32; ++db) {
      const int f = s * (D / 32) + db;
      if constexpr (PCOPS_DKV3_LAC > 0) {
        // the fragment PCOPS_DKV3_LAC steps ahead (C's first ones came with the AB phase)
        if (f + PCOPS_DKV3_LAC < D / 16) {
          va[f + PCOPS_DKV3_LAC] = tr_frag1<D>(hg, f + PCOPS_DKV3_LAC);
          ka[f + PCOPS_DKV3_LAC] = tr_frag1<D>(hq, f + PCOPS_DKV3_LAC);
        }
      }
      Y1[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va[f], pb[s], Y1[db], 0, 0, 0);
      Y2[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka[f], gb[s], Y2[db], 0, 0, 0);
    }
}

// DS: also store dS^T (bf16, the values C(j) multiplies -- the dQ pass's dS rounded the same
// way) to dsT[bh][key][q] (ds_rows x ds_cols per head), for attn_dqs_kernel: dQ = dS K
// without recomputing S and dP.  Keys >= Lk store 0 (their S would be exp2(-lse): the dQ
// pass masks them).
template <int D, int OCC, bool CS, bool DS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void attn_dkv3_kernel(
    const __bf16 *__restrict__ Q, const __bf16 *__restrict__ K, const __bf16 *__restrict__ V,
    const __bf16 *__restrict__ dO, const float *__restrict__ lse, const float *__restrict__ delta,
    __bf16 *__restrict__ dK, __bf16 *__restrict__ dV, int Lq, int Lk, float scale, Strides st,
    float *__restrict__ cpart_k, float *__restrict__ cpart_v, __bf16 *__restrict__ dsT, int ds_rows,
    int ds_cols) {
  constexpr int NW = 4, RS = Img<D>::RS, TB = kKT * RS;  // TB: elements per tile slot
  constexpr int kCPT = kKT * D / 8 / (NW * 64);           // 16-B chunks per thread per tile
  static_assert(kKT * D / 8 % (NW * 64) == 0, "tile chunks must split evenly");
  extern __shared__ __attribute__((aligned(16))) unsigned char dkv3_smem[];
  __bf16 *sq = reinterpret_cast<__bf16 *>(dkv3_smem);  // [3][TB]
  __bf16 *sg = sq + 3 * TB;                             // [3][TB]
  float *slse = reinterpret_cast<float *>(sg + 3 * TB);  // [3][64]
  float *sdl = slse + 3 * kKT;                            // [3][64]
  int rb, bh;
  xcd_block(rb, bh);
  const int l = lane_(), h = l >> 5, w = threadIdx.x >> 6;
  const int k0w = rb * (NW * 32) + w * 32;
  const int ki = k0w + (l & 31);
  const bool kv = ki < Lk;
  bf16x8 kf[D / 16], vf[D / 16];
  {
    const __bf16 *kr0 = K + st.k_off(bh) + (long long)(kv ? ki : 0) * st.k_srow + 8 * h;
    const __bf16 *vr0 = V + st.v_off(bh) + (long long)(kv ? ki : 0) * st.v_srow + 8 * h;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      kf[s] = kv ? *reinterpret_cast<const bf16x8 *>(kr0 + 16 * s) : bf16x8{};
      vf[s] = kv ? *reinterpret_cast<const bf16x8 *>(vr0 + 16 * s) : bf16x8{};
    }
  }
  const __bf16 *Qb = Q + st.q_off(bh);
  const __bf16 *Gb = dO + st.o_off(bh);
  const float *lse_b = lse + (long long)bh * Lq;
  const float *dl_b = delta + (long long)bh * Lq;
  const float sl2 = scale * kLog2e;
  f32x16 Y1[D / 32], Y2[D / 32];
#pragma unroll
  for (int db = 0; db < D / 32; ++db) {
    Y1[db] = f32x16{};
    Y2[db] = f32x16{};
  }
  // tile loads: in-tile element offsets are per-thread constants (int: the host
  // checks 64 row strides fit), the tile base is wave-uniform.  A tile that
  // runs past Lq (the last one, or one beyond it) reads row Lq-1 in place of
  // the missing rows: finite values that meet P = 0 there (lse = +inf), so
  // they add exact zeros to dK / dV
  bf16x8 qr[kCPT], gr[kCPT];
  float lr, dr;
  // The per-thread tile offsets are recomputed at every use from an opaque copy of
  // threadIdx.x (a few integer ops): hoisted out of the tile loop they are ~20 loop-
  // invariant VGPRs, which the 512-register one-wave-per-SIMD body cannot hold -- the
  // *_colsum build spilled them and reloaded ~50 dwords from scratch per tile, each
  // reload a vector-memory op queued (vmcnt, in order) behind the tile loads.
  auto tid_ = [] {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
  };
  // A thread's chunks c of a tile are rows row0 + c RB (RB = NW 64 / (D / 8) rows per pass) at one
  // column: one unsigned 32-bit offset per tensor from the opaque thread id and a wave-uniform
  // (scalar) step per chunk.  The signed form (row * (int)srow) cost ~250 VALU per tile: a signed
  // division, a 64-bit sign extension and a 64-bit shift-add per chunk and tensor.
  constexpr int RB = (NW * 64) % (D / 8) == 0 ? NW * 64 / (D / 8) : 0;
  auto load = [&](int t) {
    const int r0 = t * kKT;
    if (RB && r0 + kKT <= Lq) {
      const __bf16 *qb = Qb + (long long)r0 * st.q_srow, *gb = Gb + (long long)r0 * st.o_srow;
      const unsigned tid = (unsigned)tid_(), row0 = tid / (D / 8), col = (tid % (D / 8)) * 8;
      const unsigned oq = row0 * (unsigned)st.q_srow + col, og = row0 * (unsigned)st.o_srow + col;
#pragma unroll
      for (int c = 0; c < kCPT; ++c) {
        qr[c] = *reinterpret_cast<const bf16x8 *>(qb + (long long)(c * RB) * st.q_srow + oq);
        gr[c] = *reinterpret_cast<const bf16x8 *>(gb + (long long)(c * RB) * st.o_srow + og);
      }
      lr = lse_b[r0 + l] * kLog2e;
      dr = dl_b[r0 + l];
    } else if (r0 + kKT <= Lq) {
      const __bf16 *qb = Qb + (long long)r0 * st.q_srow, *gb = Gb + (long long)r0 * st.o_srow;
      const int tid = tid_();
#pragma unroll
      for (int c = 0; c < kCPT; ++c) {
        const int idx = tid + c * NW * 64;
        const int row = idx / (D / 8), col = (idx % (D / 8)) * 8;
        qr[c] = *reinterpret_cast<const bf16x8 *>(qb + row * (int)st.q_srow + col);
        gr[c] = *reinterpret_cast<const bf16x8 *>(gb + row * (int)st.o_srow + col);
      }
      lr = lse_b[r0 + l] * kLog2e;
      dr = dl_b[r0 + l];
    } else {
      const int tid = tid_();
#pragma unroll
      for (int c = 0; c < kCPT; ++c) {
        const int idx = tid + c * NW * 64;
        const long long rr = min(r0 + idx / (D / 8), Lq - 1);
        qr[c] = *reinterpret_cast<const bf16x8 *>(Qb + rr * st.q_srow + (idx % (D / 8)) * 8);
        gr[c] = *reinterpret_cast<const bf16x8 *>(Gb + rr * st.o_srow + (idx % (D / 8)) * 8);
      }
      const int q = r0 + l;
      const bool ok = q < Lq;
      const float a = lse_b[ok ? q : Lq - 1], b = dl_b[ok ? q : Lq - 1];
      lr = ok ? a * kLog2e : INFINITY;
      dr = ok ? b : 0.f;
    }
  };
  // every wave writes the same 64 lse / delta values (no wave-dependent branch)
  auto store = [&](int slot) {
    if constexpr (RB % 16 == 0 && RB) {
      // Img<D>'s chunk permutation reads row bits 0..3 only: rows row0 + c RB share it, so every
      // chunk of the thread lands at one base + c RB RS (an immediate offset)
      const unsigned tid = (unsigned)tid_(), row0 = tid / (D / 8), ch = tid % (D / 8);
      const unsigned so = (unsigned)img_off<D>((int)row0, (int)ch);
#pragma unroll
      for (int c = 0; c < kCPT; ++c) {
        *reinterpret_cast<bf16x8 *>(sq + slot * TB + so + c * RB * RS) = qr[c];
        *reinterpret_cast<bf16x8 *>(sg + slot * TB + so + c * RB * RS) = gr[c];
      }
    } else {
      const int tid = tid_();
#pragma unroll
      for (int c = 0; c < kCPT; ++c) {
        const int idx = tid + c * NW * 64;
        const int row = idx / (D / 8), ch = idx % (D / 8);
        *reinterpret_cast<bf16x8 *>(sq + slot * TB + img_off<D>(row, ch)) = qr[c];
        *reinterpret_cast<bf16x8 *>(sg + slot * TB + img_off<D>(row, ch)) = gr[c];
      }
    }
    slse[slot * kKT + l] = lr;
    sdl[slot * kKT + l] = dr;
  };
  const int nt = (Lq + kKT - 1) / kKT;
  load(0);
  store(0);
  if (nt > 1) load(1);
  lds_barrier();
  f32x16 Sc = f32x16{}, Gc = f32x16{};
  k_product<D>(Sc, sq, kf);
  k_product<D>(Gc, sg, vf);
  int cur = 0, nxt = 1;  // slots of tiles t and t+1
  // one half step: [A(j+1) | B(j)] then C(j).  hq / hg: this half's Q / dO rows,
  // nq / ng: the next half's (unused when !NEXT); cl / cd: this half's row constants
  __bf16 *ds_row = nullptr;  // this lane's key row of dS^T
  if constexpr (DS) ds_row = dsT + ((long long)bh * ds_rows + ki) * ds_cols + 8 * h;
  auto half = [&](auto next_c, const __bf16 *hq, const __bf16 *hg, const __bf16 *nq, const __bf16 *ng,
                  const float *cl, const float *cd, int qh0, auto &&mid) {
    constexpr bool NEXT = decltype(next_c)::value;
    bf16x8 qa[D / 16], ga[D / 16];
    if constexpr (NEXT) {
      if constexpr (PCOPS_DKV3_LA > 0) {
#pragma unroll
        for (int s0 = 0; s0 < PCOPS_DKV3_LA && s0 < D / 16; ++s0) {
          qa[s0] = row_frag1<D>(nq, s0);
          ga[s0] = row_frag1<D>(ng, s0);
        }
      } else {
        rows_frag<D>(qa, nq);
        rows_frag<D>(ga, ng);
      }
    }
    RowConsts rc;
    dkv3_rows(rc, cl, cd);
    f32x16 Sn = f32x16{}, Gn = f32x16{};
    unsigned pw[8], gw[8];
    bf16x8 va[D / 16], ka[D / 16];
    dkv3_ab<D, NEXT>(Sn, Gn, qa, ga, kf, vf, Sc, Gc, rc, sl2, pw, gw, va, ka, hq, hg, nq, ng);
    if constexpr (!(PCOPS_DKV3_ABL & 2)) dkv3_c<D>(Y1, Y2, va, ka, pw, gw, hq, hg);
    if constexpr (DS) {
      // lane (key, h) holds queries 8g + 4h + 0..3 (g = 0..3) as bf16 pairs gw[2g], gw[2g+1]:
      // one permlane32 swap per pair of words gives each lane two runs of 8 queries
      // (h = 0: queries 0-7 and 16-23, h = 1: 8-15 and 24-31), stored as 16 B each
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      unsigned w[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) w[i] = kv ? gw[i] : 0u;
      const auto a0 = __builtin_amdgcn_permlane32_swap(w[0], w[2], false, false);
      const auto a1 = __builtin_amdgcn_permlane32_swap(w[1], w[3], false, false);
      const auto b0 = __builtin_amdgcn_permlane32_swap(w[4], w[6], false, false);
      const auto b1 = __builtin_amdgcn_permlane32_swap(w[5], w[7], false, false);
#if PCOPS_DS_NT
      // streaming stores: dS^T is read once, by the dQ kernel; keep the Q / dO tiles the
      // key blocks of a head share in L2
      __builtin_nontemporal_store((u32x4){a0[0], a1[0], a0[1], a1[1]}, reinterpret_cast<u32x4 *>(ds_row + qh0));
      __builtin_nontemporal_store((u32x4){b0[0], b1[0], b0[1], b1[1]}, reinterpret_cast<u32x4 *>(ds_row + qh0 + 16));
#else
      *reinterpret_cast<u32x4 *>(ds_row + qh0) = (u32x4){a0[0], a1[0], a0[1], a1[1]};
      *reinterpret_cast<u32x4 *>(ds_row + qh0 + 16) = (u32x4){b0[0], b1[0], b0[1], b1[1]};
#endif
    }
    mid();
    Sc = Sn;
    Gc = Gn;
  };
  const auto none = [] {};
  int t = 0;
  for (; t + 1 < nt; ++t) {
    const __bf16 *cq = sq + cur * TB, *cg = sg + cur * TB;
    const float *cl = slse + cur * kKT, *cd = sdl + cur * kKT;
    half(std::true_type{}, cq, cg, cq + 32 * RS, cg + 32 * RS, cl, cd, t * kKT, [&] {
      store(nxt);
      load(t + 2);  // past the end: clamped rows, never stored
    });
    lds_barrier();
    half(std::true_type{}, cq + 32 * RS, cg + 32 * RS, sq + nxt * TB, sg + nxt * TB, cl + 32, cd + 32, t * kKT + 32,
         none);
    cur = nxt;
    nxt = nxt == 2 ? 0 : nxt + 1;
  }
  {
    const __bf16 *cq = sq + cur * TB, *cg = sg + cur * TB;
    const float *cl = slse + cur * kKT, *cd = sdl + cur * kKT;
    half(std::true_type{}, cq, cg, cq + 32 * RS, cg + 32 * RS, cl, cd, t * kKT, none);
    half(std::false_type{}, cq + 32 * RS, cg + 32 * RS, cq, cg, cl + 32, cd + 32, t * kKT + 32, none);
  }
  store_Y<__bf16, D>(Y1, dV + st.v_off(bh), st.v_srow, k0w, Lk, 1.f);
  store_Y<__bf16, D>(Y2, dK + st.k_off(bh), st.k_srow, k0w, Lk, scale);
  if constexpr (CS) {
    lds_barrier();  // every wave is past its last ring read
    float *sc = reinterpret_cast<float *>(dkv3_smem);
    const long long row = colsum_row(bh, rb, st.H, D);
    colsum_wave<D>(Y1, 1.f, kv, sc, w);
    colsum_wave<D>(Y2, scale, kv, sc + NW * D, w);
    lds_barrier();
    colsum_block<D, NW>(sc, cpart_v + row);
    colsum_block<D, NW>(sc + NW * D, cpart_k + row);
  }
}

// ----------------------------------------------------------------- dQ from the stored dS (D >= 96)
// delta = rowsum(dO o O) for the bf16 passes, in the fused-delta order of attn_dq2_kernel
// (each lane half sums its d = 16 s + 8 h + e by fma in (s, e) order, then the halves are
// added): the dK/dV pass runs first on this path and sees the same delta bitwise.
template <int D>
__global__ __launch_bounds__(256) void attn_delta2_kernel(const __bf16 *__restrict__ O, const __bf16 *__restrict__ dO,
                                                          float *__restrict__ delta, int BH, int Lq, Strides st) {
  const int l = lane_(), h = l >> 5;
  const long long row = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 32 + (l & 31);
  if (row >= (long long)BH * Lq) return;  // both halves of a row leave together
  const int bh = (int)(row / Lq), q = (int)(row - (long long)bh * Lq);
  const __bf16 *orow = O + st.o_off(bh) + (long long)q * st.o_srow + 8 * h;
  const __bf16 *grow = dO + st.o_off(bh) + (long long)q * st.o_srow + 8 * h;
  float part = 0.f;
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    const bf16x8 of = *reinterpret_cast<const bf16x8 *>(orow + 16 * s);
    const bf16x8 gf = *reinterpret_cast<const bf16x8 *>(grow + 16 * s);
#pragma unroll
    for (int e = 0; e < 8; ++e) part = __builtin_fmaf((float)of[e], (float)gf[e], part);
  }
  const float dl = swap_halves_sum(part);
  if (h == 0) delta[row] = dl;
}

// dQ = scale * dS K from the dS^T the dK/dV pass stored (attn_dkv3_kernel<.., DS>): 8 waves
// x 32 queries per block, 64-key tiles of K (Img<D>) and of dS^T (keys x the block's 256
// queries) double-buffered in LDS.  Per wave and tile the MFMAs are attn_dq2_kernel's
// v_product calls in the same order with the same bf16 operands -- the B operand read from
// the dS^T image by the same transposed-read pattern instead of converted from registers --
// so dQ equals the recomputing pass's bitwise.  HBM-bound on the dS^T read (2 B per
// (query, key)); it replaces 3 GEMM units of MFMA work (S, dP recomputed, dQ) by 1.
constexpr int kDsRS = 256 + 32;  // dS^T image row stride (elements): conflict-free tr reads (tools/lds_banks.py)

template <int D>
__device__ __forceinline__ void v_product_ds(f32x16 (&Y)[D / 32], const __bf16 *kimg, const __bf16 *dimg) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int l = lane_(), h = l >> 5, g = (l >> 4) & 1, i = l & 15, q = i >> 2, p = i & 3;
  typedef __attribute__((address_space(3))) short4v lds_s4;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int row0 = 16 * s + 4 * h + q;
    const short4v blo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(dimg + row0 * kDsRS + 16 * g + 4 * p));
    const short4v bhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(dimg + (row0 + 8) * kDsRS + 16 * g + 4 * p));
    const bf16x8 b = __builtin_shufflevector(__builtin_bit_cast(bf16x4, blo), __builtin_bit_cast(bf16x4, bhi), 0, 1, 2,
                                             3, 4, 5, 6, 7);
#pragma unroll
    for (int db = 0; db < D / 32; ++db) {
      const int ch = 4 * db + 2 * g + (p >> 1), e = 4 * (p & 1);
      const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(kimg + img_off<D>(row0, ch) + e));
      const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(kimg + img_off<D>(row0 + 8, ch) + e));
      const bf16x8 a = __builtin_shufflevector(__builtin_bit_cast(bf16x4, lo), __builtin_bit_cast(bf16x4, hi), 0, 1,
                                               2, 3, 4, 5, 6, 7);
      Y[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, Y[db], 0, 0, 0);
    }
  }
#endif
}

template <int D, bool CS>
__global__ __launch_bounds__(512) void attn_dqs_kernel(const __bf16 *__restrict__ K, const __bf16 *__restrict__ dsT,
                                                       __bf16 *__restrict__ dQ, int Lq, int Lk, float scale, Strides st,
                                                       int ds_rows, int ds_cols, float *__restrict__ cpart) {
  constexpr int NW = 8, NT = NW * 64, RS = Img<D>::RS, KB = kKT * RS, SB = kKT * kDsRS;
  constexpr int kKC = (kKT * D / 8 + NT - 1) / NT;  // K chunks per thread
  constexpr int kDC = kKT * 32 / NT;                 // dS^T chunks per thread (64 rows x 32 chunks)
  extern __shared__ __attribute__((aligned(16))) unsigned char dqs_smem[];
  __bf16 *sk = reinterpret_cast<__bf16 *>(dqs_smem);  // [2][KB]
  __bf16 *sd = sk + 2 * KB;                            // [2][SB]
  int rb, bh;
  xcd_block(rb, bh);
  const int l = lane_(), w = threadIdx.x >> 6;
  const int q0 = rb * (NW * 32) + w * 32;
  const __bf16 *Kb = K + st.k_off(bh);
  const __bf16 *Db = dsT + (long long)bh * ds_rows * ds_cols + rb * (NW * 32);
  f32x16 Y[D / 32];
#pragma unroll
  for (int db = 0; db < D / 32; ++db) Y[db] = f32x16{};
  bf16x8 kr[kKC], dr[kDC];
  auto load = [&](int t) {
    const int k0 = t * kKT;
#pragma unroll
    for (int c = 0; c < kKC; ++c) {
      const int idx = threadIdx.x + c * NT;
      const int row = idx / (D / 8), ch = idx % (D / 8);
      const bool ok = (kKT * D / 8 % NT == 0 || idx < kKT * D / 8) && k0 + row < Lk;
      kr[c] = ok ? *reinterpret_cast<const bf16x8 *>(Kb + (long long)(k0 + row) * st.k_srow + ch * 8) : bf16x8{};
    }
#pragma unroll
    for (int c = 0; c < kDC; ++c) {
      const int idx = threadIdx.x + c * NT;
      const bf16x8 *src = reinterpret_cast<const bf16x8 *>(Db + (long long)(k0 + (idx >> 5)) * ds_cols + (idx & 31) * 8);
#if PCOPS_DS_NT
      dr[c] = __builtin_nontemporal_load(src);   // read once
#else
      dr[c] = *src;
#endif
    }
  };
  auto store = [&](int slot) {
#pragma unroll
    for (int c = 0; c < kKC; ++c) {
      const int idx = threadIdx.x + c * NT;
      if (kKT * D / 8 % NT != 0 && idx >= kKT * D / 8) continue;
      *reinterpret_cast<bf16x8 *>(sk + slot * KB + img_off<D>(idx / (D / 8), idx % (D / 8))) = kr[c];
    }
#pragma unroll
    for (int c = 0; c < kDC; ++c) {
      const int idx = threadIdx.x + c * NT;
      *reinterpret_cast<bf16x8 *>(sd + slot * SB + (idx >> 5) * kDsRS + (idx & 31) * 8) = dr[c];
    }
  };
  const int nt = (Lk + kKT - 1) / kKT;
  load(0);
  store(0);
  lds_barrier();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) load(t + 1);
    const __bf16 *ck = sk + cur * KB, *cd = sd + cur * SB + 32 * w;
    v_product_ds<D>(Y, ck, cd);
    v_product_ds<D>(Y, ck + 32 * RS, cd + 32 * kDsRS);
    if (t + 1 < nt) {
      store(cur ^ 1);
      lds_barrier();
    }
  }
  store_Y<__bf16, D>(Y, dQ + st.q_off(bh), st.q_srow, q0, Lq, scale);
  if constexpr (CS) {
    lds_barrier();  // every wave is past its last tile read
    float *sc = reinterpret_cast<float *>(dqs_smem);
    colsum_wave<D>(Y, scale, q0 + (l & 31) < Lq, sc, w);
    lds_barrier();
    colsum_block<D, NW>(sc, cpart + colsum_row(bh, rb, st.H, D));
  }
}

// D = 64 runs 4-wave blocks at 3 waves per SIMD (the key-half split fits
// 162 VGPRs): three independent blocks per CU instead of one 8-wave block.
// PCOPS_DQ_NW4=0 keeps the 8-wave form (A/B).
template <int D, int NW>
struct Dq2Cfg {
  static constexpr bool kHS = (D == 64 || D == 128) && NW == 4;  // D = 128, NW = 4: short sequences only
  static constexpr int kOcc = kHS ? (D == 64 ? 3 : 2) : (D <= 96 || NW == 8) ? 2 : 1;
};

// per-block column partial sums of the gradients a backward launch stores (the
// *_colsum entry points): dQ in `a`; dK in `a`, dV in `b`; row (bh * nrb + rb) of
// D floats each, nrb = the launch's row blocks per (batch, head), set by the launcher
struct ColPart {
  float *a = nullptr, *b = nullptr;
  int nrb = 0;
};

template <int D, int NW, bool FD, bool CS>
int launch_dq2_impl(const void *q, const void *k, const void *v, const void *dout, const float *lse,
                    const float *delta, void *dq, int BH, int Lq, int Lk, float scale, const Strides &st,
                    const void *o, float *delta_out, hipStream_t s, ColPart *cp) {
  using C = Fwd2Cfg<D, NW>;
  constexpr int OCC = Dq2Cfg<D, NW>::kOcc;
  constexpr bool HS = Dq2Cfg<D, NW>::kHS;
  static const hipError_t attr = hipFuncSetAttribute((const void *)attn_dq2_kernel<D, NW, OCC, FD, HS, CS>,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)C::kLds);
  if (attr != hipSuccess) return PCOPS_ERR_LAUNCH;
  const dim3 grid((Lq + NW * 32 - 1) / (NW * 32), BH);
  if (cp) cp->nrb = grid.x;
  hipLaunchKernelGGL((attn_dq2_kernel<D, NW, OCC, FD, HS, CS>), grid, dim3(C::kThr), C::kLds, s, (const __bf16 *)q,
                     (const __bf16 *)k, (const __bf16 *)v, (const __bf16 *)dout, lse, delta, (__bf16 *)dq, Lq, Lk,
                     scale, st, (const __bf16 *)o, delta_out, cp ? cp->a : nullptr);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

// o == nullptr: delta precomputed (read from `delta`); else fused, written to delta_out
template <int D, int NW>
int launch_dq2(const void *q, const void *k, const void *v, const void *dout, const float *lse, const float *delta,
               void *dq, int BH, int Lq, int Lk, float scale, const Strides &st, hipStream_t s,
               const void *o = nullptr, float *delta_out = nullptr, ColPart *cp = nullptr) {
  if (cp) return o ? launch_dq2_impl<D, NW, true, true>(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, scale, st, o, delta_out, s, cp)
                  : PCOPS_ERR_UNSUPPORTED;  // the column sums ride on the fused-delta pass
  return o ? launch_dq2_impl<D, NW, true, false>(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, scale, st, o, delta_out, s, cp)
           : launch_dq2_impl<D, NW, false, false>(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, scale, st, o, delta_out, s, cp);
}

bool dkv_split() {  // PCOPS_DKV_SPLIT=0 keeps the one-pass dK/dV kernel for D = 128 (A/B runs)
  static const bool v = [] {
    const char *e = getenv("PCOPS_DKV_SPLIT");
    return !(e && e[0] == '0');
  }();
  return v;
}

// one dK/dV launch of a given shape: NW waves per block, MODE (0 one pass, 3 one pass by
// 32-query halves -- the same per-accumulator order as 0, half the live S / dP), OCC waves / SIMD
template <int D, int NW, int MODE, int OCC, bool CS>
int launch_dkv2_cfg(const void *q, const void *k, const void *v, const void *dout, const float *lse,
                    const float *delta, void *dk, void *dv, int BH, int Lq, int Lk, float scale, const Strides &st,
                    hipStream_t s, ColPart *cp) {
  using C = Fwd2Cfg<D, NW>;
  const size_t lds = C::kLds + 4 * kKT * sizeof(float);
  static const hipError_t attr = hipFuncSetAttribute((const void *)attn_dkv2_kernel<D, NW, MODE, OCC, CS>,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return PCOPS_ERR_LAUNCH;
  const dim3 grid((Lk + NW * 32 - 1) / (NW * 32), BH);
  if (cp) cp->nrb = grid.x;
  hipLaunchKernelGGL((attn_dkv2_kernel<D, NW, MODE, OCC, CS>), grid, dim3(C::kThr), lds, s, (const __bf16 *)q,
                     (const __bf16 *)k, (const __bf16 *)v, (const __bf16 *)dout, lse, delta, (__bf16 *)dk,
                     (__bf16 *)dv, Lq, Lk, scale, st, cp ? cp->a : nullptr, cp ? cp->b : nullptr);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

template <int D, int OCC, bool CS, bool DS = false>
int launch_dkv3(const void *q, const void *k, const void *v, const void *dout, const float *lse, const float *delta,
                void *dk, void *dv, int BH, int Lq, int Lk, float scale, const Strides &st, hipStream_t s,
                ColPart *cp, __bf16 *dsT = nullptr, int ds_rows = 0, int ds_cols = 0) {
  if ((long long)kKT * (st.q_srow > st.o_srow ? st.q_srow : st.o_srow) >= (1ll << 31)) return PCOPS_ERR_UNSUPPORTED;
  const size_t lds = 6ull * kKT * Img<D>::RS * sizeof(__bf16) + 6 * kKT * sizeof(float);
  static const hipError_t attr = hipFuncSetAttribute((const void *)attn_dkv3_kernel<D, OCC, CS, DS>,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return PCOPS_ERR_LAUNCH;
  const dim3 grid((Lk + 127) / 128, BH);
  if (cp) cp->nrb = grid.x;
  hipLaunchKernelGGL((attn_dkv3_kernel<D, OCC, CS, DS>), grid, dim3(256), lds, s, (const __bf16 *)q,
                     (const __bf16 *)k, (const __bf16 *)v, (const __bf16 *)dout, lse, delta, (__bf16 *)dk,
                     (__bf16 *)dv, Lq, Lk, scale, st, cp ? cp->a : nullptr, cp ? cp->b : nullptr, dsT, ds_rows,
                     ds_cols);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

// dK/dV pass selection: the pipelined one-pass v3 kernel for D = 96 / 128 (bitwise the
// split v2 passes' results; A/B at the PCN shapes: 2048^2 hd128 1.51 -> 1.38 ms, 512^2
// hd96 0.105 -> 0.089 ms).  D = 64 keeps the 8-wave v2 pass (v3 at one wave per SIMD:
// 0.70 -> 1.0 ms).  PCOPS_DKV3: 0 = never v3, 1 = v3 for every D >= 64 (A/B runs).
int dkv3_mode() {
  static const int v = env_int("PCOPS_DKV3", -1);
  return v;
}

template <int D, int NW, bool CS>
int launch_dkv2_cs(const void *q, const void *k, const void *v, const void *dout, const float *lse, const float *delta,
                void *dk, void *dv, int BH, int Lq, int Lk, float scale, const Strides &st, hipStream_t s,
                ColPart *cp = nullptr) {
  using C = Fwd2Cfg<D, NW>;
  if constexpr (D >= 64) {
    const int m3 = dkv3_mode();
    if (m3 == 1 || (m3 < 0 && D >= 96)) {
      const int rc = launch_dkv3<D, 1, CS>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cp);
      if (rc != PCOPS_ERR_UNSUPPORTED) return rc;  // strides too large for its 32-bit tile offsets: v2 below
    }
  }
  if constexpr (D == 64 && NW == 8 && !CS) {
    // occupancy variants of the long-sequence D = 64 pass (A/B: PCOPS_DKV64)
    static const int var = env_int("PCOPS_DKV64", 0);
    switch (var) {
      case 1: return launch_dkv2_cfg<64, 4, 3, 2, CS>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cp);
      case 2: return launch_dkv2_cfg<64, 4, 3, 3, CS>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cp);
      case 3: return launch_dkv2_cfg<64, 8, 3, 2, CS>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cp);
      case 4: return launch_dkv2_cfg<64, 4, 0, 2, CS>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cp);
      default: break;
    }
  }
  const size_t lds = C::kLds + 4 * kKT * sizeof(float);
  const dim3 grid((Lk + NW * 32 - 1) / (NW * 32), BH);
  if constexpr (D == 128 && !CS) {
    // one-pass variants of the D = 128 dK/dV (A/B: PCOPS_DKV128): by 32-query halves, 1 wave per SIMD
    static const int var = env_int("PCOPS_DKV128", 0);
    if (var == 1) return launch_dkv2_cfg<128, 4, 3, 1, CS>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cp);
  }
  if (D >= 96 && dkv_split()) {
    // 8 waves per block halve each thread's share of the tile prefetch
    using C8 = Fwd2Cfg<D, 8>;
    const size_t lds8 = C8::kLds + 4 * kKT * sizeof(float);
    const dim3 grid8((Lk + 8 * 32 - 1) / (8 * 32), BH);
    if (cp) cp->nrb = grid8.x;
    static const hipError_t a1 = hipFuncSetAttribute((const void *)attn_dkv2_kernel<D, 8, 1, 2, CS>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds8);
    static const hipError_t a2 = hipFuncSetAttribute((const void *)attn_dkv2_kernel<D, 8, 2, 2, CS>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds8);
    if (a1 != hipSuccess || a2 != hipSuccess) return PCOPS_ERR_LAUNCH;
    hipLaunchKernelGGL((attn_dkv2_kernel<D, 8, 1, 2, CS>), grid8, dim3(C8::kThr), lds8, s, (const __bf16 *)q,
                       (const __bf16 *)k, (const __bf16 *)v, (const __bf16 *)dout, lse, delta, (__bf16 *)dk,
                       (__bf16 *)dv, Lq, Lk, scale, st, cp ? cp->a : nullptr, cp ? cp->b : nullptr);
    PC_CHECK_LAUNCH();
    hipLaunchKernelGGL((attn_dkv2_kernel<D, 8, 2, 2, CS>), grid8, dim3(C8::kThr), lds8, s, (const __bf16 *)q,
                       (const __bf16 *)k, (const __bf16 *)v, (const __bf16 *)dout, lse, delta, (__bf16 *)dk,
                       (__bf16 *)dv, Lq, Lk, scale, st, cp ? cp->a : nullptr, cp ? cp->b : nullptr);
    PC_CHECK_LAUNCH();
    return PCOPS_OK;
  }
  static const hipError_t attr = hipFuncSetAttribute((const void *)attn_dkv2_kernel<D, NW, 0, 1, CS>,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return PCOPS_ERR_LAUNCH;
  if (cp) cp->nrb = grid.x;
  hipLaunchKernelGGL((attn_dkv2_kernel<D, NW, 0, 1, CS>), grid, dim3(C::kThr), lds, s, (const __bf16 *)q,
                     (const __bf16 *)k, (const __bf16 *)v, (const __bf16 *)dout, lse, delta, (__bf16 *)dk,
                     (__bf16 *)dv, Lq, Lk, scale, st, cp ? cp->a : nullptr, cp ? cp->b : nullptr);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

template <int D, int NW>
int launch_dkv2(const void *q, const void *k, const void *v, const void *dout, const float *lse, const float *delta,
                void *dk, void *dv, int BH, int Lq, int Lk, float scale, const Strides &st, hipStream_t s,
                ColPart *cp = nullptr) {
  return cp ? launch_dkv2_cs<D, NW, true>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cp)
            : launch_dkv2_cs<D, NW, false>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cp);
}

int dq2_dispatch(const void *q, const void *k, const void *v, const void *dout, const float *lse, const float *delta,
                 void *dq, int BH, int Lq, int Lk, int D, float scale, const Strides &st, hipStream_t s,
                 const void *o = nullptr, float *delta_out = nullptr, ColPart *cp = nullptr) {
  const bool wide = Lq > 128;
  switch (D) {
    case 32:
      return wide ? launch_dq2<32, 8>(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, scale, st, s, o, delta_out, cp)
                  : launch_dq2<32, 4>(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, scale, st, s, o, delta_out, cp);
    case 64: {
      static const int nw4 = env_int("PCOPS_DQ_NW4", 1);
      return (wide && !nw4) ? launch_dq2<64, 8>(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, scale, st, s, o, delta_out, cp)
                            : launch_dq2<64, 4>(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, scale, st, s, o, delta_out, cp);
    }
    case 96:
      return launch_dq2<96, 4>(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, scale, st, s, o, delta_out, cp);
    case 128: {
      static const int nw4 = env_int("PCOPS_DQ128_NW4", 0);   // A/B: 4-wave key-half blocks at any length
      return (wide && !nw4) ? launch_dq2<128, 8>(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, scale, st, s, o, delta_out, cp)
                            : launch_dq2<128, 4>(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, scale, st, s, o, delta_out, cp);
    }
    default:
      return PCOPS_ERR_UNSUPPORTED;
  }
}

int dkv2_dispatch(const void *q, const void *k, const void *v, const void *dout, const float *lse, const float *delta,
                  void *dk, void *dv, int BH, int Lq, int Lk, int D, float scale, const Strides &st, hipStream_t s,
                  ColPart *cp = nullptr) {
  const bool wide = Lk > 128;
  switch (D) {
    case 32:
      return wide ? launch_dkv2<32, 8>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cp)
                  : launch_dkv2<32, 4>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cp);
    case 64:
      return wide ? launch_dkv2<64, 8>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cp)
                  : launch_dkv2<64, 4>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cp);
    case 96:
      return launch_dkv2<96, 4>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cp);
    case 128:
      return launch_dkv2<128, 4>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cp);
    default:
      return PCOPS_ERR_UNSUPPORTED;
  }
}

// dS^T buffer geometry of the D >= 96 path: rows = the dK/dV pass's key blocks (128),
// columns = the dQ kernel's query blocks (256)
struct DsGeom {
  int rows, cols;
  DsGeom(int Lq, int Lk) : rows((Lk + 127) / 128 * 128), cols((Lq + 255) / 256 * 256) {}
  unsigned long long bytes(int BH) const { return (unsigned long long)BH * rows * cols * sizeof(__bf16); }
};

// PCOPS_ATTN_DS=0 keeps the recomputing dQ pass for D >= 96 (A/B runs)
bool ds_path_on() {
  static const bool v = env_int("PCOPS_ATTN_DS", 1) != 0;
  return v;
}

template <int D, bool CS>
int launch_bwd_ds(const void *q, const void *k, const void *v, const void *o, const void *dout, const float *lse,
                  void *dq, void *dk, void *dv, int BH, int Lq, int Lk, float scale, const Strides &st, hipStream_t s,
                  float *delta, __bf16 *dsT, ColPart *cpq, ColPart *cpkv) {
  const DsGeom gm(Lq, Lk);
  const long long rows = (long long)BH * Lq;
  hipLaunchKernelGGL((attn_delta2_kernel<D>), dim3((unsigned)((rows + 127) / 128)), dim3(256), 0, s,
                     (const __bf16 *)o, (const __bf16 *)dout, delta, BH, Lq, st);
  PC_CHECK_LAUNCH();
  int rc = launch_dkv3<D, 1, CS, true>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, scale, st, s, cpkv, dsT,
                                       gm.rows, gm.cols);
  if (rc) return rc;
  constexpr size_t lds = 2ull * kKT * (Img<D>::RS + kDsRS) * sizeof(__bf16);
  static const hipError_t attr = hipFuncSetAttribute((const void *)attn_dqs_kernel<D, CS>,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return PCOPS_ERR_LAUNCH;
  const dim3 grid((Lq + 255) / 256, BH);
  if (cpq) cpq->nrb = grid.x;
  hipLaunchKernelGGL((attn_dqs_kernel<D, CS>), grid, dim3(512), lds, s, (const __bf16 *)k, (const __bf16 *)dsT,
                     (__bf16 *)dq, Lq, Lk, scale, st, gm.rows, gm.cols, cpq ? cpq->a : nullptr);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

int fwd2_dispatch(const void *q, const void *k, const void *v, void *o, float *lse, int BH, int Lq, int Lk, int D,
                  float scale, const Strides &st, hipStream_t s) {
  const bool wide = Lq > 128;
  switch (D) {
    case 32:
      return wide ? launch_fwd2<32, 8>(q, k, v, o, lse, BH, Lq, Lk, scale, st, s)
                  : launch_fwd2<32, 4>(q, k, v, o, lse, BH, Lq, Lk, scale, st, s);
    case 64:
      return wide ? launch_fwd2<64, 8>(q, k, v, o, lse, BH, Lq, Lk, scale, st, s)
                  : launch_fwd2<64, 4>(q, k, v, o, lse, BH, Lq, Lk, scale, st, s);
    case 96:
      return wide ? launch_fwd2<96, 8>(q, k, v, o, lse, BH, Lq, Lk, scale, st, s)
                  : launch_fwd2<96, 4>(q, k, v, o, lse, BH, Lq, Lk, scale, st, s);
    case 128:
      return wide ? launch_fwd2<128, 8>(q, k, v, o, lse, BH, Lq, Lk, scale, st, s)
                  : launch_fwd2<128, 4>(q, k, v, o, lse, BH, Lq, Lk, scale, st, s);
    default:
      return PCOPS_ERR_UNSUPPORTED;
  }
}

bool use_v1() {
  static const int v = [] {
    const char *e = getenv("PCOPS_ATTN_V1");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  return v != 0;
}

bool aligned_ok(const void *p, long long sb, long long sh, long long srow, int esize) {
  const int vec = 16 / esize;
  return ((uintptr_t)p % 16 == 0) && (sb % vec == 0) && (sh % vec == 0) && (srow % vec == 0);
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

// out_s[c] = sum over r < n of part_s[r * C + c] for one or two (part, out) segments
// (the per-block partial rows of dQ, or of dK and dV, C = H * D): 32 columns x 32 row
// groups per block, each group in row order, then the groups in order -- a fixed
// order for a given launch shape.  Blocks [0, C / 32) sum segment 0, the rest segment 1.
__global__ __launch_bounds__(1024) void attn_colsum_reduce_kernel(const float *__restrict__ p0, float *__restrict__ o0,
                                                                  const float *__restrict__ p1, float *__restrict__ o1,
                                                                  int n, int C) {
  __shared__ float red[32][33];
  const int nb = C / 32, seg = (int)blockIdx.x >= nb;
  const float *part = seg ? p1 : p0;
  float *out = seg ? o1 : o0;
  const int cl = threadIdx.x & 31, grp = threadIdx.x >> 5, col = ((int)blockIdx.x - seg * nb) * 32 + cl;
  float acc = 0.f;
#pragma unroll 8
  for (int r = grp; r < n; r += 32) acc += part[(long long)r * C + col];
  red[grp][cl] = acc;
  __syncthreads();
  if (grp == 0) {
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) sum += red[i][cl];
    out[col] = sum;
  }
}

int launch_colsum_reduce(const float *p0, float *o0, const float *p1, float *o1, int n, int C, hipStream_t s) {
  hipLaunchKernelGGL(attn_colsum_reduce_kernel, dim3((p1 ? 2 : 1) * C / 32), dim3(1024), 0, s, p0, o0, p1, o1, n, C);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

unsigned long long delta_bytes(int B, int H, int Lq) {
  return ((unsigned long long)B * H * Lq * sizeof(float) + 255) & ~255ull;
}

int check_common(int BH, int Lq, int Lk, int D, int dtype) {
  if (BH < 0 || Lq < 0 || Lk < 0) return PCOPS_ERR_INVALID;
  if (D % 32 != 0 || D <= 0 || D > 128 || (dtype != 0 && dtype != 1)) return PCOPS_ERR_UNSUPPORTED;
  return PCOPS_OK;
}

}  // namespace

#define PC_ATTN_STRIDES                                                                                     \
  long long q_sb, long long q_sh, long long q_srow, long long k_sb, long long k_sh, long long k_srow, long long v_sb, \
      long long v_sh, long long v_srow, long long o_sb, long long o_sh, long long o_srow
#define PC_ATTN_STRIDE_ARGS q_sb, q_sh, q_srow, k_sb, k_sh, k_srow, v_sb, v_sh, v_srow, o_sb, o_sh, o_srow

extern "C" int pcops_attention_forward(const void *q, const void *k, const void *v, void *o, float *lse, int B, int H,
                                       int Lq, int Lk, int D, float scale, int dtype, PC_ATTN_STRIDES,
                                       pcops_stream_t stream) {
  if (B < 0 || H <= 0 || Lq < 0 || Lk < 0) return PCOPS_ERR_INVALID;
  const int BH = B * H;
  if (BH == 0 || Lq == 0) return PCOPS_OK;
  if (Lk <= 0 || !q || !k || !v || !o) return PCOPS_ERR_INVALID;
  if (D % 32 != 0 || D > 128 || (dtype != 0 && dtype != 1)) return PCOPS_ERR_UNSUPPORTED;
  const int es = dtype == 0 ? 4 : 2;
  if (!aligned_ok(q, q_sb, q_sh, q_srow, es) || !aligned_ok(k, k_sb, k_sh, k_srow, es) ||
      !aligned_ok(v, v_sb, v_sh, v_srow, es) || !aligned_ok(o, o_sb, o_sh, o_srow, es))
    return PCOPS_ERR_UNSUPPORTED;
  const Strides st{PC_ATTN_STRIDE_ARGS, H};
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 0) return launch_fwd<float>(q, k, v, o, lse, BH, Lq, Lk, D, scale, st, s);
  if (use_v1()) return launch_fwd<__bf16>(q, k, v, o, lse, BH, Lq, Lk, D, scale, st, s);
  return fwd2_dispatch(q, k, v, o, lse, BH, Lq, Lk, D, scale, st, s);
}

extern "C" unsigned long long pcops_attention_bwd_workspace_bytes(int B, int H, int Lq, int Lk, int D) {
  (void)Lk;
  (void)D;
  if (B <= 0 || H <= 0 || Lq <= 0) return 0;
  return (unsigned long long)B * H * Lq * sizeof(float);
}

extern "C" int pcops_attention_bwd_preprocess(const void *o, const void *dout, int B, int H, int Lq, int D, int dtype,
                                              long long o_sb, long long o_sh, long long o_srow, void *workspace,
                                              unsigned long long workspace_bytes, pcops_stream_t stream) {
  if (B < 0 || H <= 0 || Lq < 0) return PCOPS_ERR_INVALID;
  int rc = check_common(B * H, Lq, 1, D, dtype);
  if (rc) return rc;
  const int BH = B * H;
  if (BH == 0 || Lq == 0) return PCOPS_OK;
  if (!o || !dout) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_attention_bwd_workspace_bytes(B, H, Lq, 1, D)) return PCOPS_ERR_WORKSPACE;
  const Strides st{0, 0, 0, 0, 0, 0, 0, 0, 0, o_sb, o_sh, o_srow, H};
  hipStream_t s = (hipStream_t)stream;
  return dtype == 0 ? launch_delta<float>(o, dout, (float *)workspace, BH, Lq, D, st, s)
                    : launch_delta<__bf16>(o, dout, (float *)workspace, BH, Lq, D, st, s);
}

extern "C" int pcops_attention_bwd_dq(const void *q, const void *k, const void *v, const void *dout, const float *lse,
                                      void *dq, int B, int H, int Lq, int Lk, int D, float scale, int dtype,
                                      PC_ATTN_STRIDES, const void *workspace, unsigned long long workspace_bytes,
                                      pcops_stream_t stream) {
  if (B < 0 || H <= 0) return PCOPS_ERR_INVALID;
  int rc = check_common(B * H, Lq, Lk, D, dtype);
  if (rc) return rc;
  const int BH = B * H;
  if (BH == 0 || Lq == 0) return PCOPS_OK;
  if (!q || !k || !v || !dout || !lse || !dq || Lk <= 0) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_attention_bwd_workspace_bytes(B, H, Lq, Lk, D)) return PCOPS_ERR_WORKSPACE;
  const int es = dtype == 0 ? 4 : 2;
  if (!aligned_ok(q, q_sb, q_sh, q_srow, es) || !aligned_ok(k, k_sb, k_sh, k_srow, es) ||
      !aligned_ok(v, v_sb, v_sh, v_srow, es) || !aligned_ok(dout, o_sb, o_sh, o_srow, es) ||
      !aligned_ok(dq, q_sb, q_sh, q_srow, es))
    return PCOPS_ERR_UNSUPPORTED;
  const Strides st{PC_ATTN_STRIDE_ARGS, H};
  hipStream_t s = (hipStream_t)stream;
  const float *delta = (const float *)workspace;
  if (dtype == 0) return launch_dq<float>(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, D, scale, st, s);
  if (use_v1()) return launch_dq<__bf16>(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, D, scale, st, s);
  return dq2_dispatch(q, k, v, dout, lse, delta, dq, BH, Lq, Lk, D, scale, st, s);
}

extern "C" int pcops_attention_bwd_dq_delta(const void *q, const void *k, const void *v, const void *o,
                                            const void *dout, const float *lse, void *dq, int B, int H, int Lq, int Lk,
                                            int D, float scale, int dtype, PC_ATTN_STRIDES, void *workspace,
                                            unsigned long long workspace_bytes, pcops_stream_t stream) {
  if (B < 0 || H <= 0) return PCOPS_ERR_INVALID;
  int rc = check_common(B * H, Lq, Lk, D, dtype);
  if (rc) return rc;
  const int BH = B * H;
  if (BH == 0 || Lq == 0) return PCOPS_OK;
  if (dtype == 0 || use_v1()) {  // fp32 / first-generation kernels: the two-launch form
    rc = pcops_attention_bwd_preprocess(o, dout, B, H, Lq, D, dtype, o_sb, o_sh, o_srow, workspace, workspace_bytes,
                                        stream);
    if (rc) return rc;
    return pcops_attention_bwd_dq(q, k, v, dout, lse, dq, B, H, Lq, Lk, D, scale, dtype, PC_ATTN_STRIDE_ARGS,
                                  workspace, workspace_bytes, stream);
  }
  if (!q || !k || !v || !o || !dout || !lse || !dq || Lk <= 0) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_attention_bwd_workspace_bytes(B, H, Lq, Lk, D)) return PCOPS_ERR_WORKSPACE;
  if (!aligned_ok(q, q_sb, q_sh, q_srow, 2) || !aligned_ok(k, k_sb, k_sh, k_srow, 2) ||
      !aligned_ok(v, v_sb, v_sh, v_srow, 2) || !aligned_ok(dout, o_sb, o_sh, o_srow, 2) ||
      !aligned_ok(o, o_sb, o_sh, o_srow, 2) || !aligned_ok(dq, q_sb, q_sh, q_srow, 2))
    return PCOPS_ERR_UNSUPPORTED;
  const Strides st{PC_ATTN_STRIDE_ARGS, H};
  return dq2_dispatch(q, k, v, dout, lse, nullptr, dq, BH, Lq, Lk, D, scale, st, (hipStream_t)stream, o,
                      (float *)workspace);
}

extern "C" int pcops_attention_bwd_dkv(const void *q, const void *k, const void *v, const void *dout,
                                       const float *lse, void *dk, void *dv, int B, int H, int Lq, int Lk, int D,
                                       float scale, int dtype, PC_ATTN_STRIDES, const void *workspace,
                                       unsigned long long workspace_bytes, pcops_stream_t stream) {
  if (B < 0 || H <= 0) return PCOPS_ERR_INVALID;
  int rc = check_common(B * H, Lq, Lk, D, dtype);
  if (rc) return rc;
  const int BH = B * H;
  if (BH == 0 || Lk == 0) return PCOPS_OK;
  if (!q || !k || !v || !dout || !lse || !dk || !dv || Lq <= 0) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_attention_bwd_workspace_bytes(B, H, Lq, Lk, D)) return PCOPS_ERR_WORKSPACE;
  const int es = dtype == 0 ? 4 : 2;
  if (!aligned_ok(q, q_sb, q_sh, q_srow, es) || !aligned_ok(k, k_sb, k_sh, k_srow, es) ||
      !aligned_ok(v, v_sb, v_sh, v_srow, es) || !aligned_ok(dout, o_sb, o_sh, o_srow, es) ||
      !aligned_ok(dk, k_sb, k_sh, k_srow, es) || !aligned_ok(dv, v_sb, v_sh, v_srow, es))
    return PCOPS_ERR_UNSUPPORTED;
  const Strides st{PC_ATTN_STRIDE_ARGS, H};
  hipStream_t s = (hipStream_t)stream;
  const float *delta = (const float *)workspace;
  if (dtype == 0) return launch_dkv<float>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, D, scale, st, s);
  if (use_v1()) return launch_dkv<__bf16>(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, D, scale, st, s);
  return dkv2_dispatch(q, k, v, dout, lse, delta, dk, dv, BH, Lq, Lk, D, scale, st, s);
}

// The same two passes, each also forming the column sums of the gradients it
// stores (per head, over batch and rows: out[h * D + d]) -- the bias gradient of
// the projection that produced q / k / v, without a pass over the gradient.
extern "C" unsigned long long pcops_attention_bwd_colsum_workspace_bytes(int B, int H, int Lq, int Lk, int D) {
  if (B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0 || D <= 0) return 0;
  const long long rq = (Lq + 127) / 128, rk = 2 * ((Lk + 127) / 128);
  return delta_bytes(B, H, Lq) + (unsigned long long)B * H * (rq > rk ? rq : rk) * D * sizeof(float);
}

extern "C" int pcops_attention_bwd_dq_delta_colsum(const void *q, const void *k, const void *v, const void *o,
                                                   const void *dout, const float *lse, void *dq, float *dq_colsum,
                                                   int B, int H, int Lq, int Lk, int D, float scale, int dtype,
                                                   PC_ATTN_STRIDES, void *workspace, unsigned long long workspace_bytes,
                                                   pcops_stream_t stream) {
  if (B < 0 || H <= 0) return PCOPS_ERR_INVALID;
  int rc = check_common(B * H, Lq, Lk, D, dtype);
  if (rc) return rc;
  if (dtype != 1 || use_v1()) return PCOPS_ERR_UNSUPPORTED;  // the bf16 MFMA passes only
  const int BH = B * H;
  if (!dq_colsum) return PCOPS_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  if (BH == 0) return PCOPS_OK;
  if (Lq == 0) return pc_memset_async(dq_colsum, 0, (size_t)H * D * sizeof(float), s) == hipSuccess ? PCOPS_OK
                                                                                              : PCOPS_ERR_LAUNCH;
  if (!q || !k || !v || !o || !dout || !lse || !dq || Lk <= 0) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_attention_bwd_colsum_workspace_bytes(B, H, Lq, Lk, D))
    return PCOPS_ERR_WORKSPACE;
  if (!aligned_ok(q, q_sb, q_sh, q_srow, 2) || !aligned_ok(k, k_sb, k_sh, k_srow, 2) ||
      !aligned_ok(v, v_sb, v_sh, v_srow, 2) || !aligned_ok(dout, o_sb, o_sh, o_srow, 2) ||
      !aligned_ok(o, o_sb, o_sh, o_srow, 2) || !aligned_ok(dq, q_sb, q_sh, q_srow, 2))
    return PCOPS_ERR_UNSUPPORTED;
  const Strides st{PC_ATTN_STRIDE_ARGS, H};
  ColPart cp;
  cp.a = (float *)((char *)workspace + delta_bytes(B, H, Lq));
  rc = dq2_dispatch(q, k, v, dout, lse, nullptr, dq, BH, Lq, Lk, D, scale, st, s, o, (float *)workspace, &cp);
  if (rc) return rc;
  return launch_colsum_reduce(cp.a, dq_colsum, nullptr, nullptr, B * cp.nrb, H * D, s);
}

extern "C" int pcops_attention_bwd_dkv_colsum(const void *q, const void *k, const void *v, const void *dout,
                                              const float *lse, void *dk, void *dv, float *dk_colsum, float *dv_colsum,
                                              int B, int H, int Lq, int Lk, int D, float scale, int dtype,
                                              PC_ATTN_STRIDES, void *workspace, unsigned long long workspace_bytes,
                                              pcops_stream_t stream) {
  if (B < 0 || H <= 0) return PCOPS_ERR_INVALID;
  int rc = check_common(B * H, Lq, Lk, D, dtype);
  if (rc) return rc;
  if (dtype != 1 || use_v1()) return PCOPS_ERR_UNSUPPORTED;
  const int BH = B * H;
  if (!dk_colsum || !dv_colsum) return PCOPS_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  if (BH == 0) return PCOPS_OK;
  if (Lk == 0) {
    if (pc_memset_async(dk_colsum, 0, (size_t)H * D * sizeof(float), s) != hipSuccess ||
        pc_memset_async(dv_colsum, 0, (size_t)H * D * sizeof(float), s) != hipSuccess)
      return PCOPS_ERR_LAUNCH;
    return PCOPS_OK;
  }
  if (!q || !k || !v || !dout || !lse || !dk || !dv || Lq <= 0) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_attention_bwd_colsum_workspace_bytes(B, H, Lq, Lk, D))
    return PCOPS_ERR_WORKSPACE;
  if (!aligned_ok(q, q_sb, q_sh, q_srow, 2) || !aligned_ok(k, k_sb, k_sh, k_srow, 2) ||
      !aligned_ok(v, v_sb, v_sh, v_srow, 2) || !aligned_ok(dout, o_sb, o_sh, o_srow, 2) ||
      !aligned_ok(dk, k_sb, k_sh, k_srow, 2) || !aligned_ok(dv, v_sb, v_sh, v_srow, 2))
    return PCOPS_ERR_UNSUPPORTED;
  const Strides st{PC_ATTN_STRIDE_ARGS, H};
  ColPart cp;
  cp.a = (float *)((char *)workspace + delta_bytes(B, H, Lq));
  cp.b = cp.a + (long long)BH * ((Lk + 127) / 128) * D;
  rc = dkv2_dispatch(q, k, v, dout, lse, (const float *)workspace, dk, dv, BH, Lq, Lk, D, scale, st, s, &cp);
  if (rc) return rc;
  return launch_colsum_reduce(cp.a, dk_colsum, cp.b, dv_colsum, B * cp.nrb, H * D, s);
}

// dq/dk/dv use the q/k/v strides; dout uses the o strides.
extern "C" int pcops_attention_backward(const void *q, const void *k, const void *v, const void *o, const void *dout,
                                        const float *lse, void *dq, void *dk, void *dv, int B, int H, int Lq, int Lk,
                                        int D, float scale, int dtype, PC_ATTN_STRIDES, void *workspace,
                                        unsigned long long workspace_bytes, pcops_stream_t stream) {
  if (B < 0 || H <= 0) return PCOPS_ERR_INVALID;
  if (B == 0 || Lq == 0 || Lk == 0) return check_common(B * H, Lq, Lk, D, dtype);
  const int es = dtype == 0 ? 4 : 2;
  if (o && !aligned_ok(o, o_sb, o_sh, o_srow, es)) return PCOPS_ERR_UNSUPPORTED;
  int rc = pcops_attention_bwd_dq_delta(q, k, v, o, dout, lse, dq, B, H, Lq, Lk, D, scale, dtype, PC_ATTN_STRIDE_ARGS,
                                        workspace, workspace_bytes, stream);
  if (rc) return rc;
  return pcops_attention_bwd_dkv(q, k, v, dout, lse, dk, dv, B, H, Lq, Lk, D, scale, dtype, PC_ATTN_STRIDE_ARGS,
                                 workspace, workspace_bytes, stream);
}

// The whole backward in one call (delta, dK/dV, dQ, and with *_colsum non-null the
// in_proj bias column sums of all three).  bf16 with D >= 96: the dK/dV pass stores dS^T and
// dQ = dS K is read back from it (attn_dqs_kernel: 1 GEMM unit instead of the 3 of the
// recomputing pass; bitwise the same dQ); otherwise the two-pass sequence above.
extern "C" unsigned long long pcops_attention_bwd_fused_workspace_bytes(int B, int H, int Lq, int Lk, int D,
                                                                         int dtype) {
  if (B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0 || D <= 0) return 0;
  const unsigned long long BH = (unsigned long long)B * H;
  unsigned long long n = delta_bytes(B, H, Lq);
  const unsigned long long rq = (Lq + 127) / 128, rk = (Lk + 127) / 128;
  n += ((BH * (rq + 2 * rk) * D * sizeof(float)) + 255) & ~255ull;
  if (dtype == 1 && D >= 96) n += DsGeom(Lq, Lk).bytes((int)BH);
  return n;
}

extern "C" int pcops_attention_bwd_fused(const void *q, const void *k, const void *v, const void *o, const void *dout,
                                         const float *lse, void *dq, void *dk, void *dv, float *dq_colsum,
                                         float *dk_colsum, float *dv_colsum, int B, int H, int Lq, int Lk, int D,
                                         float scale, int dtype, PC_ATTN_STRIDES, void *workspace,
                                         unsigned long long workspace_bytes, pcops_stream_t stream) {
  if (B < 0 || H <= 0) return PCOPS_ERR_INVALID;
  int rc = check_common(B * H, Lq, Lk, D, dtype);
  if (rc) return rc;
  const bool sums = dq_colsum || dk_colsum || dv_colsum;
  if (sums && !(dq_colsum && dk_colsum && dv_colsum)) return PCOPS_ERR_INVALID;
  if (sums && (dtype != 1 || use_v1())) return PCOPS_ERR_UNSUPPORTED;
  if (workspace_bytes < pcops_attention_bwd_fused_workspace_bytes(B, H, Lq, Lk, D, dtype)) return PCOPS_ERR_WORKSPACE;
  const bool ds = dtype == 1 && !use_v1() && D >= 96 && ds_path_on();
  if (!ds) {
    if (!sums)
      return pcops_attention_backward(q, k, v, o, dout, lse, dq, dk, dv, B, H, Lq, Lk, D, scale, dtype,
                                      PC_ATTN_STRIDE_ARGS, workspace, workspace_bytes, stream);
    rc = pcops_attention_bwd_dq_delta_colsum(q, k, v, o, dout, lse, dq, dq_colsum, B, H, Lq, Lk, D, scale, dtype,
                                             PC_ATTN_STRIDE_ARGS, workspace, workspace_bytes, stream);
    if (rc) return rc;
    return pcops_attention_bwd_dkv_colsum(q, k, v, dout, lse, dk, dv, dk_colsum, dv_colsum, B, H, Lq, Lk, D, scale,
                                          dtype, PC_ATTN_STRIDE_ARGS, workspace, workspace_bytes, stream);
  }
  const int BH = B * H;
  hipStream_t s = (hipStream_t)stream;
  if (BH == 0) return PCOPS_OK;
  if (Lq == 0 || Lk == 0) {  // empty sums; dK / dV (Lq == 0) are zero
    if (Lq == 0 && Lk > 0) {
      rc = pcops_attention_backward(q, k, v, o, dout, lse, dq, dk, dv, B, H, Lq, Lk, D, scale, dtype,
                                    PC_ATTN_STRIDE_ARGS, workspace, workspace_bytes, stream);
      if (rc) return rc;
    }
    if (sums)
      for (float *p : {dq_colsum, dk_colsum, dv_colsum})
        if (pc_memset_async(p, 0, (size_t)H * D * sizeof(float), s) != hipSuccess) return PCOPS_ERR_LAUNCH;
    return PCOPS_OK;
  }
  if (!q || !k || !v || !o || !dout || !lse || !dq || !dk || !dv || !workspace) return PCOPS_ERR_INVALID;
  if (!aligned_ok(q, q_sb, q_sh, q_srow, 2) || !aligned_ok(k, k_sb, k_sh, k_srow, 2) ||
      !aligned_ok(v, v_sb, v_sh, v_srow, 2) || !aligned_ok(dout, o_sb, o_sh, o_srow, 2) ||
      !aligned_ok(o, o_sb, o_sh, o_srow, 2) || !aligned_ok(dq, q_sb, q_sh, q_srow, 2) ||
      !aligned_ok(dk, k_sb, k_sh, k_srow, 2) || !aligned_ok(dv, v_sb, v_sh, v_srow, 2))
    return PCOPS_ERR_UNSUPPORTED;
  const Strides st{PC_ATTN_STRIDE_ARGS, H};
  float *delta = (float *)workspace;
  const long long rk = (Lk + 127) / 128, rq = (Lq + 127) / 128;
  float *parts = (float *)((char *)workspace + delta_bytes(B, H, Lq));
  __bf16 *dsT = (__bf16 *)((char *)parts + ((((unsigned long long)BH * (rq + 2 * rk) * D * sizeof(float)) + 255) &
                                            ~255ull));
  ColPart cpkv, cpq;
  cpkv.a = parts;
  cpkv.b = parts + (long long)BH * rk * D;
  cpq.a = parts + 2ll * BH * rk * D;
  ColPart *pkv = sums ? &cpkv : nullptr, *pq = sums ? &cpq : nullptr;
  switch (D) {
    case 96:
      rc = sums ? launch_bwd_ds<96, true>(q, k, v, o, dout, lse, dq, dk, dv, BH, Lq, Lk, scale, st, s, delta, dsT, pq, pkv)
                : launch_bwd_ds<96, false>(q, k, v, o, dout, lse, dq, dk, dv, BH, Lq, Lk, scale, st, s, delta, dsT, pq, pkv);
      break;
    case 128:
      rc = sums ? launch_bwd_ds<128, true>(q, k, v, o, dout, lse, dq, dk, dv, BH, Lq, Lk, scale, st, s, delta, dsT, pq, pkv)
                : launch_bwd_ds<128, false>(q, k, v, o, dout, lse, dq, dk, dv, BH, Lq, Lk, scale, st, s, delta, dsT, pq, pkv);
      break;
    default:
      return PCOPS_ERR_UNSUPPORTED;
  }
  if (rc || !sums) return rc;
  rc = launch_colsum_reduce(cpkv.a, dk_colsum, cpkv.b, dv_colsum, B * cpkv.nrb, H * D, s);
  if (rc) return rc;
  return launch_colsum_reduce(cpq.a, dq_colsum, nullptr, nullptr, B * cpq.nrb, H * D, s);
}
