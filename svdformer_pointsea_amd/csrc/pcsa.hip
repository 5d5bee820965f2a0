// Point Cloud Spectral Adapter apply step (models/model_utils.py:358-430,
// PCSA.forward) for gfx950.
//
// The reference permutes the (B, C, S, K) neighbourhood features to
// (B*S*C, K), multiplies by the DCT-II basis, scales by per-(b, s) frequency
// gates, multiplies by the inverse basis and permutes back: two thin GEMMs
// (N = K = 16) and four full-size copies per call, twice that in backward.
// Per (b, s) patch the whole chain is one K x K matrix,
//     out = M x,   M = D^T diag(g) D   (D the DCT basis, g the gates),
// so here one pass reads each patch once and writes it once.  The features
// stay in the conv output's channels_last memory order (B, S, K, C): a patch
// is K*C contiguous elements, a thread owns a channel column (coalesced over
// channels).  Backward: dx = M^T dout and dg[k] = sum_c (D dout)[k][c] (D x)[k][c]
// (a per-patch channel reduction in LDS).  fp32 accumulation; x / out in fp32
// or bf16 (dtype code 0 / 1); gates fp32 or bf16; the basis is passed in (the
// reference builds it in the features' dtype).
#include <cstdlib>

#include "common.h"

namespace {

__device__ __forceinline__ float ldv(const void *p, int dt, long long i) {
  return dt == 0 ? reinterpret_cast<const float *>(p)[i] : (float)reinterpret_cast<const __bf16 *>(p)[i];
}
__device__ __forceinline__ void stv(void *p, int dt, long long i, float v) {
  if (dt == 0)
    reinterpret_cast<float *>(p)[i] = v;
  else
    reinterpret_cast<__bf16 *>(p)[i] = (__bf16)v;
}

// one block per (b, s) patch; thread c < C owns channel c of the patch.
// M (K x K) is built in LDS from the gates and the basis.
template <int K>
__global__ __launch_bounds__(256) void pcsa_fwd_kernel(const void *__restrict__ x, int xdt,
                                                       const void *__restrict__ gates, int gdt,
                                                       const float *__restrict__ basis, int C, void *__restrict__ out) {
  __shared__ float sD[K * K], sM[K * K], sg[K];
  const long long p = blockIdx.x;  // patch = b * S + s
  const int t = threadIdx.x;
  for (int i = t; i < K * K; i += blockDim.x) sD[i] = basis[i];
  if (t < K) sg[t] = ldv(gates, gdt, p * K + t);
  __syncthreads();
  for (int i = t; i < K * K; i += blockDim.x) {  // M[a][j] = sum_k D[k][a] g[k] D[k][j]
    const int a = i / K, j = i % K;
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) m = __builtin_fmaf(sD[k * K + a] * sg[k], sD[k * K + j], m);
    sM[i] = m;
  }
  __syncthreads();
  const long long base = p * K * C;
  for (int c = t; c < C; c += blockDim.x) {
    float v[K];
#pragma unroll
    for (int j = 0; j < K; ++j) v[j] = ldv(x, xdt, base + (long long)j * C + c);
#pragma unroll
    for (int a = 0; a < K; ++a) {
      float o = 0.f;
#pragma unroll
      for (int j = 0; j < K; ++j) o = __builtin_fmaf(sM[a * K + j], v[j], o);
      stv(out, xdt, base + (long long)a * C + c, o);
    }
  }
}

template <int K>
__global__ __launch_bounds__(256) void pcsa_bwd_kernel(const void *__restrict__ x, int xdt,
                                                       const void *__restrict__ dout, int ddt,
                                                       const void *__restrict__ gates, int gdt,
                                                       const float *__restrict__ basis, int C, void *__restrict__ dx,
                                                       void *__restrict__ dgates) {
  __shared__ float sD[K * K], sM[K * K], sg[K];
  __shared__ float sred[K][8];
  const long long p = blockIdx.x;
  const int t = threadIdx.x;
  for (int i = t; i < K * K; i += blockDim.x) sD[i] = basis[i];
  if (t < K) sg[t] = ldv(gates, gdt, p * K + t);
  __syncthreads();
  for (int i = t; i < K * K; i += blockDim.x) {
    const int a = i / K, j = i % K;
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) m = __builtin_fmaf(sD[k * K + a] * sg[k], sD[k * K + j], m);
    sM[i] = m;
  }
  __syncthreads();
  const long long base = p * K * C;
  float dg[K];
#pragma unroll
  for (int k = 0; k < K; ++k) dg[k] = 0.f;
  for (int c = t; c < C; c += blockDim.x) {
    float xv[K], gv[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      xv[j] = ldv(x, xdt, base + (long long)j * C + c);
      gv[j] = ldv(dout, ddt, base + (long long)j * C + c);
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {  // dx = M^T dout
      float o = 0.f;
#pragma unroll
      for (int a = 0; a < K; ++a) o = __builtin_fmaf(sM[a * K + j], gv[a], o);
      stv(dx, xdt, base + (long long)j * C + c, o);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {  // (D dout)[k] * (D x)[k]
      float dd = 0.f, dxs = 0.f;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        dd = __builtin_fmaf(sD[k * K + j], gv[j], dd);
        dxs = __builtin_fmaf(sD[k * K + j], xv[j], dxs);
      }
      dg[k] = __builtin_fmaf(dd, dxs, dg[k]);
    }
  }
  // channel reduction of dg: wave DPP-free shuffle sums, then 8-wave LDS sum
  const int lane = t & 63, w = t >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float v = dg[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) sred[k][w] = v;
  }
  __syncthreads();
  if (t < K) {
    float s = 0.f;
    const int nw = (blockDim.x + 63) >> 6;
    for (int i = 0; i < nw; ++i) s += sred[t][i];
    stv(dgates, gdt, p * K + t, s);
  }
}

// ---- wave-per-patch form (C = 64 * CPT): the lane owns CPT adjacent channels
// (one 2- or 4-element load per neighbour) and the patch index is wave-uniform
// (the gates g are scalar loads); no K x K matrix -- the chain is applied as
// the reference associates it, out = D^T (g o (D x)); D is read with scalar
// loads (uniform) and held in SGPRs (for K = 16 the compiler parks ~260 of
// them in VGPR lanes; staging D in LDS instead made it hoist the 256
// broadcast values into VGPRs and spill to scratch).  Backward: u = D dout, v = D x, dx = D^T (g o u),
// dg[k] = sum_c u[k] v[k] (wave DPP sums).
template <int K, int CPT>
__device__ __forceinline__ void ld_cols(float (&v)[K][CPT], const void *p, int dt, long long base, int C, int c0) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const long long e = base + (long long)j * C + c0;
    if (dt == 0) {
#pragma unroll
      for (int c = 0; c < CPT; ++c) v[j][c] = reinterpret_cast<const float *>(p)[e + c];
    } else {
#pragma unroll
      for (int c = 0; c < CPT; ++c) v[j][c] = (float)reinterpret_cast<const __bf16 *>(p)[e + c];
    }
  }
}
template <int K, int CPT>
__device__ __forceinline__ void st_cols(void *p, int dt, long long base, int C, int c0, const float (&v)[K][CPT]) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const long long e = base + (long long)j * C + c0;
#pragma unroll
    for (int c = 0; c < CPT; ++c) stv(p, dt, e + c, v[j][c]);
  }
}
// y[k][c] = sum_j D[k][j] x[j][c]   (D row-major K x K, uniform)
template <int K, int CPT>
__device__ __forceinline__ void dct_apply(float (&y)[K][CPT], const float *__restrict__ D, const float (&x)[K][CPT]) {
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < K; ++j) a = __builtin_fmaf(D[k * K + j], x[j][c], a);
      y[k][c] = a;
    }
}
// o[j][c] = sum_k D[k][j] g[k] y[k][c]
template <int K, int CPT>
__device__ __forceinline__ void idct_gate(float (&o)[K][CPT], const float *__restrict__ D, const float (&g)[K],
                                          const float (&y)[K][CPT]) {
  float t[K][CPT];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int c = 0; c < CPT; ++c) t[k][c] = g[k] * y[k][c];
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) a = __builtin_fmaf(D[k * K + j], t[k][c], a);
      o[j][c] = a;
    }
}

template <int K, int CPT>
__global__ __launch_bounds__(256) void pcsa_fwd_wave_kernel(const void *__restrict__ x, int xdt,
                                                            const void *__restrict__ gates, int gdt,
                                                            const float *__restrict__ basis, int patches, int C,
                                                            void *__restrict__ out) {
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const long long p = (long long)blockIdx.x * 4 + w;
  if (p >= patches) return;
  const int c0 = (threadIdx.x & 63) * CPT;
  float g[K];
#pragma unroll
  for (int k = 0; k < K; ++k) g[k] = ldv(gates, gdt, p * K + k);
  const long long base = p * K * C;
  float xv[K][CPT], y[K][CPT];
  ld_cols<K, CPT>(xv, x, xdt, base, C, c0);
  dct_apply<K, CPT>(y, basis, xv);
  idct_gate<K, CPT>(xv, basis, g, y);
  st_cols<K, CPT>(out, xdt, base, C, c0, xv);
}

template <int K, int CPT>
__global__ __launch_bounds__(256) void pcsa_bwd_wave_kernel(const void *__restrict__ x, int xdt,
                                                            const void *__restrict__ dout, int ddt,
                                                            const void *__restrict__ gates, int gdt,
                                                            const float *__restrict__ basis, int patches, int C,
                                                            void *__restrict__ dx, void *__restrict__ dgates) {
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const long long p = (long long)blockIdx.x * 4 + w;
  if (p >= patches) return;
  const int lane = threadIdx.x & 63, c0 = lane * CPT;
  float g[K];
#pragma unroll
  for (int k = 0; k < K; ++k) g[k] = ldv(gates, gdt, p * K + k);
  const long long base = p * K * C;
  float a[K][CPT], u[K][CPT];
  ld_cols<K, CPT>(a, dout, ddt, base, C, c0);
  dct_apply<K, CPT>(u, basis, a);          // u = D dout
  ld_cols<K, CPT>(a, x, xdt, base, C, c0);
  float dg[K];
  {
    float v[K][CPT];
    dct_apply<K, CPT>(v, basis, a);        // v = D x
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < CPT; ++c) s = __builtin_fmaf(u[k][c], v[k][c], s);
      dg[k] = s;
    }
  }
  idct_gate<K, CPT>(a, basis, g, u);       // dx = D^T (g o u)
  st_cols<K, CPT>(dx, xdt, base, C, c0, a);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float t = wave_sum_f32(dg[k]);
    if (lane == 0) stv(dgates, gdt, p * K + k, t);
  }
}

// ---- MFMA form for bf16 features, K = 16 (the models' PCSA: C = 128 / 256, K = 16).
// Per (b, s) patch the chain is two 16x16 matrix products per 16-channel block,
// on v_mfma_f32_16x16x16_bf16 with the rounding the reference's autocast chain
// applies (model_utils.py:413-430 under bf16 autocast: spec = bf16(x @ D^T),
// bf16(spec * gates), out = bf16(spec_g @ D)):
//   Y = D X_blk (fp32 accumulate) -> Z = bf16(bf16(Y) g) -> O = D^T Z -> bf16.
// Operand maps (16x16x16 bf16): lane l holds A[l&15][4(l>>4)+j], B[4(l>>4)+j][l&15]
// and the result D[4(l>>4)+j][l&15], j = 0..3 -- so the accumulator of the
// first product IS the B operand of the second (no lane movement).  X's B
// fragments come from an LDS image of the patch by ds_read_b64_tr_b16 (lane
// 4r+c of a 16-lane group addresses row r, columns 4c..4c+3 of its 4x16 block
// and receives one column); rows padded by 32 B so a 32-lane half's 8 rows hit
// 32 distinct banks.  One wave per patch, 4 patches per block.
// Backward: u = D dout, v = D x (both rounded to bf16 as the reference stores
// them), dgates[k] = sum_c bf16(u v) (the RepeatBackward sum, fp32), dx = D^T bf16(u g).
typedef short pc_short4 __attribute__((ext_vector_type(4)));
typedef float pc_f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 pc_bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 pc_bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bfr(float v) { return (float)(__bf16)v; }  // round to bf16 and back

__device__ __forceinline__ pc_short4 bf4(float a, float b, float c, float d) {
  const pc_bf16x4 v = {(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
  return __builtin_bit_cast(pc_short4, v);
}

// stage the 16 x C bf16 patch at src (rows C apart) into a padded LDS image
template <int C>
__device__ __forceinline__ void pcsa_stage(__bf16 *img, const __bf16 *src, int lane) {
  constexpr int RS = C + 16;
#pragma unroll
  for (int t = lane; t < 2 * C; t += 64) {  // 16 rows x C/8 chunks of 8
    const int row = t / (C / 8), ch = t % (C / 8);
    *reinterpret_cast<pc_bf16x8 *>(img + row * RS + ch * 8) = *reinterpret_cast<const pc_bf16x8 *>(src + row * C + ch * 8);
  }
}

// B fragment of channel block cb: rows 4(l>>4)..+3, column 16 cb + (l&15)
template <int C>
__device__ __forceinline__ pc_short4 pcsa_bfrag(const __bf16 *img, int lane, int cb) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int RS = C + 16;
  typedef __attribute__((address_space(3))) pc_short4 lds_s4;
  const int g = lane >> 4, i = lane & 15;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(img + (4 * g + (i >> 2)) * RS + 16 * cb + 4 * (i & 3)));
#else
  return pc_short4{};
#endif
}

template <int C>
__global__ __launch_bounds__(256) void pcsa_fwd_mfma_kernel(const __bf16 *__restrict__ x, const void *__restrict__ gates,
                                                            int gdt, const float *__restrict__ basis, int patches,
                                                            __bf16 *__restrict__ out) {
  constexpr int K = 16, RS = C + 16;
  __shared__ __attribute__((aligned(16))) __bf16 simg[4][K * RS];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, q = l >> 4, c = l & 15;
  const long long p = (long long)blockIdx.x * 4 + w;
  if (p >= patches) return;  // whole waves only; no block barrier below
  const pc_short4 da = bf4(basis[c * K + 4 * q], basis[c * K + 4 * q + 1], basis[c * K + 4 * q + 2],
                           basis[c * K + 4 * q + 3]);                            // D[c][4q + j]
  const pc_short4 dt = bf4(basis[(4 * q) * K + c], basis[(4 * q + 1) * K + c], basis[(4 * q + 2) * K + c],
                           basis[(4 * q + 3) * K + c]);                          // D[4q + j][c]
  float g[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) g[i] = ldv(gates, gdt, p * K + 4 * q + i);
  __bf16 *img = simg[w];
  pcsa_stage<C>(img, x + p * K * C, l);
  __bf16 *ob = out + p * K * C;
#pragma unroll
  for (int cb = 0; cb < C / 16; ++cb) {
    const pc_f32x4 y = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(da, pcsa_bfrag<C>(img, l, cb), pc_f32x4{}, 0, 0, 0);
    const pc_short4 z = bf4(bfr(y[0]) * g[0], bfr(y[1]) * g[1], bfr(y[2]) * g[2], bfr(y[3]) * g[3]);
    const pc_f32x4 o = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(dt, z, pc_f32x4{}, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) ob[(4 * q + i) * C + 16 * cb + c] = (__bf16)o[i];
  }
}

template <int C>
__global__ __launch_bounds__(256) void pcsa_bwd_mfma_kernel(const __bf16 *__restrict__ x, const __bf16 *__restrict__ dout,
                                                            const void *__restrict__ gates, int gdt,
                                                            const float *__restrict__ basis, int patches,
                                                            __bf16 *__restrict__ dx, void *__restrict__ dgates) {
  constexpr int K = 16, RS = C + 16;
  __shared__ __attribute__((aligned(16))) __bf16 simg[4][2][K * RS];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, q = l >> 4, c = l & 15;
  const long long p = (long long)blockIdx.x * 4 + w;
  if (p >= patches) return;
  const pc_short4 da = bf4(basis[c * K + 4 * q], basis[c * K + 4 * q + 1], basis[c * K + 4 * q + 2],
                           basis[c * K + 4 * q + 3]);
  const pc_short4 dt = bf4(basis[(4 * q) * K + c], basis[(4 * q + 1) * K + c], basis[(4 * q + 2) * K + c],
                           basis[(4 * q + 3) * K + c]);
  float g[4], dg[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) g[i] = ldv(gates, gdt, p * K + 4 * q + i);
  __bf16 *ix = simg[w][0], *id = simg[w][1];
  pcsa_stage<C>(ix, x + p * K * C, l);
  pcsa_stage<C>(id, dout + p * K * C, l);
  __bf16 *ob = dx + p * K * C;
#pragma unroll
  for (int cb = 0; cb < C / 16; ++cb) {
    const pc_f32x4 u = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(da, pcsa_bfrag<C>(id, l, cb), pc_f32x4{}, 0, 0, 0);
    const pc_f32x4 v = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(da, pcsa_bfrag<C>(ix, l, cb), pc_f32x4{}, 0, 0, 0);
    float ub[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ub[i] = bfr(u[i]);
      dg[i] += bfr(ub[i] * bfr(v[i]));
    }
    const pc_short4 s = bf4(ub[0] * g[0], ub[1] * g[1], ub[2] * g[2], ub[3] * g[3]);
    const pc_f32x4 o = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(dt, s, pc_f32x4{}, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) ob[(4 * q + i) * C + 16 * cb + c] = (__bf16)o[i];
  }
  // sum over the 16 channel lanes of each 16-lane group (rows 4q .. 4q+3)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) dg[i] += __shfl_xor(dg[i], o, 64);
    if (c == 0) stv(dgates, gdt, p * K + 4 * q + i, dg[i]);
  }
}

// A/B: PCOPS_PCSA_MFMA=0 keeps the fp32-VALU kernels for bf16 features too
bool pcsa_mfma(int K, int C, int xdt) {
  static const bool off = [] {
    const char *e = getenv("PCOPS_PCSA_MFMA");
    return e && e[0] == '0';
  }();
  return !off && xdt == 1 && K == 16 && (C == 64 || C == 128 || C == 256);
}

// A/B: PCOPS_PCSA_V1=1 keeps the block-per-patch kernels
bool pcsa_wave(int K, int C) {
  static const bool v1 = [] {
    const char *e = getenv("PCOPS_PCSA_V1");
    return e && e[0] == '1';
  }();
  return !v1 && K <= 16 && (C == 64 || C == 128 || C == 256);
}

}  // namespace

extern "C" int pcops_pcsa_forward(const void *x, int x_dtype, const void *gates, int gates_dtype, const float *basis,
                                  int patches, int K, int C, void *out, pcops_stream_t stream) {
  if (patches < 0 || C <= 0 || (K != 4 && K != 8 && K != 16 && K != 32)) return PCOPS_ERR_INVALID;
  if (patches == 0) return PCOPS_OK;
  if (!x || !gates || !basis || !out || (x_dtype & ~1) || (gates_dtype & ~1)) return PCOPS_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  if (pcsa_mfma(K, C, x_dtype)) {
    const dim3 grid((patches + 3) / 4);
#define PCSA_FM(CC)                                                                                             \
  if (C == CC) {                                                                                              \
    hipLaunchKernelGGL(pcsa_fwd_mfma_kernel<CC>, grid, dim3(256), 0, s, (const __bf16 *)x, gates, gates_dtype, \
                       basis, patches, (__bf16 *)out);                                                          \
    PC_CHECK_LAUNCH();                                                                                        \
    return PCOPS_OK;                                                                                          \
  }
    PCSA_FM(64) PCSA_FM(128) PCSA_FM(256)
#undef PCSA_FM
  }
  if (pcsa_wave(K, C) && C <= 128) {  // C = 256 forward: the block form measured faster (0.110 vs 0.133 ms)
    const dim3 grid((patches + 3) / 4);
#define PCSA_FW(KK, CC)                                                                                        \
  if (K == KK && C == 64 * CC) {                                                                               \
    hipLaunchKernelGGL((pcsa_fwd_wave_kernel<KK, CC>), grid, dim3(256), 0, s, x, x_dtype, gates, gates_dtype, \
                       basis, patches, C, out);                                                                \
    PC_CHECK_LAUNCH();                                                                                         \
    return PCOPS_OK;                                                                                           \
  }
    PCSA_FW(4, 1) PCSA_FW(4, 2) PCSA_FW(4, 4) PCSA_FW(8, 1) PCSA_FW(8, 2) PCSA_FW(8, 4)
    PCSA_FW(16, 1) PCSA_FW(16, 2) PCSA_FW(16, 4)
#undef PCSA_FW
  }
  const int threads = C >= 256 ? 256 : (C + 63) / 64 * 64;
  switch (K) {
    case 4: hipLaunchKernelGGL(pcsa_fwd_kernel<4>, dim3(patches), dim3(threads), 0, s, x, x_dtype, gates, gates_dtype, basis, C, out); break;
    case 8: hipLaunchKernelGGL(pcsa_fwd_kernel<8>, dim3(patches), dim3(threads), 0, s, x, x_dtype, gates, gates_dtype, basis, C, out); break;
    case 16: hipLaunchKernelGGL(pcsa_fwd_kernel<16>, dim3(patches), dim3(threads), 0, s, x, x_dtype, gates, gates_dtype, basis, C, out); break;
    default: hipLaunchKernelGGL(pcsa_fwd_kernel<32>, dim3(patches), dim3(threads), 0, s, x, x_dtype, gates, gates_dtype, basis, C, out); break;
  }
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_pcsa_backward(const void *x, int x_dtype, const void *dout, int dout_dtype, const void *gates,
                                   int gates_dtype, const float *basis, int patches, int K, int C, void *dx,
                                   void *dgates, pcops_stream_t stream) {
  if (patches < 0 || C <= 0 || (K != 4 && K != 8 && K != 16 && K != 32)) return PCOPS_ERR_INVALID;
  if (patches == 0) return PCOPS_OK;
  if (!x || !dout || !gates || !basis || !dx || !dgates || (x_dtype & ~1) || (dout_dtype & ~1) || (gates_dtype & ~1))
    return PCOPS_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  if (pcsa_mfma(K, C, x_dtype) && dout_dtype == 1) {
    const dim3 grid((patches + 3) / 4);
#define PCSA_BM(CC)                                                                                              \
  if (C == CC) {                                                                                               \
    hipLaunchKernelGGL(pcsa_bwd_mfma_kernel<CC>, grid, dim3(256), 0, s, (const __bf16 *)x, (const __bf16 *)dout, \
                       gates, gates_dtype, basis, patches, (__bf16 *)dx, dgates);                              \
    PC_CHECK_LAUNCH();                                                                                         \
    return PCOPS_OK;                                                                                           \
  }
    PCSA_BM(64) PCSA_BM(128) PCSA_BM(256)
#undef PCSA_BM
  }
  if (pcsa_wave(K, C)) {
    const dim3 grid((patches + 3) / 4);
#define PCSA_BW(KK, CC)                                                                                        \
  if (K == KK && C == 64 * CC) {                                                                               \
    hipLaunchKernelGGL((pcsa_bwd_wave_kernel<KK, CC>), grid, dim3(256), 0, s, x, x_dtype, dout, dout_dtype,   \
                       gates, gates_dtype, basis, patches, C, dx, dgates);                                     \
    PC_CHECK_LAUNCH();                                                                                         \
    return PCOPS_OK;                                                                                           \
  }
    PCSA_BW(4, 1) PCSA_BW(4, 2) PCSA_BW(4, 4) PCSA_BW(8, 1) PCSA_BW(8, 2) PCSA_BW(8, 4)
    PCSA_BW(16, 1) PCSA_BW(16, 2) PCSA_BW(16, 4)
#undef PCSA_BW
  }
  const int threads = C >= 256 ? 256 : (C + 63) / 64 * 64;
#define PCSA_BWD(KK)                                                                                          \
  hipLaunchKernelGGL(pcsa_bwd_kernel<KK>, dim3(patches), dim3(threads), 0, s, x, x_dtype, dout, dout_dtype, gates, \
                     gates_dtype, basis, C, dx, dgates)
  switch (K) {
    case 4: PCSA_BWD(4); break;
    case 8: PCSA_BWD(8); break;
    case 16: PCSA_BWD(16); break;
    default: PCSA_BWD(32); break;
  }
#undef PCSA_BWD
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
