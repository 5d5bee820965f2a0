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

}  // namespace

extern "C" int pcops_pcsa_forward(const void *x, int x_dtype, const void *gates, int gates_dtype, const float *basis,
                                  int patches, int K, int C, void *out, pcops_stream_t stream) {
  if (patches < 0 || C <= 0 || (K != 4 && K != 8 && K != 16 && K != 32)) return PCOPS_ERR_INVALID;
  if (patches == 0) return PCOPS_OK;
  if (!x || !gates || !basis || !out || (x_dtype & ~1) || (gates_dtype & ~1)) return PCOPS_ERR_INVALID;
  const int threads = C >= 256 ? 256 : (C + 63) / 64 * 64;
  hipStream_t s = (hipStream_t)stream;
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
  const int threads = C >= 256 ? 256 : (C + 63) / 64 * 64;
  hipStream_t s = (hipStream_t)stream;
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
