// Skinny 1x1 convolutions of EdgeConv (models/model_utils.py:847-881): the three Conv2d(k=1) of
// gcn_1 (6 -> 32, 32 -> 32, 32 -> 64 channels) run over B x N x k = 1 M edge rows.  As GEMMs they
// are (1 M x K) . (K x N) with K, N <= 64: pure streaming work (read K, write N bf16 per row).  The
// side stream's rocBLAS picks 32 x 256 output tiles for them -- 7/8 of every tile outside N = 32 --
// and ran them at 105-165 us; here a wave owns 32 rows and keeps the whole weight in registers.
//
//   y[t][n] = bf16( sum_k x[t][k] A[n][k] + bias[n] )     x (rows, K), A (N, K), y (rows, N) bf16
//
// Forward: A = the conv weight (Cout, Cin).  Input gradient: A = W^T (the host passes it
// transposed), x = the output gradient, no bias.  One v_mfma_f32_32x32x16_bf16 per (32 output
// channels, 16 of K): A is the matrix operand whose rows are output channels (fragments loaded
// once per wave), x^T the other, so a lane's 8 K values are 16 contiguous bytes of its row and a
// lane ends with 16 output channels of ONE row (acc_row map) -- stored as four 8-byte runs.
// Products of bf16 values are exact in fp32; the sum over K runs in the MFMA's fp32 accumulate
// (the same instruction family the GEMM libraries use for bf16; the order inside a 16-wide step
// is the hardware's), bias added in fp32, one rounding to bf16.
#include "common.h"

namespace {

typedef __bf16 sk_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 sk_bf16x4 __attribute__((ext_vector_type(4)));
typedef float sk_f32x16 __attribute__((ext_vector_type(16)));

// row i of the accumulator held in register r of lane half h (32x32 MFMA C/D layout)
__device__ __forceinline__ int sk_acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// K values [k0, k0 + 8) of a row of K bf16, zero past K.  K % 8 == 0: one 16-B load (row bases
// 16-B aligned: host-checked); otherwise (K = 6) 4-B pairs
template <int K>
__device__ __forceinline__ sk_bf16x8 sk_load8(const __bf16 *row, int k0) {
  sk_bf16x8 v;
  if constexpr (K % 8 == 0) {
    if (k0 < K) return *reinterpret_cast<const sk_bf16x8 *>(row + k0);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (__bf16)0.f;
    return v;
  } else {
    static_assert(K % 2 == 0, "K must be even");
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      if (k0 + e < K) {
        const unsigned u = *reinterpret_cast<const unsigned *>(row + k0 + e);
        typedef __bf16 b2 __attribute__((ext_vector_type(2)));
        const b2 p = __builtin_bit_cast(b2, u);
        v[e] = p[0];
        v[e + 1] = p[1];
      } else {
        v[e] = (__bf16)0.f;
        v[e + 1] = (__bf16)0.f;
      }
    }
    return v;
  }
}

template <int K, int NT, bool BIAS>
__global__ __launch_bounds__(256) void linear_skinny_kernel(const __bf16 *__restrict__ x, long long rows,
                                                            const __bf16 *__restrict__ A,
                                                            const __bf16 *__restrict__ bias, __bf16 *__restrict__ y) {
  constexpr int KC = (K + 15) / 16, N = NT * 32;
  const int l = threadIdx.x & 63, h = l >> 5, c32 = l & 31;
  // the weight's fragments, for the whole kernel: af[ct][kc][e] = A[32 ct + c32][16 kc + 8 h + e]; element
  // loads (once per wave): A may be a view into the flat bf16 parameter buffer at any 2-byte offset
  sk_bf16x8 af[NT][KC];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = 16 * kc + 8 * h + e;
        af[ct][kc][e] = k < K ? A[(size_t)(32 * ct + c32) * K + k] : (__bf16)0.f;
      }
  float bv[NT][16];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) bv[ct][r] = BIAS ? (float)bias[32 * ct + sk_acc_row(r, h)] : 0.f;
  const long long ntile = (rows + 31) / 32;
  for (long long tile = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); tile < ntile; tile += (long long)gridDim.x * 4) {
    const long long t = tile * 32 + c32;
    const bool ok = t < rows;
    const __bf16 *xr = x + (size_t)(ok ? t : rows - 1) * K;
    sk_bf16x8 bf[KC];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) bf[kc] = sk_load8<K>(xr, 16 * kc + 8 * h);
    sk_f32x16 acc[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) {
      acc[ct] = sk_f32x16{};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc)
        acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ct][kc], bf[kc], acc[ct], 0, 0, 0);
    }
    if (ok) {
      __bf16 *yr = y + (size_t)t * N;
#pragma unroll
      for (int ct = 0; ct < NT; ++ct)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          sk_bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (__bf16)(acc[ct][4 * g + e] + bv[ct][4 * g + e]);
          // registers 4g..4g+3 are channels 32 ct + 8 g + 4 h + 0..3
          *reinterpret_cast<sk_bf16x4 *>(yr + 32 * ct + 8 * g + 4 * h) = o;
        }
    }
  }
}

template <int K, int NT>
void launch_skinny(const __bf16 *x, long long rows, const __bf16 *A, const __bf16 *bias, __bf16 *y, hipStream_t s) {
  const long long tiles = (rows + 31) / 32;
  long long blocks = (tiles + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  if (bias)
    hipLaunchKernelGGL((linear_skinny_kernel<K, NT, true>), dim3((unsigned)blocks), dim3(256), 0, s, x, rows, A, bias, y);
  else
    hipLaunchKernelGGL((linear_skinny_kernel<K, NT, false>), dim3((unsigned)blocks), dim3(256), 0, s, x, rows, A, bias, y);
}

}  // namespace

extern "C" int pcops_linear_skinny(const void *x, long long rows, int K, const void *A, const void *bias, void *y,
                                   int N, pcops_stream_t stream) {
  if (rows < 0 || K <= 0 || N <= 0) return PCOPS_ERR_INVALID;
  if (rows == 0) return PCOPS_OK;
  if (!x || !A || !y) return PCOPS_ERR_INVALID;
  if (N % 32 || N > 64) return PCOPS_ERR_UNSUPPORTED;
  const unsigned long long al = reinterpret_cast<unsigned long long>(x) | reinterpret_cast<unsigned long long>(y);
  if ((K % 8 == 0 && (al & 15)) || (al & 7) || (reinterpret_cast<unsigned long long>(A) & 1) ||
      (bias && (reinterpret_cast<unsigned long long>(bias) & 1)))
    return PCOPS_ERR_UNSUPPORTED;
  const __bf16 *xb = (const __bf16 *)x, *Ab = (const __bf16 *)A, *bb = (const __bf16 *)bias;
  __bf16 *yb = (__bf16 *)y;
  hipStream_t s = (hipStream_t)stream;
#define SK_CASE(K_)                                         \
  case K_:                                                  \
    if (N == 32)                                            \
      launch_skinny<K_, 1>(xb, rows, Ab, bb, yb, s);        \
    else                                                    \
      launch_skinny<K_, 2>(xb, rows, Ab, bb, yb, s);        \
    break;
  switch (K) {
    SK_CASE(6)
    SK_CASE(32)
    SK_CASE(64)
    default:
      return PCOPS_ERR_UNSUPPORTED;
  }
#undef SK_CASE
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
