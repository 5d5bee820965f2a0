// Shared device helpers for the gfx950 (CDNA4) point-cloud kernels.
// Wave size is 64 everywhere (hard-coded, never warpSize-derived).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pcops.h"

#define PC_WAVE 64

// nvcc-contraction order of the reference's `a*a + b*b + c*c` (see
// oracle/pcops_oracle.c header): fmaf(c,c, fmaf(a,a, b*b)).  All files are
// compiled with -ffp-contract=off so these explicit fmas are the only fusion.
__device__ __forceinline__ float sqd3(float a, float b, float c) {
  return __builtin_fmaf(c, c, __builtin_fmaf(a, a, b * b));
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// ---- wave-level reductions (DPP / swizzle lowered by the compiler) ----
__device__ __forceinline__ float wave_max_f32(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, PC_WAVE));
  return v;
}
__device__ __forceinline__ float wave_min_f32(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fminf(v, __shfl_xor(v, off, PC_WAVE));
  return v;
}
__device__ __forceinline__ int wave_min_i32(int v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = min(v, __shfl_xor(v, off, PC_WAVE));
  return v;
}
__device__ __forceinline__ float wave_sum_f32(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, PC_WAVE);
  return v;
}

// Among the lanes set in `mask`, the one whose lane number has the smallest
// bit-reversal (prefer bit0 == 0, then bit1 == 0, ...).  Scalar-only work.
__device__ __forceinline__ int min_bitrev_lane(uint64_t mask) {
  const uint64_t zero_bit[6] = {0x5555555555555555ull, 0x3333333333333333ull, 0x0F0F0F0F0F0F0F0Full,
                                0x00FF00FF00FF00FFull, 0x0000FFFF0000FFFFull, 0x00000000FFFFFFFFull};
#pragma unroll
  for (int b = 0; b < 6; ++b) {
    const uint64_t m = mask & zero_bit[b];
    mask = m ? m : mask;
  }
  return (int)__builtin_ctzll(mask);
}

__device__ __forceinline__ unsigned bitrev_bits(unsigned v, int bits) {
  return bits == 0 ? 0u : (__builtin_bitreverse32(v) >> (32 - bits));
}

#define PC_CHECK_LAUNCH()                               \
  do {                                                  \
    hipError_t _e = hipGetLastError();                  \
    if (_e != hipSuccess) return PCOPS_ERR_LAUNCH;      \
  } while (0)
