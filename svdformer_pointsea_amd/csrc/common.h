// Shared device helpers for the gfx950 (CDNA4) point-cloud kernels.
// Wave size is 64 everywhere (hard-coded, never warpSize-derived).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <climits>

#include "../../include/pcops.h"

#define PC_WAVE 64

// nvcc-contraction order of the reference's `a*a + b*b + c*c` (see
// oracle/pcops_oracle.c header): fmaf(c,c, fmaf(a,a, b*b)).  All files are
// compiled with -ffp-contract=off so these explicit fmas are the only fusion.
__device__ __forceinline__ float sqd3(float a, float b, float c) {
  return __builtin_fmaf(c, c, __builtin_fmaf(a, a, b * b));
}

// packed form of sqd3 on two independent (a, b, c) triples: v_pk_mul_f32 +
// 2 x v_pk_fma_f32, per-half bit-identical to sqd3
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 sqd3_pk(f32x2 a, f32x2 b, f32x2 c) {
  return __builtin_elementwise_fma(c, c, __builtin_elementwise_fma(a, a, b * b));
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

// Wave sum without LDS: __shfl_xor lowers to ds_bpermute_b32, six dependent
// LDS round trips (each behind an lgkmcnt(0) wait) per sum.  Here four DPP
// steps inside each 16-lane row (xor 1, xor 2, half-row mirror, row mirror)
// and the gfx950 row swaps (v_permlane16_swap: rows 0<->1, 2<->3;
// v_permlane32_swap: halves) -- all VALU.  Every lane ends with the same
// bits (each step adds a commutative pair).  The association differs from
// wave_sum_f32's, so results differ from it in the last bits.
template <int CTRL>
__device__ __forceinline__ float dpp_add_f32(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum_f32_dpp(float v) {
  v = dpp_add_f32<0xB1>(v);   // quad_perm [1,0,3,2]
  v = dpp_add_f32<0x4E>(v);   // quad_perm [2,3,0,1]
  v = dpp_add_f32<0x141>(v);  // row_half_mirror
  v = dpp_add_f32<0x140>(v);  // row_mirror
  const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
  const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
}

// ---- DPP wave reductions (no LDS traffic; result broadcast via readlane) ----
// quad_perm [1,0,3,2] / [2,3,0,1], row_half_mirror, row_mirror give every lane
// its 16-lane row's value; row_bcast15 / row_bcast31 (GFX9 DPP, available on
// gfx950) fold the four rows into lane 63.
// `ident` (the op's identity) is the DPP "old" value so LLVM's DPP combiner
// folds each v_mov_dpp into the following v_max/v_min (one instr per step).
template <typename Op>
__device__ __forceinline__ int wave_reduce_i32_dpp(int v, Op op, int ident) {
  v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0xB1, 0xF, 0xF, false));
  v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0x4E, 0xF, 0xF, false));
  v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0x141, 0xF, 0xF, false));
  v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0x140, 0xF, 0xF, false));
  v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0x142, 0xA, 0xF, false));
  v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0x143, 0xC, 0xF, false));
  return __builtin_amdgcn_readlane(v, 63);
}
struct OpMaxI32 {
  __device__ __forceinline__ int operator()(int a, int b) const { return a > b ? a : b; }
};
struct OpMinI32 {
  __device__ __forceinline__ int operator()(int a, int b) const { return a < b ? a : b; }
};
__device__ __forceinline__ int wave_max_i32(int v) { return wave_reduce_i32_dpp(v, OpMaxI32(), INT_MIN); }
__device__ __forceinline__ int wave_min_i32_dpp(int v) { return wave_reduce_i32_dpp(v, OpMinI32(), INT_MAX); }

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

// Workgroup barrier that only orders LDS: waits for this wave's LDS ops, not
// for its outstanding global stores (__syncthreads() would also emit
// s_waitcnt vmcnt(0) and stall on a store's round trip every iteration).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

#define PC_CHECK_LAUNCH()                               \
  do {                                                  \
    hipError_t _e = hipGetLastError();                  \
    if (_e != hipSuccess) return PCOPS_ERR_LAUNCH;      \
  } while (0)

// ---- stream-ordered fill (replaces hipMemsetAsync everywhere in the library) ----
// A hipMemsetAsync captured into a graph with the HIP runtime torch ships (7.0.51831) is correct
// on the graph's FIRST launch only: later launches leave the buffer holding other values
// (tools/capture_memset_probe.py: 1.2e9 where 0 was due, replay 2 onward), which corrupted every
// "zero, then accumulate" output in the replayed train step.  A kernel node has
// no such problem, so every fill in libpcops is this kernel.  `pattern` is the 32-bit word to
// repeat (0 for zeros, 0xFFFFFFFF for the -NaN sentinel); the byte order is little-endian, so a
// byte-granular head/tail writes the matching byte of the pattern.
namespace {
__global__ void pc_fill_kernel(unsigned char *__restrict__ p, size_t bytes, unsigned pattern) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  // head up to 16-B alignment, then 16-B stores, then the tail (address-based pattern phase)
  const size_t head = (16 - ((uintptr_t)p & 15)) & 15;
  const size_t h = head < bytes ? head : bytes;
  if (tid < h) p[tid] = (unsigned char)(pattern >> (8 * (((uintptr_t)p + tid) & 3)));
  const size_t body = (bytes - h) / 16;
  uint4 *q = (uint4 *)(p + h);
  const unsigned rot = (unsigned)(((uintptr_t)p + h) & 3);  // 0: p + h is 16-B aligned
  const unsigned w = rot ? ((pattern >> (8 * rot)) | (pattern << (32 - 8 * rot))) : pattern;
  const uint4 v = make_uint4(w, w, w, w);
  for (size_t i = tid; i < body; i += stride) q[i] = v;
  const size_t t0 = h + body * 16;
  if (tid < bytes - t0) p[t0 + tid] = (unsigned char)(pattern >> (8 * (((uintptr_t)p + t0 + tid) & 3)));
}
}  // namespace

// hipMemsetAsync's contract (bytes of value `byte`), as a kernel: returns hipSuccess or the launch
// error.  Grid: one 16-B store per thread up to 2048 blocks of 256.
static inline hipError_t pc_memset_async(void *p, int byte, size_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  const unsigned b = (unsigned)byte & 0xFFu;
  const size_t vec = bytes / 16 + 32;
  size_t blocks = (vec + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(pc_fill_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (unsigned char *)p, bytes,
                     b * 0x01010101u);
  return hipGetLastError();
}
