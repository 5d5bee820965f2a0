// Diagnostic: VALU throughput per instruction kind on gfx950 (cycles per
// wave-instruction per SIMD), 8 independent chains per lane, 4 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAINS 8
template <int KIND>
__global__ __launch_bounds__(1024) void k(float *out, unsigned long long *cyc, int iters) {
  float a[CHAINS], b = 1.0001f + threadIdx.x * 1e-7f, c = 0.999f;
  int ia[CHAINS];
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 p[CHAINS], pb = {b, b * 1.0001f}, pc = {c, c};
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) { a[i] = threadIdx.x * 1e-3f + i; ia[i] = threadIdx.x + i; p[i] = f2{a[i], a[i] + 0.5f}; }
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) {
      if (KIND == 0) a[i] = __builtin_fmaf(a[i], b, c);                 // v_fma_f32
      if (KIND == 1) a[i] = a[i] - b;                                    // v_sub_f32
      if (KIND == 2) ia[i] = min(ia[i] ^ 0x55, (int)it);                 // v_xor + v_min_i32
      if (KIND == 3) ia[i] = ia[i] + it;                                 // v_add_u32
      if (KIND == 4) a[i] = fmaxf(a[i] * b, c);                          // v_mul + v_max
      if (KIND == 5) p[i] = __builtin_elementwise_fma(p[i], pb, pc);     // v_pk_fma_f32
      if (KIND == 6) p[i] = p[i] - pb;                                   // v_pk_add_f32
      if (KIND == 7) p[i] = p[i] * pb;                                   // v_pk_mul_f32
    }
    asm volatile("" ::: "memory");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0; int si = 0;
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) { s += a[i] + p[i].x + p[i].y; si += ia[i]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s + si;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
void run(const char *name, float ops_per_chain_iter, float *out, unsigned long long *cyc) {
  const int iters = 20000, blocks = 256;
  k<KIND><<<blocks, 1024>>>(out, cyc, iters);
  (void)hipDeviceSynchronize();
  k<KIND><<<blocks, 1024>>>(out, cyc, iters);
  (void)hipDeviceSynchronize();
  unsigned long long h[256];
  (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double c = 0; for (int i = 0; i < blocks; ++i) c += h[i]; c /= blocks;
  // per SIMD: 4 waves, each issues iters*CHAINS*ops instructions
  double instr = 4.0 * iters * CHAINS * ops_per_chain_iter;
  printf("%-28s %.2f cycles per wave-instruction per SIMD\n", name, c / instr);
}

int main() {
  float *out; unsigned long long *cyc;
  (void)hipMalloc(&out, 256 * 1024 * 4); (void)hipMalloc(&cyc, 256 * 8);
  run<0>("v_fma_f32", 1, out, cyc);
  run<1>("v_sub_f32", 1, out, cyc);
  run<2>("v_xor+v_min_i32", 2, out, cyc);
  run<3>("v_add_u32", 1, out, cyc);
  run<4>("v_mul_f32+v_max_f32", 2, out, cyc);
  run<5>("v_pk_fma_f32", 1, out, cyc);
  run<6>("v_pk_add_f32", 1, out, cyc);
  run<7>("v_pk_mul_f32", 1, out, cyc);
  return 0;
}
