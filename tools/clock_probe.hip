// Diagnostic: in-kernel shader clock (s_memtime ticks / s_memrealtime @100 MHz)
// for a VALU-bound loop on 32 and 256 workgroups of 512 threads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void busy(float *out, unsigned long long *stamps, int iters) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 0.9999f, d = 0.5f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    a = __builtin_fmaf(a, b, c);
    d = __builtin_fmaf(d, c, b);
    b = __builtin_fmaf(b, c, a);
    c = __builtin_fmaf(c, d, a);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    stamps[blockIdx.x * 2] = t1 - t0;
    stamps[blockIdx.x * 2 + 1] = r1 - r0;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}

int main() {
  float *out;
  unsigned long long *st;
  hipMalloc(&out, 256 * 512 * 4);
  hipMalloc(&st, 256 * 16);
  for (int blocks : {32, 256}) {
    for (int rep = 0; rep < 3; ++rep) {
      busy<<<blocks, 512>>>(out, st, 200000);
      hipDeviceSynchronize();
    }
    std::vector<unsigned long long> h(blocks * 2);
    hipMemcpy(h.data(), st, blocks * 16, hipMemcpyDeviceToHost);
    double ghz = 0;
    for (int i = 0; i < blocks; ++i) ghz += (double)h[2 * i] / h[2 * i + 1] * 0.1;
    printf("blocks %d: in-kernel clock %.3f GHz\n", blocks, ghz / blocks);
  }
  return 0;
}
