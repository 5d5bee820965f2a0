// When does a HIP graph replay start a branch that depends on a node in the MIDDLE of another
// branch?  Captured on stream s0 with a side stream s1 (events for fork / join, as _lib.fork):
//   s0: R | fork s1 after R | s0: n_main kernels | s1: n_side kernels | join | s0: Z
// Variant "side_first" captures the side chain before the main chain.  Each kernel's block 0 / lane 0
// stores its start and end (wall clock, 100 MHz) to a device array; the replay prints every
// kernel's start relative to R's.  Ideal: I1 starts right after R ends, beside L1.
//   hipcc --offload-arch=gfx950 -O2 tools/graph_sched.hip -o tools/graph_sched
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

__global__ void spin(unsigned long long *ts, int slot, int iters, float *sink) {
  const unsigned long long t0 = wall_clock64();
  float x = threadIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) x = x * 0.999f + 1e-4f;
  if (x == 12345.f) sink[threadIdx.x] = x;   // never taken; keeps the loop
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ts[2 * slot] = t0;
    ts[2 * slot + 1] = wall_clock64();
  }
}

int main(int argc, char **argv) {
  // argv: order (main_first | side_first), n_main, n_side, spin iterations per kernel
  const bool side_first = argc > 1 && !strcmp(argv[1], "side_first");
  const int nm = argc > 2 ? atoi(argv[2]) : 4, ns = argc > 3 ? atoi(argv[3]) : 3;
  const int IT = argc > 4 ? atoi(argv[4]) : 20000, NB = 64;
  const int nk = 2 + nm + ns;   // R, main chain, side chain, Z
  unsigned long long *ts;
  float *sink;
  CK(hipMalloc(&ts, 2 * nk * sizeof(unsigned long long)));
  CK(hipMalloc(&sink, 1024 * sizeof(float)));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t ef, ej;
  CK(hipEventCreateWithFlags(&ef, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
  hipGraph_t g;
  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
  hipLaunchKernelGGL(spin, dim3(NB), dim3(256), 0, s0, ts, 0, IT, sink);
  CK(hipEventRecord(ef, s0));
  CK(hipStreamWaitEvent(s1, ef, 0));
  auto mains = [&] {
    for (int k = 0; k < nm; ++k) hipLaunchKernelGGL(spin, dim3(NB), dim3(256), 0, s0, ts, 1 + k, IT, sink);
  };
  auto sides = [&] {
    for (int k = 0; k < ns; ++k) hipLaunchKernelGGL(spin, dim3(NB), dim3(256), 0, s1, ts, 1 + nm + k, IT, sink);
  };
  if (side_first) {
    sides();
    mains();
  } else {
    mains();
    sides();
  }
  CK(hipEventRecord(ej, s1));
  CK(hipStreamWaitEvent(s0, ej, 0));
  hipLaunchKernelGGL(spin, dim3(NB), dim3(256), 0, s0, ts, nk - 1, IT, sink);
  CK(hipStreamEndCapture(s0, &g));
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  unsigned long long *h = (unsigned long long *)malloc(2 * nk * sizeof(unsigned long long));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipGraphLaunch(ge, s0));
    CK(hipStreamSynchronize(s0));
    CK(hipMemcpy(h, ts, 2 * nk * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    auto us = [&](unsigned long long t) { return (double)(t - h[0]) / 100.0; };
    printf("%s main %d side %d: R %.0f-%.0f | main %.0f..%.0f | side %.0f..%.0f | Z %.0f-%.0f (us)\n",
           side_first ? "side_first" : "main_first", nm, ns, us(h[0]), us(h[1]), us(h[2]), us(h[2 * nm + 1]),
           us(h[2 * (1 + nm)]), us(h[2 * (nm + ns) + 1]), us(h[2 * (nk - 1)]), us(h[2 * (nk - 1) + 1]));
  }
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return 0;
}
