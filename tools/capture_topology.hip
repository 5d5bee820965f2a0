// Stream-capture topologies of `_lib.fork` under hipStreamBeginCapture (global mode), without torch.
//
// The PointSea step's capture segfaulted in capture_end when a fork was opened INSIDE another fork
// (tests/test_gpu_capture_fork.py reproduces it).  Each variant below builds one fork/join shape
// the way torch's Stream.wait_stream does it (a fresh event recorded on the waited-for stream,
// hipStreamWaitEvent on the waiting one), captures it from an origin stream M, instantiates,
// launches and checks the result.  Usage: capture_topology <variant>; exit 0 = captured, replayed
// and correct.  Variants:
//   flat      M -> S0, M -> S3, both joined into M                     (the bench's shape today)
//   nested_k  M -> S0, kernel on S0, S0 -> S3, S3 -> S0, S0 -> M        (inner fork after S0 work)
//   nested    M -> S0, S0 -> S3 (S0 empty), S3 -> S0, S0 -> M           (the crashing torch shape)
//   cross     M -> S0, M -> S3, S3 -> S0, S0 -> M                       (sibling joined into sibling)
//   nested_m  as nested, but S3 also waits on M first, and M waits on S3 at the end
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      printf("FAIL %s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      fflush(stdout);                                                                      \
      return 2;                                                                            \
    }                                                                                      \
  } while (0)

__global__ void add_kernel(float *x, int n, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] += v;
}

// dst[i] = src[i] * 2 + dst[i]: makes the join order observable
__global__ void mix_kernel(float *dst, const float *src, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i] * 2.f + dst[i];
}

static hipError_t wait_stream(hipStream_t waiter, hipStream_t waited) {
  hipEvent_t e;
  hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
  if (r != hipSuccess) return r;
  if ((r = hipEventRecord(e, waited)) != hipSuccess) return r;
  if ((r = hipStreamWaitEvent(waiter, e, 0)) != hipSuccess) return r;
  return hipEventDestroy(e);   // torch drops its temporary event right away, as here
}

int main(int argc, char **argv) {
  const char *v = argc > 1 ? argv[1] : "flat";
  int rtv = 0;
  CK(hipRuntimeGetVersion(&rtv));
  printf("%s: HIP runtime %d\n", v, rtv);
  const int n = 1 << 16;
  float *a, *b, *c;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  CK(hipMalloc(&c, n * 4));
  hipStream_t M, S0, S3;
  CK(hipStreamCreateWithFlags(&M, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&S0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&S3, hipStreamNonBlocking));
  CK(hipMemset(a, 0, n * 4));
  CK(hipMemset(b, 0, n * 4));
  CK(hipMemset(c, 0, n * 4));
  CK(hipDeviceSynchronize());
  const dim3 g((n + 255) / 256), t(256);

  CK(hipStreamBeginCapture(M, hipStreamCaptureModeGlobal));
  hipLaunchKernelGGL(add_kernel, g, t, 0, M, a, n, 1.f);                 // a = 1
  if (!strcmp(v, "flat")) {
    CK(wait_stream(S0, M));
    CK(wait_stream(S3, M));
    hipLaunchKernelGGL(add_kernel, g, t, 0, S3, b, n, 3.f);              // b = 3
    hipLaunchKernelGGL(mix_kernel, g, t, 0, S0, c, a, n);                // c = 2
    CK(wait_stream(M, S3));
    CK(wait_stream(M, S0));
    hipLaunchKernelGGL(mix_kernel, g, t, 0, M, c, b, n);                 // c = 8
  } else if (!strcmp(v, "nested_k") || !strcmp(v, "nested") || !strcmp(v, "nested_m")) {
    CK(wait_stream(S0, M));
    if (!strcmp(v, "nested_k")) hipLaunchKernelGGL(add_kernel, g, t, 0, S0, c, n, 0.f);
    if (!strcmp(v, "nested_m")) CK(wait_stream(S3, M));
    CK(wait_stream(S3, S0));
    {  // what the caching allocator asks of every stream it allocates on during capture
      hipStreamCaptureStatus st[3];
      unsigned long long id[3];
      hipStream_t ss[3] = {M, S0, S3};
      for (int k = 0; k < 3; ++k) CK(hipStreamGetCaptureInfo(ss[k], &st[k], &id[k]));
      printf("%s: capture info M (%d, %llu) S0 (%d, %llu) S3 (%d, %llu)\n", v, (int)st[0], id[0], (int)st[1], id[1],
             (int)st[2], id[2]);
      hipGraph_t gg = nullptr;
      const hipGraphNode_t *deps = nullptr;
      size_t nd = 0;
      CK(hipStreamGetCaptureInfo_v2(S3, &st[2], &id[2], &gg, &deps, &nd));
      printf("%s: S3 v2 status %d id %llu graph %p deps %zu\n", v, (int)st[2], id[2], (void *)gg, nd);
    }
    hipLaunchKernelGGL(add_kernel, g, t, 0, S3, b, n, 3.f);              // b = 3
    hipLaunchKernelGGL(mix_kernel, g, t, 0, S0, c, a, n);                // c = 2
    CK(wait_stream(S0, S3));
    hipLaunchKernelGGL(mix_kernel, g, t, 0, S0, c, b, n);                // c = 8
    CK(wait_stream(M, S0));
    if (!strcmp(v, "nested_m")) CK(wait_stream(M, S3));
  } else if (!strcmp(v, "cross")) {
    CK(wait_stream(S0, M));
    CK(wait_stream(S3, M));
    hipLaunchKernelGGL(add_kernel, g, t, 0, S3, b, n, 3.f);
    hipLaunchKernelGGL(mix_kernel, g, t, 0, S0, c, a, n);
    CK(wait_stream(S0, S3));
    hipLaunchKernelGGL(mix_kernel, g, t, 0, S0, c, b, n);
    CK(wait_stream(M, S0));
  } else {
    printf("unknown variant %s\n", v);
    return 2;
  }
  hipGraph_t graph;
  printf("%s: ending capture\n", v);
  fflush(stdout);
  CK(hipStreamEndCapture(M, &graph));
  size_t nodes = 0;
  CK(hipGraphGetNodes(graph, nullptr, &nodes));
  printf("%s: captured %zu nodes; instantiating\n", v, nodes);
  fflush(stdout);
  hipGraphExec_t exec;
  CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  CK(hipGraphLaunch(exec, M));
  CK(hipStreamSynchronize(M));
  float h = 0.f;
  CK(hipMemcpy(&h, c + 1234, 4, hipMemcpyDeviceToHost));
  printf("%s: replayed, c = %g (expect 8)\n", v, h);
  CK(hipGraphExecDestroy(exec));
  CK(hipGraphDestroy(graph));
  return h == 8.f ? 0 : 1;
}
