// Which dependency edges does stream capture record for the fork/join shapes `_lib.fork` and the
// autograd engine produce?  Each variant captures kernels k<ID> on streams M (origin), S0, S3 and
// prints every kernel node with the IDs of the kernel nodes it depends on (through empty /
// event-wait nodes, transitively collapsed to kernel nodes).  No replay: capture + inspection only.
//   cross   M:k0 | S0<-M, S0:k1 | S3<-M, S3:k2 | S0<-S3, S0:k3 | M<-S0, M:k4     (want k3 <- {k1, k2})
//   rewait  M:k0 | S0<-M, S0:k1 | M:k2 | S0<-M, S0:k3 | M<-S0, M:k4             (want k3 <- {k1, k2})
//   chain   M:k0 | S0<-M, S0:k1 | S3<-S0, S3:k2 | M<-S3, M:k3 | S0<-M, S0:k4 | M<-S0 (want k4 <- {k1, k3})
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      printf("FAIL %s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      fflush(stdout);                                                                      \
      return 2;                                                                            \
    }                                                                                      \
  } while (0)

template <int ID>
__global__ void k(float *x) {
  x[threadIdx.x] += ID;
}

static hipError_t wait_stream(hipStream_t waiter, hipStream_t waited) {
  hipEvent_t e;
  hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
  if (r != hipSuccess) return r;
  if ((r = hipEventRecord(e, waited)) != hipSuccess) return r;
  if ((r = hipStreamWaitEvent(waiter, e, 0)) != hipSuccess) return r;
  return hipEventDestroy(e);
}

#define L(ID, S) hipLaunchKernelGGL(k<ID>, dim3(1), dim3(64), 0, S, x)

int main(int argc, char **argv) {
  const char *v = argc > 1 ? argv[1] : "cross";
  int rtv = 0;
  CK(hipRuntimeGetVersion(&rtv));
  float *x;
  CK(hipMalloc(&x, 256));
  hipStream_t M, S0, S3;
  CK(hipStreamCreateWithFlags(&M, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&S0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&S3, hipStreamNonBlocking));
  std::map<const void *, int> ids = {{(const void *)k<0>, 0}, {(const void *)k<1>, 1}, {(const void *)k<2>, 2},
                                     {(const void *)k<3>, 3}, {(const void *)k<4>, 4}, {(const void *)k<5>, 5}};
  CK(hipStreamBeginCapture(M, hipStreamCaptureModeGlobal));
  if (!strcmp(v, "cross")) {
    L(0, M);
    CK(wait_stream(S0, M)); L(1, S0);
    CK(wait_stream(S3, M)); L(2, S3);
    CK(wait_stream(S0, S3)); L(3, S0);
    CK(wait_stream(M, S0)); L(4, M);
  } else if (!strcmp(v, "rewait")) {
    L(0, M);
    CK(wait_stream(S0, M)); L(1, S0);
    L(2, M);
    CK(wait_stream(S0, M)); L(3, S0);
    CK(wait_stream(M, S0)); L(4, M);
  } else if (!strcmp(v, "chain")) {
    L(0, M);
    CK(wait_stream(S0, M)); L(1, S0);
    CK(wait_stream(S3, S0)); L(2, S3);
    CK(wait_stream(M, S3)); L(3, M);
    CK(wait_stream(S0, M)); L(4, S0);
    CK(wait_stream(M, S0));
  } else {
    printf("unknown variant\n");
    return 2;
  }
  hipGraph_t graph;
  CK(hipStreamEndCapture(M, &graph));
  size_t n = 0;
  CK(hipGraphGetNodes(graph, nullptr, &n));
  std::vector<hipGraphNode_t> nodes(n);
  CK(hipGraphGetNodes(graph, nodes.data(), &n));
  // kernel-node ancestors (direct kernel predecessors, looking through non-kernel nodes)
  std::map<hipGraphNode_t, int> kid;
  for (auto nd : nodes) {
    hipGraphNodeType t;
    CK(hipGraphNodeGetType(nd, &t));
    if (t == hipGraphNodeTypeKernel) {
      hipKernelNodeParams p;
      CK(hipGraphKernelNodeGetParams(nd, &p));
      kid[nd] = ids.count(p.func) ? ids[p.func] : -1;
    }
  }
  printf("%s (HIP runtime %d): %zu nodes\n", v, rtv, n);
  for (auto nd : nodes) {
    if (!kid.count(nd)) continue;
    std::set<int> preds;
    std::vector<hipGraphNode_t> stack = {nd};
    std::set<hipGraphNode_t> seen;
    while (!stack.empty()) {
      auto cur = stack.back();
      stack.pop_back();
      size_t nd_ = 0;
      CK(hipGraphNodeGetDependencies(cur, nullptr, &nd_));
      std::vector<hipGraphNode_t> deps(nd_);
      if (nd_) CK(hipGraphNodeGetDependencies(cur, deps.data(), &nd_));
      for (auto d : deps) {
        if (seen.count(d)) continue;
        seen.insert(d);
        if (kid.count(d)) preds.insert(kid[d]);
        else stack.push_back(d);
      }
    }
    printf("  k%d <-", kid[nd]);
    for (int p : preds) printf(" k%d", p);
    printf("\n");
  }
  return 0;
}
