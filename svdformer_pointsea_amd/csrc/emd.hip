// Approximate EMD by auction (metrics/EMD/emd_cuda.cu:23-316, driver
// emd_cuda_forward :228-282), as a DETERMINISTIC Jacobi auction -- the exact
// rules are oracle_emd's (oracle/pcops_oracle.c), which fix the reference's
// races (atomicAdd slot order, last-writer-wins GetMax, racy last Assign):
//   bid      every unassigned j: best / second-best value over ALL objects k
//            at the iteration's start prices, lowest k among equal bests;
//            value (float)((3.0 - (double)sqrtf(d2)) - (double)price[k]);
//   pick     object k's winner = the LOWEST bidder whose increment lies
//            within 1e-6 (double) of the largest increment on k;
//   assign   winners replace the previous owner; price[k] += increment;
//            in the last iteration every unassigned bidder takes its target.
//
// gfx950 layout: one lane per bidder (256-lane blocks, grid (n/256, B)); the
// object cloud + prices stream through LDS in 1024-point float4 tiles that
// every lane reads by broadcast, so the per-lane scan runs in ascending k
// exactly like the sequential rule (no cross-lane merge, no ties to break).
// Blocks with no unassigned bidder exit before touching LDS.  The per-object
// maximum is an atomicMax on an order-preserving integer key of the float
// increment; the lowest qualifying bidder an atomicMin.  Per iteration:
// bid, pick, assign = 3 launches; state lives in the caller's workspace.
#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kTile = 1024;

__device__ __forceinline__ unsigned order_key(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_value(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

struct State {
  float *price;       // (B,n)
  int *ass_inv;       // (B,n) object -> bidder, -1 free
  int *bid;           // (B,n) bidder -> object of this iteration
  float *bid_inc;     // (B,n)
  unsigned *max_key;  // (B,n) order_key(max increment on object), 0 = none
  int *max_idx;       // (B,n) lowest qualifying bidder, INT_MAX = none
};

__global__ void emd_init_kernel(int total, int *ass, State st) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  ass[i] = -1;
  st.ass_inv[i] = -1;
  st.price[i] = 0.f;
  st.max_key[i] = 0u;
  st.max_idx[i] = INT_MAX;
}

// Bid-pair counting (the -DPCOPS_COUNT_PAIRS build only, tools/emd_bench.py): [0] (bidder, object)
// pairs of the UNASSIGNED bidders -- the auction's work -- and [1] the lane-pairs the scan runs
// (every lane of a block with at least one unassigned bidder scans along)
#ifdef PCOPS_COUNT_PAIRS
__device__ unsigned long long g_emd_pairs[2];
#endif

__global__ __launch_bounds__(kThreads) void emd_bid_kernel(const float *__restrict__ xyz1,
                                                           const float *__restrict__ xyz2, int n, float eps,
                                                           const int *__restrict__ ass, State st) {
  __shared__ float4 tile[kTile];
  const int b = blockIdx.y;
  const int j = blockIdx.x * kThreads + threadIdx.x;
  const size_t base = (size_t)b * n;
  const bool active = j < n && ass[base + j] == -1;
  if (!__syncthreads_or(active)) return;
#ifdef PCOPS_COUNT_PAIRS
  atomicAdd(&g_emd_pairs[0], active ? (unsigned long long)n : 0ull);
  atomicAdd(&g_emd_pairs[1], (unsigned long long)n);
#endif
  float x1 = 0.f, y1 = 0.f, z1 = 0.f;
  if (active) {
    x1 = xyz1[(base + j) * 3];
    y1 = xyz1[(base + j) * 3 + 1];
    z1 = xyz1[(base + j) * 3 + 2];
  }
  float best = -1e9f, better = -1e9f;
  int best_i = -1;
  const float *p2 = xyz2 + base * 3;
  const float *price = st.price + base;
  for (int k0 = 0; k0 < n; k0 += kTile) {
    const int cnt = min(kTile, n - k0);
    for (int t = threadIdx.x; t < cnt; t += kThreads) {
      const int k = k0 + t;
      tile[t] = make_float4(p2[3 * k], p2[3 * k + 1], p2[3 * k + 2], price[k]);
    }
    __syncthreads();
    if (active) {
      for (int t = 0; t < cnt; ++t) {
        const float4 q = tile[t];
        const float d2 = sqd3(q.x - x1, q.y - y1, q.z - z1);
        const float d = (float)((3.0 - (double)sqrtf(d2)) - (double)q.w);
        if (d > best) {
          better = best;
          best = d;
          best_i = k0 + t;
        } else if (d > better) {
          better = d;
        }
      }
    }
    __syncthreads();
  }
  if (active) {
    const float inc = best - better + eps;
    st.bid[base + j] = best_i;
    st.bid_inc[base + j] = inc;
    if (best_i >= 0) atomicMax(&st.max_key[base + best_i], order_key(inc));
  }
}

__global__ void emd_pick_kernel(int n, const int *__restrict__ ass, State st) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const size_t base = (size_t)b * n;
  if (ass[base + j] != -1) return;
  const int k = st.bid[base + j];
  if (k < 0) return;
  const double bi = st.bid_inc[base + j];
  const double mi = key_value(st.max_key[base + k]);
  if (bi - 1e-6 <= mi && mi <= bi + 1e-6) atomicMin(&st.max_idx[base + k], j);
}

// Not the last iteration: per object k.
__global__ void emd_assign_kernel(int n, int *ass, State st) {
  const int b = blockIdx.y;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const size_t base = (size_t)b * n;
  const int j = st.max_idx[base + k];
  st.max_idx[base + k] = INT_MAX;
  st.max_key[base + k] = 0u;
  if (j == INT_MAX) return;
  const int prev = st.ass_inv[base + k];
  if (prev != -1) ass[base + prev] = -1;
  st.ass_inv[base + k] = j;
  ass[base + j] = k;
  st.price[base + k] += st.bid_inc[base + j];
}

// Last iteration: per bidder j, no eviction.
__global__ void emd_assign_last_kernel(int n, int *ass, State st) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const size_t base = (size_t)b * n;
  if (ass[base + j] == -1 && st.bid[base + j] >= 0) ass[base + j] = st.bid[base + j];
}

__global__ void emd_dist_kernel(const float *__restrict__ xyz1, const float *__restrict__ xyz2, int n,
                                const int *__restrict__ ass, float *__restrict__ dist) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const size_t base = (size_t)b * n;
  const int k = ass[base + j];
  if (k < 0) {
    dist[base + j] = 0.f;
    return;
  }
  const float *a = xyz1 + (base + j) * 3, *c = xyz2 + (base + k) * 3;
  dist[base + j] = sqd3(a[0] - c[0], a[1] - c[1], a[2] - c[2]);
}

__global__ void emd_grad_kernel(const float *__restrict__ xyz1, const float *__restrict__ xyz2,
                                const float *__restrict__ graddist, const int *__restrict__ ass, int n,
                                float *__restrict__ grad) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const size_t base = (size_t)b * n;
  const int k = ass[base + j];
  const float g = graddist[base + j] * 2.f;
  const float *a = xyz1 + (base + j) * 3;
  float *o = grad + (base + j) * 3;
  if (k < 0) {
    o[0] = o[1] = o[2] = 0.f;
    return;
  }
  const float *c = xyz2 + (base + k) * 3;
  o[0] = g * (a[0] - c[0]);
  o[1] = g * (a[1] - c[1]);
  o[2] = g * (a[2] - c[2]);
}

State carve(void *ws, int B, int n) {
  const size_t m = (size_t)B * n;
  char *p = (char *)ws;
  State st;
  st.price = (float *)p;
  st.ass_inv = (int *)(p + 4 * m);
  st.bid = (int *)(p + 8 * m);
  st.bid_inc = (float *)(p + 12 * m);
  st.max_key = (unsigned *)(p + 16 * m);
  st.max_idx = (int *)(p + 20 * m);
  return st;
}

}  // namespace

extern "C" unsigned long long pcops_emd_workspace_bytes(int B, int n) {
  if (B <= 0 || n <= 0) return 0;
  return 24ull * (unsigned long long)B * (unsigned long long)n;
}

extern "C" int pcops_emd_forward(const float *xyz1, const float *xyz2, int B, int n, float eps, int iters,
                                 float *dist, int *assignment, void *workspace, unsigned long long workspace_bytes,
                                 pcops_stream_t stream) {
  if (B < 0 || n < 0 || iters < 0) return PCOPS_ERR_INVALID;
  if (B == 0 || n == 0) return PCOPS_OK;
  if (!xyz1 || !xyz2 || !dist || !assignment) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_emd_workspace_bytes(B, n)) return PCOPS_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const State st = carve(workspace, B, n);
  const int total = B * n;
  hipLaunchKernelGGL(emd_init_kernel, dim3((total + 255) / 256), dim3(256), 0, s, total, assignment, st);
  const dim3 g((n + kThreads - 1) / kThreads, B);
  for (int it = 0; it < iters; ++it) {
    hipLaunchKernelGGL(emd_bid_kernel, g, dim3(kThreads), 0, s, xyz1, xyz2, n, eps, assignment, st);
    if (it < iters - 1) {
      hipLaunchKernelGGL(emd_pick_kernel, g, dim3(kThreads), 0, s, n, assignment, st);
      hipLaunchKernelGGL(emd_assign_kernel, g, dim3(kThreads), 0, s, n, assignment, st);
    } else {
      hipLaunchKernelGGL(emd_assign_last_kernel, g, dim3(kThreads), 0, s, n, assignment, st);
    }
  }
  hipLaunchKernelGGL(emd_dist_kernel, g, dim3(kThreads), 0, s, xyz1, xyz2, n, assignment, dist);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

#ifdef PCOPS_COUNT_PAIRS
// counting build only (not in include/pcops.h): the two bid-pair counters to `out`, then zeroed
extern "C" int pcops_debug_emd_pair_counts(unsigned long long *out) {
  if (hipDeviceSynchronize() != hipSuccess) return PCOPS_ERR_LAUNCH;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_emd_pairs), sizeof(unsigned long long) * 2) != hipSuccess)
    return PCOPS_ERR_LAUNCH;
  const unsigned long long zero[2] = {0, 0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_emd_pairs), zero, sizeof(zero)) != hipSuccess) return PCOPS_ERR_LAUNCH;
  return PCOPS_OK;
}
#endif

extern "C" int pcops_emd_backward(const float *xyz1, const float *xyz2, const float *graddist, const int *assignment,
                                  int B, int n, float *gradxyz1, pcops_stream_t stream) {
  if (B < 0 || n < 0) return PCOPS_ERR_INVALID;
  if (B == 0 || n == 0) return PCOPS_OK;
  if (!xyz1 || !xyz2 || !graddist || !assignment || !gradxyz1) return PCOPS_ERR_INVALID;
  const dim3 g((n + kThreads - 1) / kThreads, B);
  hipLaunchKernelGGL(emd_grad_kernel, g, dim3(kThreads), 0, (hipStream_t)stream, xyz1, xyz2, graddist, assignment, n,
                     gradxyz1);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
