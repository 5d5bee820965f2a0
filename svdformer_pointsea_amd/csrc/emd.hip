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
// gfx950 layout: one lane per UNASSIGNED bidder.  After each assignment a
// compaction pass lists every batch's unassigned bidders (the list order comes
// from atomics, and does not matter: a bid depends on its bidder and the
// iteration-start prices only, and the per-object maximum / lowest qualifying
// bidder are order-independent atomics), and the bid launch runs 256-lane
// blocks over that list; blocks past a batch's count exit at once.  Lanes no
// longer idle beside assigned neighbours: after the first iterations ~90 % of
// the bidders hold an object, and the one-lane-per-bidder grid had every block
// scan all n objects while any of its 256 bidders bid (profiles/
// r6_emd_pairs.json: lane-pairs = all pairs, active pairs 9.9 % at B 32 n 2048).
// The object cloud + prices stream through LDS in 1024-point float4 tiles
// that every lane reads by broadcast, so the per-lane scan runs in ascending k
// exactly like the sequential rule (no cross-lane merge, no ties to break).
// The per-object maximum is an atomicMax on an order-preserving integer key of
// the float increment; the lowest qualifying bidder an atomicMin.  Per
// iteration: bid, pick, assign, compact = 4 launches; state lives in the
// caller's workspace.
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
  int *list;          // (B,n) the unassigned bidders of the iteration (any order)
  int *cnt;           // (B) their number
};

// every bidder unassigned: the first list is 0..n-1 in order
__global__ void emd_init_kernel(int total, int n, int *ass, State st) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  ass[i] = -1;
  st.ass_inv[i] = -1;
  st.price[i] = 0.f;
  st.max_key[i] = 0u;
  st.max_idx[i] = INT_MAX;
  st.list[i] = i % n;
  if (i % n == 0) st.cnt[i / n] = n;
}

// the unassigned bidders of batch b appended to its list (cnt was zeroed by the pick launch)
__global__ void emd_compact_kernel(int n, const int *__restrict__ ass, State st) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const bool un = j < n && ass[(size_t)b * n + j] == -1;
  // one atomic per wave: the wave's unassigned lanes take consecutive slots
  const unsigned long long m = __ballot(un);
  if (m == 0) return;
  const int lane = threadIdx.x & 63;
  int base = 0;
  if (lane == (int)__builtin_ctzll(m)) base = atomicAdd(&st.cnt[b], (int)__popcll(m));
  base = __shfl(base, (int)__builtin_ctzll(m), 64);
  if (un) st.list[(size_t)b * n + base + (int)__popcll(m & ((1ull << lane) - 1))] = j;
}

// Bid-pair counting (the -DPCOPS_COUNT_PAIRS build only, tools/emd_bench.py): [0] (bidder, object)
// pairs of the UNASSIGNED bidders -- the auction's work -- and [1] the lane-pairs the scan runs
// (every lane of a block with at least one unassigned bidder scans along)
#ifdef PCOPS_COUNT_PAIRS
__device__ unsigned long long g_emd_pairs[2];
#endif

// (best, better, index) of one bidder over a range of objects, merged in any order: the
// sequential rule's result -- the largest value at its LOWEST k, and the largest of all the
// other values (the second largest as a multiset) -- is order-free once equal bests keep the
// lower k.  Float max / compares only: bitwise the ascending scan's result.
__device__ __forceinline__ void bid_merge(float &best, float &better, int &bi, float ob, float obt, int oi) {
  if (ob > best || (ob == best && oi >= 0 && (bi < 0 || oi < bi))) {
    better = fmaxf(best, obt);
    best = ob;
    bi = oi;
  } else {
    better = fmaxf(better, ob);
  }
}

// Block x of batch b takes bidders [x upb, (x+1) upb) of the batch's unassigned list,
// upb = ceil(count / blocks), with T = the largest power of two <= min(64, 256 / upb) lanes per
// bidder: lane t of a bidder scans objects [t s, (t+1) s) of every 1024-object LDS tile (s =
// 1024 / T), in ascending order, and the T lanes' results are merged by a shuffle tree.  Early
// iterations (every bidder unassigned) run T = 1: one lane per bidder over all objects; late
// ones spread a few bidders over whole waves instead of leaving the chip idle behind them
// (the reference splits bidders over threads the same way, emd_cuda.cu:95-175).
__global__ __launch_bounds__(kThreads) void emd_bid_kernel(const float *__restrict__ xyz1,
                                                           const float *__restrict__ xyz2, int n, float eps,
                                                           const int *__restrict__ ass, State st) {
  __shared__ float4 tile[kTile];
  const int b = blockIdx.y;
  const int nact = st.cnt[b];
  const int upb = (nact + (int)gridDim.x - 1) / (int)gridDim.x;   // bidders per block
  const int first = (int)blockIdx.x * upb;
  if (upb == 0 || first >= nact) return;   // block-uniform: nothing of this batch's list here
  int T = 1;
  while (T < 64 && 2 * T * upb <= kThreads) T *= 2;
  const int mine = min(upb, nact - first);   // bidders of this block
  const int slot = threadIdx.x / T, t = threadIdx.x % T;
  const bool active = slot < mine;
  const size_t base = (size_t)b * n;
  const int j = active ? st.list[base + first + slot] : 0;
#ifdef PCOPS_COUNT_PAIRS
  if (active && t == 0) atomicAdd(&g_emd_pairs[0], (unsigned long long)n);
  if (threadIdx.x == 0) atomicAdd(&g_emd_pairs[1], (unsigned long long)kThreads * ((n + T - 1) / T));
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
  const int seg = kTile / T;
  for (int k0 = 0; k0 < n; k0 += kTile) {
    const int cnt = min(kTile, n - k0);
    for (int q = threadIdx.x; q < cnt; q += kThreads) {
      const int k = k0 + q;
      tile[q] = make_float4(p2[3 * k], p2[3 * k + 1], p2[3 * k + 2], price[k]);
    }
    __syncthreads();
    if (active) {
      const int e = min(cnt, (t + 1) * seg);
      for (int q = t * seg; q < e; ++q) {
        const float4 o = tile[q];
        const float d2 = sqd3(o.x - x1, o.y - y1, o.z - z1);
        const float d = (float)((3.0 - (double)sqrtf(d2)) - (double)o.w);
        if (d > best) {
          better = best;
          best = d;
          best_i = k0 + q;
        } else if (d > better) {
          better = d;
        }
      }
    }
    __syncthreads();
  }
  // the T lanes of a bidder (consecutive lanes of one wave): tree merge
  for (int o = 1; o < T; o <<= 1) {
    const float ob = __shfl_down(best, o, 64), obt = __shfl_down(better, o, 64);
    const int oi = __shfl_down(best_i, o, 64);
    if ((t & (2 * o - 1)) == 0) bid_merge(best, better, best_i, ob, obt, oi);
  }
  if (active && t == 0) {
    const float inc = best - better + eps;
    st.bid[base + j] = best_i;
    st.bid_inc[base + j] = inc;
    if (best_i >= 0) atomicMax(&st.max_key[base + best_i], order_key(inc));
  }
}

__global__ void emd_pick_kernel(int n, const int *__restrict__ ass, State st) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j == 0) st.cnt[b] = 0;   // the bid launch has read the list: the compaction refills it
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
  st.list = (int *)(p + 24 * m);
  st.cnt = (int *)(p + 28 * m);
  return st;
}

}  // namespace

extern "C" unsigned long long pcops_emd_workspace_bytes(int B, int n) {
  if (B <= 0 || n <= 0) return 0;
  return 28ull * (unsigned long long)B * (unsigned long long)n + 4ull * (unsigned long long)B;
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
  hipLaunchKernelGGL(emd_init_kernel, dim3((total + 255) / 256), dim3(256), 0, s, total, n, assignment, st);
  const dim3 g((n + kThreads - 1) / kThreads, B);
  for (int it = 0; it < iters; ++it) {
    hipLaunchKernelGGL(emd_bid_kernel, g, dim3(kThreads), 0, s, xyz1, xyz2, n, eps, assignment, st);
    if (it < iters - 1) {
      hipLaunchKernelGGL(emd_pick_kernel, g, dim3(kThreads), 0, s, n, assignment, st);
      hipLaunchKernelGGL(emd_assign_kernel, g, dim3(kThreads), 0, s, n, assignment, st);
      hipLaunchKernelGGL(emd_compact_kernel, g, dim3(kThreads), 0, s, n, assignment, st);
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
