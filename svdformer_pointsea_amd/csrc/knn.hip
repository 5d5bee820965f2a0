// k-nearest-neighbour selection (models/model_utils.py:258-286 query_knn,
// :807-810 query_knn_point) for gfx950.
//
// The reference materialises the full (B,S,N) distance matrix in HBM through
// a BLAS matmul, then argsorts every row.  Here one thread owns one query,
// candidates stream through LDS, and a sorted top-(K+pad) list lives in
// VGPRs (static indices, strict-'<' insertion => ascending (distance, index)
// order).  The distance is evaluated in exactly the fp32 order torch's CPU
// kernels use for square_distance (verified bit-for-bit by the golden vectors):
//   dot  = sequential fma chain over channels (sgemm micro-kernel)
//   |v|^2 = torch.sum(v**2,-1) reduction order (see torch_sumsq below)
//   d = ((-2*dot) + |q|^2) + |p|^2
#include <cstdlib>

#include "common.h"

namespace {

// torch CPU sum-of-squares order (oracle_torch_sumsq): C%32==0 (<=512) ->
// four 8-lane accumulators over 32-element chunks; otherwise sequential.
__device__ __forceinline__ float torch_sumsq(const float *v, int C) {
  if (C % 32 == 0 && C >= 32 && C <= 512) {
    float acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int l = 0; l < 8; ++l) acc[j][l] = 0.f;
    for (int c0 = 0; c0 < C; c0 += 32) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int l = 0; l < 8; ++l) {
          const float x = v[c0 + j * 8 + l];
          acc[j][l] = acc[j][l] + x * x;
        }
    }
    float s = 0.f;
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      const float t = ((acc[0][l] + acc[1][l]) + acc[2][l]) + acc[3][l];
      s = (l == 0) ? t : s + t;
    }
    return s;
  }
  float s = v[0] * v[0];
  for (int c = 1; c < C; ++c) s = s + v[c] * v[c];
  return s;
}

template <int KK>
__device__ __forceinline__ void topk_insert(float (&bd)[KK], int (&bi)[KK], float d, int k) {
  if (d < bd[KK - 1]) {
    bd[KK - 1] = d;
    bi[KK - 1] = k;
#pragma unroll
    for (int s = KK - 1; s > 0; --s) {
      const bool sw = bd[s] < bd[s - 1];
      const float d0 = bd[s - 1], d1 = bd[s];
      const int i0 = bi[s - 1], i1 = bi[s];
      bd[s - 1] = sw ? d1 : d0;
      bd[s] = sw ? d0 : d1;
      bi[s - 1] = sw ? i1 : i0;
      bi[s] = sw ? i0 : i1;
    }
  }
}

template <int KK>
__device__ __forceinline__ void topk_store(const float (&bd)[KK], const int (&bi)[KK], int K, int pad, int n_avail,
                                           int *out_idx, float *out_dist) {
#pragma unroll
  for (int k = 0; k < KK; ++k) {
    if (k >= pad && k < pad + K) {
      const bool ok = k < n_avail;
      out_idx[k - pad] = ok ? bi[k] : 0;
      if (out_dist) out_dist[k - pad] = ok ? bd[k] : 0.f;
    }
  }
}

// Block = 64 queries x G waves.  Wave w scans its own slice of every LDS
// candidate tile (ascending index inside the slice), so each (query, wave)
// keeps a sorted top-KK of a candidate subset; the G lists are then merged in
// LDS by wave 0 in lexicographic (distance, index) order -- the same total
// order the single-list scan produces.  G > 1 multiplies the waves in flight
// (the small-S calls would otherwise occupy a handful of CUs).
template <int KK, int G>
struct MergeBuf {
  float d[G][KK][64];
  int i[G][KK][64];
};

template <int KK, int G>
__device__ __forceinline__ void merge_and_store(MergeBuf<KK, G> &mb, const float (&bd)[KK], const int (&bi)[KK],
                                                int w, int lane, bool valid, int K, int pad, int n_avail,
                                                int *out_idx, float *out_dist) {
  if (G == 1) {
    if (valid) topk_store<KK>(bd, bi, K, pad, n_avail, out_idx, out_dist);
    return;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < KK; ++k) {
    mb.d[w][k][lane] = bd[k];
    mb.i[w][k][lane] = bi[k];
  }
  __syncthreads();
  if (w != 0 || !valid) return;
  int head[G];
#pragma unroll
  for (int g = 0; g < G; ++g) head[g] = 0;
  const int need = min(KK, K + pad);
  for (int o = 0; o < need; ++o) {
    float bdv = INFINITY;
    int biv = INT_MAX, bw = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (head[g] < KK) {
        const float dv = mb.d[g][head[g]][lane];
        const int iv = mb.i[g][head[g]][lane];
        if (dv < bdv || (dv == bdv && iv < biv)) {
          bdv = dv;
          biv = iv;
          bw = g;
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) head[g] += (g == bw);
    if (o >= pad) {
      const bool ok = o < n_avail;
      out_idx[o - pad] = ok ? biv : 0;
      if (out_dist) out_dist[o - pad] = ok ? bdv : 0.f;
    }
  }
}

// Buffered top-K selection.  A candidate can only enter a lane's list if it
// beats the list's last entry, so the scan filters against that threshold and
// APPENDS passing (distance, index) pairs to a per-lane LDS queue; the queue
// is drained into the sorted register list (topk_insert) only when some lane
// of the wave nears CAP entries, and after the last candidate.  Between
// drains the list does not change, so the filter is exactly the insertion
// test; the queue keeps scan order, so strict-'<' insertion still yields the
// (distance, index) order of a sequential scan.  What this buys: the
// 16-deep compare-swap network runs once per *passing* candidate per drain
// round instead of once per candidate whenever ANY lane of the wave inserts
// (with ~5 % of candidates passing per lane, ~95 % of a wave's candidate
// steps used to pay the whole network).
#ifndef PCOPS_KNN_ABL   // diagnostic builds: 1 = scan only, 2 = scan + filter/append, no insertion
#define PCOPS_KNN_ABL 0
#endif
template <int KK, int CAP, int NT>
struct TopK {
  float bd[KK];
  int bi[KK];
  float thr;
  int cnt;
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int k = 0; k < KK; ++k) {
      bd[k] = INFINITY;
      bi[k] = 0;
    }
    thr = INFINITY;
    cnt = 0;
  }
  // queue[j * NT + tid]: lane tid's j-th pending candidate
  __device__ __forceinline__ void offer(int2 *queue, int tid, float d, int k) {
    if (d < thr) {
      queue[cnt * NT + tid] = make_int2(__float_as_int(d), k);
      ++cnt;
    }
  }
  __device__ __forceinline__ void drain(const int2 *queue, int tid) {
    for (int j = 0; __any(j < cnt); ++j) {
      if (j < cnt) {
        const int2 v = queue[j * NT + tid];
        topk_insert<KK>(bd, bi, __int_as_float(v.x), v.y);
      }
    }
    thr = bd[KK - 1];
    cnt = 0;
  }
  // branch-free offer: the pair is always written to the lane's next free slot and the
  // slot is kept only when `pass` (a rejected pair is overwritten by the next one); no
  // exec-mask branch per candidate -- the VALU -> SALU -> exec chain of a divergent `if`
  // stalled every candidate step.  The caller has drained so that cnt + pending <= CAP.
  __device__ __forceinline__ void append(int2 *queue, int tid, float d, int k, bool pass) {
    queue[cnt * NT + tid] = make_int2(__float_as_int(d), k);
    cnt += pass ? 1 : 0;
  }
  // drain when a further `room` offers could overflow some lane's queue
  __device__ __forceinline__ void maybe_drain(const int2 *queue, int tid, int room) {
    if (__any(cnt > CAP - room)) drain(queue, tid);
  }
};

// smallest float above x (x itself for +inf and NaN)
__device__ __forceinline__ float next_up(float x) {
  if (!(x < INFINITY)) return x;
  if (x == 0.f) return __int_as_float(1);
  const int b = __float_as_int(x);
  return __int_as_float(x > 0.f ? b + 1 : b - 1);
}

// C == 3: candidates staged as float4 (x, y, z, |p|^2), TN per tile.
// Large grids (>= 3 blocks per CU): G = 4, TN = 512 -> 40 KB of LDS, so four
// blocks (16 waves) fit a CU and the whole grid is resident at once; small
// grids: G = 8 waves per 64 queries, TN = 1024.
template <int KK, int G, int TN>
__global__ __launch_bounds__(64 * G) void knn3_kernel(const float *__restrict__ q, const float *__restrict__ p, int S,
                                                      int N, int K, int pad, int *__restrict__ idx,
                                                      float *__restrict__ dist, bool share) {
  // CAP 15 leaves room for the shared thresholds inside the merge buffer's footprint
  // (40 KB at G = 4, TN = 512: four blocks per CU)
  constexpr int SL = TN / G, U = 8, CAP = 15, NT = 64 * G;
  __shared__ float4 tile[TN];
  __shared__ union {
    MergeBuf<KK, G> mb;
    struct {
      int2 queue[CAP * NT];
      float sthr[G][64];
    } sc;
  } sh;
  const int b = blockIdx.y, tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int s = blockIdx.x * 64 + lane;
  const float *qb = q + (size_t)b * S * 3;
  const float *pb = p + (size_t)b * N * 3;
  const int sc = s < S ? s : S - 1;
  const float qx = qb[3 * sc], qy = qb[3 * sc + 1], qz = qb[3 * sc + 2];
  const float qn = (qx * qx + qy * qy) + qz * qz;
  const float mx = -2.f * qx, my = -2.f * qy, mz = -2.f * qz;  // (-2q).p == -2(q.p) bit-exactly
  TopK<KK, CAP, NT> tk;
  tk.init();
  // Shared thresholds: a candidate farther than ANY wave's current KK-th distance for this
  // query cannot be in the merged top KK (that wave already holds KK closer ones), so each
  // wave also filters against the others' published thresholds -- the G lists then converge
  // like one list over G times the candidates instead of G lists each built from scratch
  // (the selection was ~70 % of the kernel, profiles/r4_knn_ab.txt).  Ties (d equal to the
  // other wave's threshold) still pass, and a stale threshold is only a looser filter, so
  // the merged result is exactly the unfiltered one.  Relaxed LDS atomics, no barrier.
  float(&sthr)[G][64] = sh.sc.sthr;
  __hip_atomic_store(&sthr[w][lane], INFINITY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  float xthr = INFINITY, teff = INFINITY;
  for (int t0 = 0; t0 < N; t0 += TN) {
    const int cnt = min(TN, N - t0);
    for (int e = tid; e < cnt; e += NT) {
      const float *src = pb + (size_t)(t0 + e) * 3;
      const float x = src[0], y = src[1], z = src[2];
      tile[e] = make_float4(x, y, z, (x * x + y * y) + z * z);
    }
    __syncthreads();
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const int e1 = min(cnt, (wu + 1) * SL);  // scalar
    for (int e0 = wu * SL; e0 < e1; e0 += U) {
      // the U candidates' LDS reads first, all in flight together.  e0 + u < (w + 1) * SL <= TN:
      // in the tile even past e1 (the last, partial tile), where `live` drops them.
      float4 c[U];
#pragma unroll
      for (int u = 0; u < U; ++u) c[u] = tile[e0 + u];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool live = e0 + u < e1;  // scalar
        const float dot = __builtin_fmaf(mz, c[u].z, __builtin_fmaf(my, c[u].y, mx * c[u].x));
#if PCOPS_KNN_ABL == 1
        // diagnostic ablation (tools builds only): distances without the selection
        const float dd = (dot + qn) + c[u].w;
        if (live && dd < tk.bd[0]) { tk.bd[0] = dd; tk.bi[0] = t0 + e0 + u; }
#else
        float d = (dot + qn) + c[u].w;
        asm volatile("" : "+v"(d));  // keep the chains scalar (SLP paired them into v_pk_* + moves)
        tk.append(sh.sc.queue, tid, d, t0 + e0 + u, live && d < teff);
#endif
      }
#if PCOPS_KNN_ABL != 1
#if PCOPS_KNN_ABL == 2
      if (__any(tk.cnt > CAP - U)) tk.cnt = 0;  // diagnostic: appends and filters, no insertion
#else
      tk.maybe_drain(sh.sc.queue, tid, U);
#endif
      if (G > 1 && share) {
        // every wave's threshold, this wave's own included
        __hip_atomic_store(&sthr[w][lane], tk.thr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        float o[G];
#pragma unroll
        for (int g = 0; g < G; ++g) o[g] = __hip_atomic_load(&sthr[g][lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
        for (int g = 0; g < G; ++g) xthr = __builtin_fminf(xthr, o[g]);
      }
      // one strict test for both filters: d < own threshold (ties lose to the list's earlier
      // indices) and d <= any wave's threshold (a tie there may still win on its index), i.e.
      // d < nextup(xthr); nextup(+inf) = +inf keeps +inf distances out, as the unshared scan does
      teff = __builtin_fminf(tk.thr, next_up(xthr));
#endif
    }
    __syncthreads();
  }
  tk.drain(sh.sc.queue, tid);
  merge_and_store<KK, G>(sh.mb, tk.bd, tk.bi, w, lane, s < S, K, pad, N, idx + ((size_t)b * S + sc) * K,
                         dist ? dist + ((size_t)b * S + sc) * K : nullptr);
}

// generic C (feature space): candidates staged 32 at a time (32 x C floats),
// wave w takes candidates [w*32/G, (w+1)*32/G) of each tile; query channels
// read in 32-wide chunks, the per-candidate dot keeps the sequential channel
// order across chunks.
template <int KK, int G>
__global__ __launch_bounds__(64 * G) void knnC_kernel(const float *__restrict__ q, const float *__restrict__ p, int S,
                                                      int N, int C, int K, int pad, int *__restrict__ idx,
                                                      float *__restrict__ dist) {
  extern __shared__ __attribute__((aligned(16))) float smem[];  // [32][C] candidates + [32] norms
  constexpr int TN = 32, PW = TN / G;
  __shared__ MergeBuf<KK, G> mb;
  float *tc = smem;
  float *tn = smem + TN * C;
  const int b = blockIdx.y;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int s = blockIdx.x * 64 + lane;
  const float *qb = q + (size_t)b * S * C;
  const float *pb = p + (size_t)b * N * C;
  const int sc = s < S ? s : S - 1;
  const float *qq = qb + (size_t)sc * C;
  const float qn = torch_sumsq(qq, C);
  float bd[KK];
  int bi[KK];
#pragma unroll
  for (int k = 0; k < KK; ++k) {
    bd[k] = INFINITY;
    bi[k] = 0;
  }
  for (int t0 = 0; t0 < N; t0 += TN) {
    const int cnt = min(TN, N - t0);
    for (int e = threadIdx.x; e < TN * C; e += 64 * G) {
      const int kk = e / C;
      tc[e] = kk < cnt ? pb[(size_t)t0 * C + e] : 0.f;
    }
    __syncthreads();
    if (threadIdx.x < cnt) tn[threadIdx.x] = torch_sumsq(tc + threadIdx.x * C, C);
    float dot[PW];
#pragma unroll
    for (int k = 0; k < PW; ++k) dot[k] = 0.f;
    const float *tw = tc + w * PW * C;
    for (int c0 = 0; c0 < C; c0 += 32) {
      const int cw = min(32, C - c0);
      float qc[32];
#pragma unroll
      for (int c = 0; c < 32; ++c) qc[c] = c < cw ? qq[c0 + c] : 0.f;
      if (cw == 32) {
#pragma unroll
        for (int k = 0; k < PW; ++k) {
          const float *pc = tw + k * C + c0;
#pragma unroll
          for (int c = 0; c < 32; ++c) dot[k] = __builtin_fmaf(qc[c], pc[c], dot[k]);
        }
      } else {
#pragma unroll
        for (int k = 0; k < PW; ++k) {
          const float *pc = tw + k * C + c0;
          for (int c = 0; c < cw; ++c) dot[k] = __builtin_fmaf(qc[c], pc[c], dot[k]);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PW; ++k) {
      const int e = w * PW + k;
      if (e < cnt) topk_insert<KK>(bd, bi, ((-2.f * dot[k]) + qn) + tn[e], t0 + e);
    }
    __syncthreads();
  }
  merge_and_store<KK, G>(mb, bd, bi, w, lane, s < S, K, pad, N, idx + ((size_t)b * S + sc) * K,
                         dist ? dist + ((size_t)b * S + sc) * K : nullptr);
}


// generic C, v2 (C >= 32): distance tiles on a 4x4 register micro-tile.
// Block = 64 queries; candidates in tiles of 64, channels staged 32 at a time
// for both sides ([64][36] float images: the 16 lanes of a ds_read_b128 group
// read 16 consecutive rows -> conflict-free).  Thread (tq, tc) accumulates the
// dots of queries tq+16i x candidates tc+16j over the channels IN ORDER (the
// sequential fma chain of the oracle / torch CPU sgemm), so the distance bits
// equal knnC_kernel's.  The 64x64 distance tile goes to LDS, then thread
// (w, lane) runs the top-KK insertion for query `lane` over candidates
// [16w, 16w+16) of the tile -- the same 4-way split + (distance, index) merge
// as knnC_kernel.  The old kernel re-read every query row from global memory
// per candidate tile and issued one LDS read per 4 fma; this one issues one
// per 8 fma from LDS images and keeps 16 independent fma chains per thread.
template <int KK>
__global__ __launch_bounds__(256) void knnC2_kernel(const float *__restrict__ q, const float *__restrict__ p, int S,
                                                    int N, int C, int K, int pad, int *__restrict__ idx,
                                                    float *__restrict__ dist) {
  constexpr int QT = 64, CT = 64, CC = 32, LS = CC + 4;
  __shared__ __attribute__((aligned(16))) float sq[QT * LS];
  __shared__ __attribute__((aligned(16))) float sp[CT * LS];
  __shared__ float sd[QT][CT + 1];
  __shared__ float sqn[QT], spn[CT];
  constexpr int CAP = 16, NT = 256;
  __shared__ union {
    MergeBuf<KK, 4> mb;
    int2 queue[CAP * NT];
  } sh;
  const int b = blockIdx.y, t = threadIdx.x, tq = t >> 4, tc = t & 15;
  const int w = t >> 6, lane = t & 63;
  const int q0 = blockIdx.x * QT;
  const float *qb = q + (size_t)b * S * C;
  const float *pb = p + (size_t)b * N * C;
  const int s = q0 + lane;
  const int sc = s < S ? s : S - 1;
  if (t < QT) sqn[t] = torch_sumsq(qb + (size_t)sc * C, C);
  TopK<KK, CAP, NT> tk;
  tk.init();
  for (int t0 = 0; t0 < N; t0 += CT) {
    if (t < CT) spn[t] = t0 + t < N ? torch_sumsq(pb + (size_t)(t0 + t) * C, C) : 0.f;
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
    for (int c0 = 0; c0 < C; c0 += CC) {
      const int cw = min(CC, C - c0);
      for (int e = t; e < QT * CC; e += 256) {
        const int r = e / CC, c = e % CC;
        const int qi = q0 + r, pi = t0 + r;
        sq[r * LS + c] = (qi < S && c < cw) ? qb[(size_t)qi * C + c0 + c] : 0.f;
        sp[r * LS + c] = (pi < N && c < cw) ? pb[(size_t)pi * C + c0 + c] : 0.f;
      }
      __syncthreads();
      int c = 0;
      for (; c + 4 <= cw; c += 4) {
        float4 qv[4], pv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) qv[i] = *reinterpret_cast<const float4 *>(sq + (tq + 16 * i) * LS + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) pv[j] = *reinterpret_cast<const float4 *>(sp + (tc + 16 * j) * LS + c);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[i][j] = __builtin_fmaf(qv[i].x, pv[j].x, acc[i][j]);
            acc[i][j] = __builtin_fmaf(qv[i].y, pv[j].y, acc[i][j]);
            acc[i][j] = __builtin_fmaf(qv[i].z, pv[j].z, acc[i][j]);
            acc[i][j] = __builtin_fmaf(qv[i].w, pv[j].w, acc[i][j]);
          }
      }
      for (; c < cw; ++c) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_fmaf(sq[(tq + 16 * i) * LS + c], sp[(tc + 16 * j) * LS + c], acc[i][j]);
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        sd[tq + 16 * i][tc + 16 * j] = ((-2.f * acc[i][j]) + sqn[tq + 16 * i]) + spn[tc + 16 * j];
    __syncthreads();
    const int e1 = min(CT, N - t0);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = w * 16 + k;
      if (e < e1) tk.offer(sh.queue, t, sd[lane][e], t0 + e);
      if (k == 7 || k == 15) tk.maybe_drain(sh.queue, t, 8);
    }
    __syncthreads();
  }
  tk.drain(sh.queue, t);
  merge_and_store<KK, 4>(sh.mb, tk.bd, tk.bi, w, lane, s < S, K, pad, N, idx + ((size_t)b * S + sc) * K,
                         dist ? dist + ((size_t)b * S + sc) * K : nullptr);
}

// ----------------------------------------------------------------- C >= 32, streamed (v3)
// knnC2_kernel's arithmetic (4x4 register micro-tile, each distance a sequential fma chain over
// the channels in order, then ((-2 dot) + |q|^2) + |p|^2 with torch_sumsq norms) with the
// latency it exposed removed: at the model's shapes (S, N <= 1024, C = 64 / 256) its grid was
// 256 blocks of 4 waves (one wave per SIMD) whose every 32-channel chunk was staged by scalar
// loads between two barriers, and each candidate tile recomputed |p|^2 serially from global
// memory.  Here the norms come from a separate pass (knn_norms_kernel), the (query chunk,
// candidate chunk) stream is double-buffered through registers (float4 loads of step k+1 issue
// before step k's fmas, one barrier per step), and the candidate range is split over `splits`
// blocks whose sorted partial lists knn_merge_kernel merges as (distance, index) pairs.
__global__ __launch_bounds__(256) void knn_norms_kernel(const float *__restrict__ x, long long rows, int C,
                                                        float *__restrict__ out) {
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r < rows) out[r] = torch_sumsq(x + r * C, C);
}

template <int KK>
__global__ __launch_bounds__(256) void knnC3_kernel(const float *__restrict__ q, const float *__restrict__ p,
                                                    const float *__restrict__ qnorm, const float *__restrict__ pnorm,
                                                    int S, int N, int C, int splits, int span, int K, int pad,
                                                    int *__restrict__ idx, float *__restrict__ dist,
                                                    float *__restrict__ part_d, int *__restrict__ part_i) {
  constexpr int QT = 64, CT = 64, CC = 32, LS = CC + 4, SLOT = QT * LS;
  constexpr int CAP = 8, NT = 256;
  // one LDS arena: the two chunk slots of each side; at a tile's end the distance tile over
  // the query slots (between barriers); at the end the wave merge over all of it
  constexpr size_t kArena = sizeof(MergeBuf<KK, 4>) > 4 * SLOT * sizeof(float) ? sizeof(MergeBuf<KK, 4>)
                                                                                   : 4 * SLOT * sizeof(float);
  static_assert(QT * (CT + 1) <= 2 * SLOT, "distance tile must fit the query slots");
  __shared__ __attribute__((aligned(16))) unsigned char arena[kArena];
  __shared__ int2 queue_[CAP * NT];
  float *sq = reinterpret_cast<float *>(arena);
  float *sp = sq + 2 * SLOT;
  float(*sd)[CT + 1] = reinterpret_cast<float(*)[CT + 1]>(arena);
  struct {
    int2 *queue;
    MergeBuf<KK, 4> &mb;
  } sh{queue_, *reinterpret_cast<MergeBuf<KK, 4> *>(arena)};
  const int b = blockIdx.y, t = threadIdx.x, tq = t >> 4, tc = t & 15;
  const int w = t >> 6, lane = t & 63;
  const int qt = blockIdx.x / splits, sp_i = blockIdx.x - qt * splits;
  const int q0 = qt * QT;
  const int n0 = sp_i * span, n1 = min(N, n0 + span);
  const float *qb = q + (size_t)b * S * C;
  const float *pb = p + (size_t)b * N * C;
  const int s = q0 + lane;
  const int sc = s < S ? s : S - 1;
  TopK<KK, CAP, NT> tk;
  tk.init();
  const int nch = (C + CC - 1) / CC, ntile = (n1 - n0 + CT - 1) / CT, steps = nch * ntile;
  // this thread's two float4 of each side per step: rows r = e / 8 (e = t, t + 256), channels 4 (e % 8)
  float4 rq[2], rp[2];
  auto load = [&](int k) {
    const int tile = k / nch, ch = k - tile * nch;
    const int t0 = n0 + tile * CT, c0 = ch * CC, cw = min(CC, C - c0);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = t + 256 * u, r = e >> 3, c = (e & 7) * 4;
      const int qi = q0 + r, pi = t0 + r;
      if (cw == CC) {
        rq[u] = qi < S ? *reinterpret_cast<const float4 *>(qb + (size_t)qi * C + c0 + c) : make_float4(0, 0, 0, 0);
        rp[u] = pi < n1 ? *reinterpret_cast<const float4 *>(pb + (size_t)pi * C + c0 + c) : make_float4(0, 0, 0, 0);
      } else {
        float a[4], z[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a[i] = (qi < S && c + i < cw) ? qb[(size_t)qi * C + c0 + c + i] : 0.f;
          z[i] = (pi < n1 && c + i < cw) ? pb[(size_t)pi * C + c0 + c + i] : 0.f;
        }
        rq[u] = make_float4(a[0], a[1], a[2], a[3]);
        rp[u] = make_float4(z[0], z[1], z[2], z[3]);
      }
    }
  };
  float acc[4][4];
  if (steps > 0) load(0);
  for (int k = 0; k < steps; ++k) {
    const int slot = k & 1, tile = k / nch, ch = k - tile * nch;
    const int t0 = n0 + tile * CT, cw = min(CC, C - ch * CC);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = t + 256 * u, r = e >> 3, c = (e & 7) * 4;
      *reinterpret_cast<float4 *>(sq + slot * SLOT + r * LS + c) = rq[u];
      *reinterpret_cast<float4 *>(sp + slot * SLOT + r * LS + c) = rp[u];
    }
    __syncthreads();
    if (k + 1 < steps) load(k + 1);
    if (ch == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
    }
    const float *cq = sq + slot * SLOT, *cp = sp + slot * SLOT;
    int c = 0;
    for (; c + 4 <= cw; c += 4) {
      float4 qv[4], pv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) qv[i] = *reinterpret_cast<const float4 *>(cq + (tq + 16 * i) * LS + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) pv[j] = *reinterpret_cast<const float4 *>(cp + (tc + 16 * j) * LS + c);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[i][j] = __builtin_fmaf(qv[i].x, pv[j].x, acc[i][j]);
          acc[i][j] = __builtin_fmaf(qv[i].y, pv[j].y, acc[i][j]);
          acc[i][j] = __builtin_fmaf(qv[i].z, pv[j].z, acc[i][j]);
          acc[i][j] = __builtin_fmaf(qv[i].w, pv[j].w, acc[i][j]);
        }
    }
    for (; c < cw; ++c) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_fmaf(cq[(tq + 16 * i) * LS + c], cp[(tc + 16 * j) * LS + c], acc[i][j]);
    }
    if (ch == nch - 1) {  // the tile's distances, then its selection
      __syncthreads();    // every thread is past its reads of the query slots
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qr = min(q0 + tq + 16 * i, S - 1);
        const float qn = qnorm[(size_t)b * S + qr];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int pr = min(t0 + tc + 16 * j, N - 1);
          sd[tq + 16 * i][tc + 16 * j] = ((-2.f * acc[i][j]) + qn) + pnorm[(size_t)b * N + pr];
        }
      }
      __syncthreads();
      const int e1 = min(CT, n1 - t0);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        // 8 distances read first, together (inside the offer branches each read waited alone:
        // the compiler cannot move it above a queue write); columns past e1 hold clamped rows
        float dv[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) dv[kk] = sd[lane][w * 16 + 8 * h + kk];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const int e = w * 16 + 8 * h + kk;
          tk.append(sh.queue, t, dv[kk], t0 + e, e < e1 && dv[kk] < tk.thr);
        }
        tk.maybe_drain(sh.queue, t, 8);
      }
      __syncthreads();    // the distance tile is read before the next step's query chunk lands
    }
  }
  tk.drain(sh.queue, t);
  if (splits == 1) {
    merge_and_store<KK, 4>(sh.mb, tk.bd, tk.bi, w, lane, s < S, K, pad, N, idx + ((size_t)b * S + sc) * K,
                           dist ? dist + ((size_t)b * S + sc) * K : nullptr);
    return;
  }
  // the block's sorted top-KK over its candidate range (all KK entries, no pad), for the merge
  const size_t row = (((size_t)b * S + sc) * splits + sp_i) * KK;
  merge_and_store<KK, 4>(sh.mb, tk.bd, tk.bi, w, lane, s < S, KK, 0, n1 - n0 < KK ? n1 - n0 : KK, part_i + row,
                         part_d + row);
}

// per query: the splits' sorted (distance, index) lists merged lexicographically (the index-order
// scan's result: every list is the exact top-KK of its range), entries [pad, pad + K) stored
template <int KK>
__global__ __launch_bounds__(256) void knn_merge_kernel(const float *__restrict__ part_d, const int *__restrict__ part_i,
                                                        long long rows, int splits, int span, int N, int K, int pad,
                                                        int *__restrict__ idx, float *__restrict__ dist) {
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  int head[16];
  for (int g = 0; g < splits; ++g) head[g] = 0;
  for (int o = 0; o < K + pad; ++o) {
    float bdv = INFINITY;
    int biv = INT_MAX, bw = -1;
    for (int g = 0; g < splits; ++g) {
      const int avail = min(KK, min(N, (g + 1) * span) - g * span);
      if (head[g] < avail) {
        const size_t e = (r * splits + g) * KK + head[g];
        const float dv = part_d[e];
        const int iv = part_i[e];
        if (bw < 0 || dv < bdv || (dv == bdv && iv < biv)) {
          bdv = dv;
          biv = iv;
          bw = g;
        }
      }
    }
    if (bw >= 0) head[bw] += 1;
    if (o >= pad) {
      const bool ok = o < N && bw >= 0;
      idx[r * K + o - pad] = ok ? biv : 0;
      if (dist) dist[r * K + o - pad] = ok ? bdv : 0.f;
    }
  }
}

bool knn_v1() {  // PCOPS_KNN_V1=1: the first-generation feature-space kernel (A/B runs)
  static const bool v = [] {
    const char *e = getenv("PCOPS_KNN_V1");
    return e && e[0] == '1';
  }();
  return v;
}

bool knn_share_on() {  // PCOPS_KNN_SHARE=0: no cross-wave threshold sharing (A/B)
  static const bool v = [] {
    const char *e = getenv("PCOPS_KNN_SHARE");
    return !(e && e[0] == '0');
  }();
  return v;
}

template <int KK>
int launch_knn(const float *q, const float *p, int B, int S, int N, int C, int K, int pad, int *idx, float *dist,
               hipStream_t st) {
  constexpr int G = KK <= 16 ? 4 : (KK <= 32 ? 2 : 1);
  const dim3 grid((S + 63) / 64, B);
  if (C == 3) {
    if constexpr (KK <= 16) {
      if ((long)grid.x * grid.y < 768) {  // < 3 blocks per CU: more waves per query
        hipLaunchKernelGGL((knn3_kernel<KK, 8, 1024>), grid, dim3(512), 0, st, q, p, S, N, K, pad, idx, dist,
                           knn_share_on());
        PC_CHECK_LAUNCH();
        return PCOPS_OK;
      }
      hipLaunchKernelGGL((knn3_kernel<KK, 4, 512>), grid, dim3(256), 0, st, q, p, S, N, K, pad, idx, dist,
                         knn_share_on());
    } else {
      hipLaunchKernelGGL((knn3_kernel<KK, G, 1024>), grid, dim3(64 * G), 0, st, q, p, S, N, K, pad, idx, dist,
                         knn_share_on());
    }
    PC_CHECK_LAUNCH();
    return PCOPS_OK;
  }
  if constexpr (KK <= 32) {
    if (C >= 32 && !knn_v1()) {
      hipLaunchKernelGGL((knnC2_kernel<KK>), grid, dim3(256), 0, st, q, p, S, N, C, K, pad, idx, dist);
      PC_CHECK_LAUNCH();
      return PCOPS_OK;
    }
  }
  {
    const size_t lds = sizeof(float) * (32 * (size_t)C + 32);
    hipLaunchKernelGGL((knnC_kernel<KK, G>), grid, dim3(64 * G), lds, st, q, p, S, N, C, K, pad, idx, dist);
  }
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

}  // namespace

// feature-space kNN scratch: both clouds' norms, then the splits' partial lists
int kk_of(int kk) { return kk <= 4 ? 4 : kk <= 8 ? 8 : kk <= 16 ? 16 : kk <= 20 ? 20 : 32; }
int knnC3_splits(int B, int S, int N) {
  const int blocks = (S + 63) / 64 * B;
  int sp = (1024 + blocks - 1) / blocks;
  sp = sp < 1 ? 1 : (sp > 16 ? 16 : sp);
  while (sp > 1 && (N + sp - 1) / sp < 64) --sp;
  return sp;
}
size_t knnC3_bytes(int B, int S, int N, int kk) {
  auto a = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t parts = (size_t)B * S * knnC3_splits(B, S, N) * kk_of(kk);
  return a((size_t)B * S * 4) + a((size_t)B * N * 4) + 2 * a(parts * 4);
}

template <int KK>
int launch_knnC3(const float *q, const float *p, int B, int S, int N, int C, int K, int pad, int *idx, float *dist,
                 void *ws, hipStream_t st) {
  auto a = [](size_t x) { return (x + 255) & ~size_t(255); };
  char *w = (char *)ws;
  float *qn = (float *)w;
  w += a((size_t)B * S * 4);
  float *pn = (float *)w;
  w += a((size_t)B * N * 4);
  const int splits = knnC3_splits(B, S, N);
  const size_t parts = (size_t)B * S * splits * KK;
  float *pd = (float *)w;
  w += a(parts * 4);
  int *pi = (int *)w;
  const long long rq = (long long)B * S, rp = (long long)B * N;
  const bool self = q == p && S == N;
  hipLaunchKernelGGL(knn_norms_kernel, dim3((unsigned)((rp + 255) / 256)), dim3(256), 0, st, p, rp, C, pn);
  if (!self) hipLaunchKernelGGL(knn_norms_kernel, dim3((unsigned)((rq + 255) / 256)), dim3(256), 0, st, q, rq, C, qn);
  const int span = ((N + splits - 1) / splits + 63) / 64 * 64;
  const dim3 grid((S + 63) / 64 * splits, B);
  hipLaunchKernelGGL((knnC3_kernel<KK>), grid, dim3(256), 0, st, q, p, self ? pn : qn, pn, S, N, C, splits, span, K,
                     pad, idx, dist, pd, pi);
  if (splits > 1)
    hipLaunchKernelGGL((knn_merge_kernel<KK>), dim3((unsigned)((rq + 255) / 256)), dim3(256), 0, st, pd, pi, rq,
                       splits, span, N, K, pad, idx, dist);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

bool knnC3_on() {  // PCOPS_KNN_C3=0: knnC2_kernel (A/B)
  static const bool v = [] {
    const char *e = getenv("PCOPS_KNN_C3");
    return !(e && e[0] == '0');
  }();
  return v;
}

// the one predicate for the streamed, candidate-split form: the size query and the call agree, so
// a caller never grows scratch that the call would not use (kk = K + pad)
bool knnC3_eligible(int C, int kk) { return knnC3_on() && C >= 32 && C <= 512 && (C & 3) == 0 && kk <= 32 && !knn_v1(); }

extern "C" unsigned long long pcops_knn_workspace_bytes(int B, int S, int N, int C, int K) {
  if (B <= 0 || S <= 0 || N <= 0 || C <= 0 || K <= 0) return 0;
  return knnC3_eligible(C, K) ? knnC3_bytes(B, S, N, K) : 0;
}

extern "C" int pcops_knn(const float *q, const float *p, int B, int S, int N, int C, int K, int pad, int *idx,
                         float *dist, pcops_stream_t stream);

// pcops_knn with scratch: C >= 32 (C % 4 == 0, K + pad <= 32) takes the streamed, candidate-split
// form (knnC3_kernel + knn_merge_kernel); every other case, or a short workspace, is pcops_knn.
// Same output as pcops_knn bit for bit.
extern "C" int pcops_knn_ws(const float *q, const float *p, int B, int S, int N, int C, int K, int pad, int *idx,
                            float *dist, void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream) {
  if (B < 0 || S < 0 || N < 0 || C <= 0 || K < 0 || pad < 0 || C > 512) return PCOPS_ERR_INVALID;
  if (B == 0 || S == 0 || K == 0) return PCOPS_OK;
  if (!q || !p || !idx || N <= 0) return PCOPS_ERR_INVALID;
  if (K + pad > N) return PCOPS_ERR_INVALID;
  const int kk = K + pad;
  if (knnC3_eligible(C, kk) && workspace && workspace_bytes >= knnC3_bytes(B, S, N, kk)) {
    hipStream_t st = (hipStream_t)stream;
    switch (kk_of(kk)) {
      case 4: return launch_knnC3<4>(q, p, B, S, N, C, K, pad, idx, dist, workspace, st);
      case 8: return launch_knnC3<8>(q, p, B, S, N, C, K, pad, idx, dist, workspace, st);
      case 16: return launch_knnC3<16>(q, p, B, S, N, C, K, pad, idx, dist, workspace, st);
      case 20: return launch_knnC3<20>(q, p, B, S, N, C, K, pad, idx, dist, workspace, st);
      default: return launch_knnC3<32>(q, p, B, S, N, C, K, pad, idx, dist, workspace, st);
    }
  }
  return pcops_knn(q, p, B, S, N, C, K, pad, idx, dist, stream);
}

extern "C" int pcops_knn(const float *q, const float *p, int B, int S, int N, int C, int K, int pad, int *idx,
                         float *dist, pcops_stream_t stream) {
  if (B < 0 || S < 0 || N < 0 || C <= 0 || K < 0 || pad < 0 || C > 512) return PCOPS_ERR_INVALID;
  if (B == 0 || S == 0 || K == 0) return PCOPS_OK;
  if (!q || !p || !idx || N <= 0) return PCOPS_ERR_INVALID;
  const int kk = K + pad;
  hipStream_t st = (hipStream_t)stream;
  if (kk <= 4) return launch_knn<4>(q, p, B, S, N, C, K, pad, idx, dist, st);
  if (kk <= 8) return launch_knn<8>(q, p, B, S, N, C, K, pad, idx, dist, st);
  if (kk <= 16) return launch_knn<16>(q, p, B, S, N, C, K, pad, idx, dist, st);
  if (kk <= 20) return launch_knn<20>(q, p, B, S, N, C, K, pad, idx, dist, st);
  if (kk <= 32) return launch_knn<32>(q, p, B, S, N, C, K, pad, idx, dist, st);
  if (kk <= 64) return launch_knn<64>(q, p, B, S, N, C, K, pad, idx, dist, st);
  return PCOPS_ERR_UNSUPPORTED;
}
