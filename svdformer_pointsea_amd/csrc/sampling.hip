// Furthest point sampling + gather (pointnet2_ops sampling.cpp / sampling_gpu.cu).
//
// FPS design (gfx950): one workgroup per cloud, the whole cloud and its running
// min-distance kept in VGPRs (thread t owns points t, t+T, t+2T, ... -- the
// reference's own thread->point map, so the in-thread first-index rule carries
// over unchanged).  One round = register sweep (10 VALU ops / point) ->
// wave max via DPP -> tie-break lane picked on the SCALAR unit (smallest
// bit-reversed thread id among equal maxima == the reference LDS tree's
// winner, see oracle/pcops_oracle.c) -> one LDS slot per wave (double
// buffered by round parity) -> ONE barrier -> every thread reduces the 8 slots
// itself (broadcast LDS reads), so the next centre's coordinates arrive with
// the argmax and no second barrier or global read is needed.
// Index parity with sampling_gpu.cu:69-173 is bit-exact (same fused distance,
// same tie order, same |p|^2 <= 1e-3 skip).
#include <climits>
#include <cstdlib>
#include <cmath>

#include "common.h"

// Diagnostic build only (tools/fps_probe.hip defines FPS_STAMPS): per-segment
// s_memtime sums of block 0 / thread 0, never present in libpcops.so.
#ifdef FPS_STAMPS
__device__ unsigned long long g_fps_stamps[8];
__device__ unsigned long long g_fps_wave_stamps[16][4];
#define FPS_STAMP_DECL unsigned long long _st_prev = __builtin_amdgcn_s_memtime(), _st_acc[4] = {0, 0, 0, 0};
#define FPS_STAMP(seg)                                          \
  {                                                             \
    __builtin_amdgcn_sched_barrier(0);                          \
    unsigned long long _n;                                      \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_n)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                          \
    _st_acc[seg] += _n - _st_prev;                              \
    _st_prev = _n;                                              \
  }
#define FPS_STAMP_FLUSH \
  if (blockIdx.x == 0 && threadIdx.x == 0)                      \
    for (int _s = 0; _s < 4; ++_s) g_fps_stamps[_s] = _st_acc[_s]; \
  if (blockIdx.x == 0 && (threadIdx.x & 63) == 0)               \
    for (int _s = 0; _s < 4; ++_s) g_fps_wave_stamps[threadIdx.x >> 6][_s] = _st_acc[_s];
#else
#define FPS_STAMP_DECL
#define FPS_STAMP(seg)
#define FPS_STAMP_FLUSH
#endif

namespace {

constexpr int kFpsThreads = 512;  // == TOTAL_THREADS (cuda_utils.h:13) for N >= 512
constexpr int kFpsMaxPPT = 32;    // 512 * 32 = 16384 points resident in VGPRs (k < 2^14)

// Distances are >= 0 (or the -1 "never" marker), so IEEE fminf/fmaxf and
// '>' on them equal signed-integer min/max/'>' on their bit patterns; the
// integer forms need no NaN canonicalisation (v_max x,x,x) in the sweep.
__device__ __forceinline__ int fbits(float f) { return __float_as_int(f); }

// Hardware lane -> reference thread map.  The reference (T threads) breaks
// ties by the smallest bit-reversed thread id r = rev_L(t), then the smallest
// k.  Each reference thread's points may be split over SPLIT hardware
// threads ("halves", SPLIT*PPT points per reference thread).  Hardware
// thread (w, l) with half h = w / NWT, wv = w % NWT gets the reference thread
// whose r = l*NWT + wv, so inside a wave the tie-winner is the LOWEST set lane
// of the ballot (s_ff1), and across waves the order key is r' = r*SPLIT + h.
// The cross-wave step packs (distance bits, 1023 - r', k) into one 64-bit
// key and max-reduces the <= 16 per-wave slots with DPP in one row of lanes.
// ALLRED: after the one barrier every wave reduces the (round-parity double
// buffered) slots itself, so the centre arrives without the leader wave's
// second barrier and LDS round trip; ALLRED = false is the leader-wave form.
// Measured: ALLRED wins with 8 waves (32x2048->512: 0.318 -> 0.307 ms) and
// loses with 16, where 16 concurrent reductions contend for the VALU
// (32x16384->2048: 2.78 -> 2.91 ms), so 16-wave blocks keep the leader.
// CNT: per-cloud valid counts (pcops_furthest_point_sampling_counts) -- points k >= counts[b] are
// absent, exactly as the reference treats the zero rows of a zero-padded buffer (|p|^2 <= 1e-3:
// never selected, never updated); slot i of this wave covers k in [T*(PPT*half + i), +T), so the
// slots wholly past the count are skipped by a wave-uniform branch.
template <int PPT, bool ALLRED, bool CNT = false>
__global__ __launch_bounds__(ALLRED ? 512 : 1024) void fps_reg_kernel(const float *__restrict__ xyz, int N, int M, int T, int L,
                                                        int NWT, int SPLIT, int *__restrict__ idx,
                                                        const int *__restrict__ counts = nullptr) {
  const int b = blockIdx.x;
  const float *p = xyz + (size_t)b * N * 3;
  int *out = idx + (size_t)b * M;
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  constexpr int kNeverBits = 0xBF800000;  // -1.0f
  const int half = w / NWT, wv = w - half * NWT;
  const int rkey = lane * NWT + wv;  // == rev_L(reference thread)
  const bool active = rkey < T;
  const int tref = active ? (int)bitrev_bits((unsigned)rkey, L) : 0;
  const int kbase = tref + T * PPT * half;
  const int nb = CNT ? min(max(counts[b], 0), N) : N;
  // slots of this wave holding any point below nb (wave-uniform)
  const int nsl = CNT ? __builtin_amdgcn_readfirstlane((nb + T - 1) / T - PPT * half) : PPT;

  typedef float fvec __attribute__((ext_vector_type(PPT)));
  typedef int ivec __attribute__((ext_vector_type(PPT)));
  fvec px, py, pz;
  ivec tmp;  // running min distance, as float bits
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int k = kbase + T * i;
    if (active && k < nb) {
      px[i] = p[3 * k];
      py[i] = p[3 * k + 1];
      pz[i] = p[3 * k + 2];
      const float mag = sqd3(px[i], py[i], pz[i]);
      tmp[i] = ((double)mag <= 1e-3) ? kNeverBits : fbits(1e10f);  // sampling_gpu.cu:100-101
    } else {
      px[i] = py[i] = pz[i] = 0.f;
      tmp[i] = kNeverBits;
    }
  }
  // per-wave slots: key (hi, lo) + coords; the leader wave's result
  __shared__ uint2 skey2[2][16];
  __shared__ float4 sxyz2[2][16];
  __shared__ float4 sres;
  if (t < 32) {
    skey2[t >> 4][t & 15] = make_uint2(0u, 0u);  // absent waves never win
    sxyz2[t >> 4][t & 15] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();

  const float x0 = p[0], y0 = p[1], z0 = p[2];
  float ox = x0, oy = y0, oz = z0;
  if (t == 0 && M > 0) out[0] = 0;
  FPS_STAMP_DECL
  for (int j = 1; j < M; ++j) {
    uint2 *skey = skey2[ALLRED ? (j & 1) : 0];
    float4 *sxyz = sxyz2[ALLRED ? (j & 1) : 0];
    // sweep: 8 VALU ops / point, no compare/select chain -- the lane only
    // tracks its max; the winning slot is recovered once per wave below.
    int best = kNeverBits;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      if (!CNT || i < nsl) {   // slots wholly past the count hold no point (wave-uniform branch)
        int d = fbits(sqd3(px[i] - ox, py[i] - oy, pz[i] - oz));
        // PPT >= 16: keep the distance chains scalar -- LLVM's SLP pass pairs
        // them into v_pk_add/mul/fma_f32, which on gfx950 issue at half rate
        // and add hazard s_nops (16384->2048: 2.78 -> 2.49 ms scalar); at small
        // PPT the packed form measured slightly faster, so it is left there
        if constexpr (PPT >= 16) asm volatile("" : "+v"(d));
        tmp[i] = min(d, tmp[i]);
        best = max(best, tmp[i]);
      }
    }
    FPS_STAMP(0)
    const int wmax = wave_max_i32(best);
    const uint64_t tied = __ballot(best == wmax);
    const int wl = (int)__builtin_ctzll(tied);  // lowest lane == smallest r in this wave
    // first slot of lane wl holding the maximum (in-thread strict '>' rule):
    // every lane finds its own first slot equal to wmax with VALU selects
    // (two interleaved chains), then one readlane from lane wl -- the former
    // PPT serial readlane + scalar compare steps were ~27 cycles each on the
    // round's critical path
    int wbi;
    {
      int b0 = PPT - 1, b1 = PPT - 1;
#pragma unroll
      for (int i = PPT - 2; i >= 0; i -= 2) {
        b0 = (tmp[i] == wmax) ? i : b0;
        if (i >= 1) b1 = (tmp[i - 1] == wmax) ? i - 1 : b1;
      }
      wbi = __builtin_amdgcn_readlane(min(b0, b1), wl);
    }
    // uniform-index extraction (s_set_gpr_idx / movrel on a register vector)
    const float cx = px[wbi], cy = py[wbi], cz = pz[wbi];
    if (lane == wl) {
      const int r = wl * NWT + wv;
      const int rp = r * SPLIT + half;
      const int k = (int)bitrev_bits((unsigned)r, L) + T * (PPT * half + wbi);
      // lo word: (1023 - r') in [31:18], wave id in [17:14], k in [13:0]
      skey[w] = make_uint2((unsigned)wmax ^ 0x80000000u,
                           ((unsigned)(1023 - rp) << 18) | ((unsigned)w << 14) | (unsigned)k);
      sxyz[w] = make_float4(cx, cy, cz, 0.f);
    }
    FPS_STAMP(1)
    lds_barrier();
    FPS_STAMP(2)
    float4 rv;
    if (ALLRED || w == 0) {  // 64-bit max over the <= 16 slots in one DPP row
      const uint2 kv = skey[lane & 15];
      const float4 cv = sxyz[lane & 15];
      unsigned long long key = ((unsigned long long)kv.x << 32) | kv.y;
#define FPS_DPP_MAX(CTRL)                                                                                   \
  {                                                                                                        \
    const unsigned hi = __builtin_amdgcn_update_dpp(0, (int)(key >> 32), CTRL, 0xF, 0xF, false);           \
    const unsigned lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)key, CTRL, 0xF, 0xF, false);         \
    const unsigned long long o = ((unsigned long long)hi << 32) | lo;                                      \
    key = o > key ? o : key;                                                                               \
  }
      FPS_DPP_MAX(0xB1)
      FPS_DPP_MAX(0x4E)
      FPS_DPP_MAX(0x141)
      FPS_DPP_MAX(0x140)
#undef FPS_DPP_MAX
      const unsigned ghi = __builtin_amdgcn_readfirstlane((unsigned)(key >> 32));
      const unsigned glo = __builtin_amdgcn_readfirstlane((unsigned)key);
      if ((int)(ghi ^ 0x80000000u) != kNeverBits) {
        const int gw = (int)((glo >> 14) & 15u);  // winning wave == its slot lane
        const int k = (int)(glo & 0x3FFFu);
        if constexpr (ALLRED) {
          rv = make_float4(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(cv.x), gw)),
                           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cv.y), gw)),
                           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cv.z), gw)), __int_as_float(k));
        } else if (lane == gw) {
          sres = make_float4(cv.x, cv.y, cv.z, __int_as_float(k));
        }
      } else {  // no valid point at all: the reference's dists_i[0] == 0
        if constexpr (ALLRED) {
          rv = make_float4(x0, y0, z0, __int_as_float(0));
        } else if (lane == 0) {
          sres = make_float4(x0, y0, z0, __int_as_float(0));
        }
      }
    }
    if constexpr (!ALLRED) {
      lds_barrier();
      rv = sres;
    }
    ox = rv.x;
    oy = rv.y;
    oz = rv.z;
    if (t == 0) out[j] = __float_as_int(rv.w);
    FPS_STAMP(3)
  }
  FPS_STAMP_FLUSH
}

// One wave per cloud (small clouds): each lane holds R = T / 64 reference threads (r = lane * R + j,
// so lane order is r order), PPL = R * PPT slots ordered by (j, i) -- the reference thread's k = tref +
// T * i -- so "lowest lane with the max, then its first slot" is the reference's tie order (smallest
// r, then smallest k).  A round is the sweep + one DPP wave max + the first-slot search + readlanes:
// no LDS, no barrier.  Measured (B = 32, tools/fps_bench.py, profiles/r3_fps_wave_ab.txt): 512 -> 128
// 0.471 -> 0.406 us/round, 1024 -> 256 equal, 2048 -> 512 0.577 -> 0.830 (the one wave's sweep of 32
// slots is VALU-bound where 8 waves split it), so it runs only up to 8 slots per lane (<= 512 points).
template <int PPL>
__global__ __launch_bounds__(64) void fps_wave_kernel(const float *__restrict__ xyz, int N, int M, int T, int L,
                                                      int R, int PPT, int *__restrict__ idx,
                                                      const int *__restrict__ counts) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const float *p = xyz + (size_t)b * N * 3;
  const int nb = counts ? min(max(counts[b], 0), N) : N;
  int *out = idx + (size_t)b * M;
  constexpr int kNeverBits = 0xBF800000;  // -1.0f
  float px[PPL], py[PPL], pz[PPL];
  int tmp[PPL];
#pragma unroll
  for (int s = 0; s < PPL; ++s) {
    const int j = s / PPT, i = s - j * PPT;  // PPT is uniform; s, j, i compile-time per slot only when PPT is
    const int r = lane * R + j;
    const int k = (int)bitrev_bits((unsigned)r, L) + T * i;
    if (j < R && r < T && k < nb) {
      px[s] = p[3 * k];
      py[s] = p[3 * k + 1];
      pz[s] = p[3 * k + 2];
      const float mag = sqd3(px[s], py[s], pz[s]);
      tmp[s] = ((double)mag <= 1e-3) ? kNeverBits : fbits(1e10f);  // sampling_gpu.cu:100-101
    } else {
      px[s] = py[s] = pz[s] = 0.f;
      tmp[s] = kNeverBits;
    }
  }
  const float x0 = p[0], y0 = p[1], z0 = p[2];
  float ox = x0, oy = y0, oz = z0;
  if (lane == 0 && M > 0) out[0] = 0;
  for (int jr = 1; jr < M; ++jr) {
    int best = kNeverBits;
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      int d = fbits(sqd3(px[s] - ox, py[s] - oy, pz[s] - oz));
      if constexpr (PPL >= 16) asm volatile("" : "+v"(d));  // scalar chains (see fps_reg_kernel)
      tmp[s] = min(d, tmp[s]);
      best = max(best, tmp[s]);
    }
    const int wmax = wave_max_i32(best);
    const uint64_t tied = __ballot(best == wmax);
    const int wl = (int)__builtin_ctzll(tied);
    int b0 = PPL - 1, b1 = PPL - 1;
#pragma unroll
    for (int s = PPL - 2; s >= 0; s -= 2) {
      b0 = (tmp[s] == wmax) ? s : b0;
      if (s >= 1) b1 = (tmp[s - 1] == wmax) ? s - 1 : b1;
    }
    const int wbi = __builtin_amdgcn_readlane(min(b0, b1), wl);
    int k;
    if (wmax != kNeverBits) {
      ox = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(px[wbi]), wl));
      oy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(py[wbi]), wl));
      oz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pz[wbi]), wl));
      const int j = wbi / PPT;
      k = (int)bitrev_bits((unsigned)(wl * R + j), L) + T * (wbi - j * PPT);
    } else {  // no valid point at all: the reference's dists_i[0] == 0
      ox = x0, oy = y0, oz = z0;
      k = 0;
    }
    if (lane == 0) out[jr] = k;
  }
}

// NW waves per cloud, each lane holding R = T / (64 NW) reference threads (r = (w * 64 + lane) * R + j:
// lane and wave order are r order) with PPL = R * PPT slots ordered by (j, i), as fps_wave_kernel: the
// wave's winner is its lowest lane with the maximum, that lane's first slot; the waves' winners meet in
// one LDS slot row (double buffered by round parity, ONE barrier), where the lowest wave with the
// maximum wins -- the reference's order (distance, then smallest r, then smallest k).  Fewer waves than
// fps_reg_kernel's one per 64 reference threads: a shorter cross-wave step for a longer sweep.  Used
// for 512-thread clouds of 5-8 points per reference thread (2048 < N <= 4096): the model's 2304-point
// merge 0.657 -> 0.585 us per round, 4096 equal; at 2048 points (4 per thread) the 8-wave kernel stays
// ahead (0.576 vs 0.62), and 2-wave blocks lose everywhere (profiles/r5_fps_mw_ab.txt).
template <int PPL, int NW>
__global__ __launch_bounds__(64 * NW) void fps_mw_kernel(const float *__restrict__ xyz, int N, int M, int T, int L,
                                                          int R, int PPT, int *__restrict__ idx,
                                                          const int *__restrict__ counts) {
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float *p = xyz + (size_t)b * N * 3;
  const int nb = counts ? min(max(counts[b], 0), N) : N;
  int *out = idx + (size_t)b * M;
  constexpr int kNeverBits = 0xBF800000;  // -1.0f
  const int gl = w * 64 + lane;
  typedef float fvec __attribute__((ext_vector_type(PPL)));
  typedef int ivec __attribute__((ext_vector_type(PPL)));
  fvec px, py, pz;   // register vectors: a uniform index extracts by movrel (fps_reg_kernel)
  ivec tmp;
#pragma unroll
  for (int s = 0; s < PPL; ++s) {
    const int j = s / PPT, i = s - j * PPT;
    const int r = gl * R + j;
    const int k = (int)bitrev_bits((unsigned)r, L) + T * i;
    if (j < R && r < T && k < nb) {
      px[s] = p[3 * k];
      py[s] = p[3 * k + 1];
      pz[s] = p[3 * k + 2];
      const float mag = sqd3(px[s], py[s], pz[s]);
      tmp[s] = ((double)mag <= 1e-3) ? kNeverBits : fbits(1e10f);  // sampling_gpu.cu:100-101
    } else {
      px[s] = py[s] = pz[s] = 0.f;
      tmp[s] = kNeverBits;
    }
  }
  __shared__ int sd[2][NW];       // per-wave maximum (float bits)
  __shared__ float4 sc[2][NW];    // its point (x, y, z, k as int bits)
  const float x0 = p[0], y0 = p[1], z0 = p[2];
  float ox = x0, oy = y0, oz = z0;
  if (threadIdx.x == 0 && M > 0) out[0] = 0;
  for (int jr = 1; jr < M; ++jr) {
    const int par = jr & 1;
    int best = kNeverBits;
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      int d = fbits(sqd3(px[s] - ox, py[s] - oy, pz[s] - oz));
      if constexpr (PPL >= 16) asm volatile("" : "+v"(d));  // scalar chains (see fps_reg_kernel)
      tmp[s] = min(d, tmp[s]);
      best = max(best, tmp[s]);
    }
    const int wmax = wave_max_i32(best);
    const uint64_t tied = __ballot(best == wmax);
    const int wl = (int)__builtin_ctzll(tied);
    int b0 = PPL - 1, b1 = PPL - 1;
#pragma unroll
    for (int s = PPL - 2; s >= 0; s -= 2) {
      b0 = (tmp[s] == wmax) ? s : b0;
      if (s >= 1) b1 = (tmp[s - 1] == wmax) ? s - 1 : b1;
    }
    const int wbi = __builtin_amdgcn_readlane(min(b0, b1), wl);
    const float cx = px[wbi], cy = py[wbi], cz = pz[wbi];   // uniform index: outside the lane branch
    if (lane == wl) {
      const int j = wbi / PPT;
      const int k = (int)bitrev_bits((unsigned)(gl * R + j), L) + T * (wbi - j * PPT);
      sd[par][w] = wmax;
      sc[par][w] = make_float4(cx, cy, cz, __int_as_float(k));
    }
    lds_barrier();
    // every wave: the lowest wave holding the largest maximum (strict '>' in wave order)
    int gd = sd[par][0], gw = 0;
#pragma unroll
    for (int q = 1; q < NW; ++q) {
      const int d = sd[par][q];
      if (d > gd) {
        gd = d;
        gw = q;
      }
    }
    int k;
    if (gd != kNeverBits) {
      const float4 c = sc[par][gw];
      ox = c.x, oy = c.y, oz = c.z;
      k = __float_as_int(c.w);
    } else {  // no valid point at all: the reference's dists_i[0] == 0
      ox = x0, oy = y0, oz = z0;
      k = 0;
    }
    if (threadIdx.x == 0) out[jr] = k;
  }
}

struct __align__(16) FpsSlot {
  float d, x, y, z;
  int k;
  unsigned r;
  int pad0, pad1;
};

// Large clouds (N > 16384): same reduction, points streamed from global memory
// (L2-resident after the first round) and running distances in the workspace.
__global__ __launch_bounds__(kFpsThreads) void fps_stream_kernel(const float *__restrict__ xyz, int N, int M, int T,
                                                                  int L, float *__restrict__ temp,
                                                                  int *__restrict__ idx,
                                                                  const int *__restrict__ counts) {
  const int b = blockIdx.x;
  const int nb = counts ? min(max(counts[b], 0), N) : N;
  const float *p = xyz + (size_t)b * N * 3;
  float *tm = temp + (size_t)b * N;
  int *out = idx + (size_t)b * M;
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int nw = blockDim.x >> 6;
  for (int k = t; k < nb; k += blockDim.x) {
    const float mag = sqd3(p[3 * k], p[3 * k + 1], p[3 * k + 2]);
    tm[k] = ((double)mag <= 1e-3) ? -1.f : 1e10f;
  }
  __shared__ FpsSlot slots[2][kFpsThreads / 64];
  const float x0 = p[0], y0 = p[1], z0 = p[2];
  float ox = x0, oy = y0, oz = z0;
  if (t == 0 && M > 0) out[0] = 0;
  __syncthreads();
  int par = 0;
  for (int j = 1; j < M; ++j) {
    float best = -1.f;
    int bk = 0;
    if (t < T) {
      for (int k = t; k < nb; k += T) {
        const float d = sqd3(p[3 * k] - ox, p[3 * k + 1] - oy, p[3 * k + 2] - oz);
        const float d2 = fminf(d, tm[k]);
        tm[k] = d2;
        if (d2 > best) {
          best = d2;
          bk = k;
        }
      }
    }
    const float wmax = __int_as_float(wave_max_i32(fbits(best)));
    const uint64_t tied = __ballot(best == wmax);
    const int wl = min_bitrev_lane(tied);
    const int wk = __builtin_amdgcn_readlane(bk, wl);
    if (lane == 0) {
      const int tw = w * 64 + wl;
      FpsSlot s;
      s.d = wmax;
      s.x = p[3 * wk];
      s.y = p[3 * wk + 1];
      s.z = p[3 * wk + 2];
      s.k = wk;
      s.r = bitrev_bits((unsigned)tw, L);
      slots[par][w] = s;
    }
    __syncthreads();
    float gd = slots[par][0].d;
    int gw = 0;
    unsigned gr = slots[par][0].r;
    for (int ww = 1; ww < nw; ++ww) {
      const float d = slots[par][ww].d;
      const unsigned r = slots[par][ww].r;
      if (d > gd || (d == gd && r < gr)) {
        gd = d;
        gr = r;
        gw = ww;
      }
    }
    int k;
    if (gd > -1.f) {
      k = slots[par][gw].k;
      ox = slots[par][gw].x;
      oy = slots[par][gw].y;
      oz = slots[par][gw].z;
    } else {
      k = 0;
      ox = x0;
      oy = y0;
      oz = z0;
    }
    if (t == 0) out[j] = k;
    par ^= 1;
  }
}

// The output elements are cut into 8 contiguous ranges, one per XCD (workgroups
// are dispatched to the XCDs round-robin: block % 8): each XCD then gathers from
// the point rows of its own batches only, and a 64-B line of `points` is fetched
// into one XCD's L2 instead of up to eight (PMC: 5.5x the algorithmic bytes with
// the plain grid-stride order).  gridDim.x is a multiple of 8.
__device__ __forceinline__ void xcd_span(size_t total, size_t &e, size_t &end, size_t &stride) {
  const unsigned xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, per = gridDim.x >> 3;
  const size_t chunk = (total + 7) / 8;
  const size_t begin = xcd * chunk;
  end = begin + chunk < total ? begin + chunk : total;
  e = begin + (size_t)slot * blockDim.x + threadIdx.x;
  stride = (size_t)per * blockDim.x;
}

__global__ void gather_kernel(const float *__restrict__ points, const int *__restrict__ idx, int C, int N, int M,
                              size_t total, float *__restrict__ out) {
  size_t e, end, stride;
  xcd_span(total, e, end, stride);
  for (; e < end; e += stride) {
    const int m = (int)(e % M);
    const size_t bc = e / M;
    const size_t b = bc / C;
    const int a = idx[b * M + m];
    out[e] = ((unsigned)a < (unsigned)N) ? points[bc * N + a] : 0.f;
  }
}

__global__ void gather_grad_kernel(const float *__restrict__ grad_out, const int *__restrict__ idx, int C, int N,
                                   int M, size_t total, float *__restrict__ grad_points) {
  size_t e, end, stride;
  xcd_span(total, e, end, stride);
  for (; e < end; e += stride) {
    const int m = (int)(e % M);
    const size_t bc = e / M;
    const size_t b = bc / C;
    const int a = idx[b * M + m];
    if ((unsigned)a < (unsigned)N) atomicAdd(grad_points + bc * N + a, grad_out[e]);
  }
}

int opt_n_threads(int work_size) {  // cuda_utils.h:15-19
  const int pow_2 = (int)(std::log((double)work_size) / std::log(2.0));
  int t = 1 << pow_2;
  return t > 512 ? 512 : (t < 1 ? 1 : t);
}

bool fps_v1() {  // PCOPS_FPS_V1=1: leader-wave slot reduction (A/B runs)
  static const bool v = [] {
    const char *e = getenv("PCOPS_FPS_V1");
    return e && e[0] == '1';
  }();
  return v;
}

int fps_split_ppt() {  // PCOPS_FPS_SPLIT_PPT: points per reference thread above which 1024 threads are used
  static const int v = [] {
    const char *e = getenv("PCOPS_FPS_SPLIT_PPT");
    return e ? atoi(e) : 16;
  }();
  return v;
}

// One FPS workgroup per CU.  An FPS launch is B workgroups (one per cloud), each a serial chain of M rounds
// bound by its own CU's VALU and LDS latency; the workgroup dispatcher may place two of them -- of one launch,
// or of the FPS launches the models run side by side on other streams (the loss's gt chain, the next step's
// crop, the partial cloud) -- on the same CU, where they split that CU's issue slots and each runs up to 2x
// slower.  Every FPS launch therefore reserves kFpsExclLds bytes of dynamic LDS it never touches: two FPS
// workgroups (> 80 KB each) cannot share a CU's 160 KB.  PCOPS_FPS_EXCL=0 turns the reservation off (A/B).
constexpr int kFpsExclLds = 96 * 1024;
template <auto K>
unsigned fps_excl_lds() {
  static const unsigned bytes = [] {
    const char *e = getenv("PCOPS_FPS_EXCL");
    if (e && e[0] == '0') return 0u;
    return hipFuncSetAttribute((const void *)K, hipFuncAttributeMaxDynamicSharedMemorySize, kFpsExclLds) ==
                   hipSuccess
               ? (unsigned)kFpsExclLds
               : 0u;
  }();
  return bytes;
}

unsigned grid_for(size_t total, int block) {
  size_t g = (total + block - 1) / block;
  if (g > 8192) g = 8192;
  return (unsigned)(g < 1 ? 1 : g);
}

unsigned grid_xcd(size_t total, int block) {  // a multiple of 8 workgroups (xcd_span)
  return (grid_for(total, block) + 7u) & ~7u;
}

}  // namespace

extern "C" unsigned long long pcops_fps_workspace_bytes(int B, int N) {
  if (B <= 0 || N <= 0) return 0;
  return (N > kFpsThreads * kFpsMaxPPT) ? (unsigned long long)B * N * sizeof(float) : 0ull;
}

namespace {
int fps_impl(const float *xyz, const int *counts, int B, int N, int M, int *idx, void *workspace,
             unsigned long long workspace_bytes, pcops_stream_t stream) {
  if (B < 0 || M < 0 || (M > 0 && N <= 0)) return PCOPS_ERR_INVALID;
  if (B == 0 || M == 0) return PCOPS_OK;
  if (!xyz || !idx) return PCOPS_ERR_INVALID;
  const int T = opt_n_threads(N);
  int L = 0;
  while ((1 << L) < T) ++L;
  const int nthreads = T < 64 ? 64 : T;
  const int ppt = (N + T - 1) / T;  // points per reference thread
  hipStream_t s = (hipStream_t)stream;
  {
    // small clouds: one wave per cloud when its lanes hold <= PCOPS_FPS_WAVE slots (0: never)
    static const int wave_cap = [] {
      const char *e = getenv("PCOPS_FPS_WAVE");
      return e ? atoi(e) : 8;
    }();
    const int R = T >= 64 ? T / 64 : 1;
    const int ppl = R * ppt;
#define FPS_WAVE_CASE(P)                                                                                     \
  if (ppl <= P) {                                                                                            \
    hipLaunchKernelGGL((fps_wave_kernel<P>), dim3(B), dim3(64), fps_excl_lds<fps_wave_kernel<P>>(), s, xyz, N, \
                       M, T, L, R, ppt, idx, counts);                                                        \
    PC_CHECK_LAUNCH();                                                                                       \
    return PCOPS_OK;                                                                                         \
  }
    if (ppl <= wave_cap) {
      FPS_WAVE_CASE(8)
      FPS_WAVE_CASE(16)
      FPS_WAVE_CASE(24)
      FPS_WAVE_CASE(32)   // larger register arrays spill (PPL 40: 496 B of scratch per lane)
    }
#undef FPS_WAVE_CASE
  }
  {
    // 4-wave blocks for 512-thread clouds of 5-8 points per reference thread (PCOPS_FPS_MW=0: off, A/B)
    static const bool mw = [] {
      const char *e = getenv("PCOPS_FPS_MW");
      return !(e && e[0] == '0');
    }();
    if (mw && T == 512 && ppt >= 5 && ppt <= 8) {
      constexpr int NW = 4;
      const int R = T / (64 * NW);
      const int ppl = R * ppt;
#define FPS_MW_CASE(P)                                                                                        \
  if (ppl <= P) {                                                                                             \
    const unsigned lds_ = fps_excl_lds<fps_mw_kernel<P, NW>>();                                              \
    hipLaunchKernelGGL((fps_mw_kernel<P, NW>), dim3(B), dim3(64 * NW), lds_, s, xyz, N, M, T, L, R, ppt, idx, \
                       counts);                                                                               \
    PC_CHECK_LAUNCH();                                                                                        \
    return PCOPS_OK;                                                                                          \
  }
      FPS_MW_CASE(10)
      FPS_MW_CASE(12)
      FPS_MW_CASE(14)
      FPS_MW_CASE(16)
#undef FPS_MW_CASE
    }
  }
  if (ppt <= kFpsMaxPPT) {
    // clouds with > 16 points per reference thread use 2 hardware threads per
    // reference thread (1024 threads, 4 waves / SIMD).  Up to 16 the 8-wave
    // block wins: 32x8192->2048 2.41 -> 2.06 ms (fewer slots, one barrier).
    const int split = (ppt > fps_split_ppt() && T == 512) ? 2 : 1;
    const int per = (ppt + split - 1) / split;
    const int nwt = nthreads / 64;
#define FPS_LAUNCH(P, AR, CN)                                                                             \
  do {                                                                                                    \
    const unsigned lds_ = fps_excl_lds<fps_reg_kernel<P, AR, CN>>();                                      \
    hipLaunchKernelGGL((fps_reg_kernel<P, AR, CN>), dim3(B), dim3(nthreads * split), lds_, s, xyz, N, M, T, L, \
                       nwt, split, idx, counts);                                                          \
  } while (0)
#define FPS_CASE(P)                                                                                       \
  if (per <= P) {                                                                                         \
    const bool ar = !(fps_v1() || nthreads * split > 512);                                                \
    if (counts) {                                                                                         \
      if (ar) FPS_LAUNCH(P, true, true); else FPS_LAUNCH(P, false, true);                                 \
    } else {                                                                                              \
      if (ar) FPS_LAUNCH(P, true, false); else FPS_LAUNCH(P, false, false);                               \
    }                                                                                                     \
    PC_CHECK_LAUNCH();                                                                                    \
    return PCOPS_OK;                                                                                      \
  }
    // exact slot counts for the model's clouds (2304 -> 5 per thread, 6144 -> 12): the
    // sweep runs every slot of the template, so a power-of-two P wasted up to 3 / 4 of 8 / 16
    FPS_CASE(1)
    FPS_CASE(2)
    FPS_CASE(4)
    FPS_CASE(6)
    FPS_CASE(8)
    FPS_CASE(12)
    FPS_CASE(16)
    FPS_CASE(32)
#undef FPS_CASE
#undef FPS_LAUNCH
  }
  if (!workspace || workspace_bytes < pcops_fps_workspace_bytes(B, N)) return PCOPS_ERR_WORKSPACE;
  hipLaunchKernelGGL(fps_stream_kernel, dim3(B), dim3(nthreads), fps_excl_lds<fps_stream_kernel>(), s, xyz, N, M, T,
                     L, (float *)workspace, idx, counts);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
}  // namespace

extern "C" int pcops_furthest_point_sampling(const float *xyz, int B, int N, int M, int *idx, void *workspace,
                                             unsigned long long workspace_bytes, pcops_stream_t stream) {
  return fps_impl(xyz, nullptr, B, N, M, idx, workspace, workspace_bytes, stream);
}

extern "C" int pcops_furthest_point_sampling_counts(const float *xyz, const int *counts, int B, int N, int M, int *idx,
                                                    void *workspace, unsigned long long workspace_bytes,
                                                    pcops_stream_t stream) {
  if (!counts && B > 0 && M > 0) return PCOPS_ERR_INVALID;
  return fps_impl(xyz, counts, B, N, M, idx, workspace, workspace_bytes, stream);
}

extern "C" int pcops_gather_points(const float *points, const int *idx, int B, int C, int N, int M, float *out,
                                   pcops_stream_t stream) {
  if (B < 0 || C < 0 || N < 0 || M < 0) return PCOPS_ERR_INVALID;
  const size_t total = (size_t)B * C * M;
  if (total == 0) return PCOPS_OK;
  if (!points || !idx || !out) return PCOPS_ERR_INVALID;
  hipLaunchKernelGGL(gather_kernel, dim3(grid_xcd(total, 256)), dim3(256), 0, (hipStream_t)stream, points, idx, C,
                     N, M, total, out);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_gather_points_grad(const float *grad_out, const int *idx, int B, int C, int N, int M,
                                        float *grad_points, pcops_stream_t stream) {
  if (B < 0 || C < 0 || N < 0 || M < 0) return PCOPS_ERR_INVALID;
  if ((size_t)B * C * N == 0) return PCOPS_OK;
  if (!grad_points) return PCOPS_ERR_INVALID;
  if (pc_memset_async(grad_points, 0, sizeof(float) * (size_t)B * C * N, (hipStream_t)stream) != hipSuccess)
    return PCOPS_ERR_LAUNCH;
  const size_t total = (size_t)B * C * M;
  if (total == 0) return PCOPS_OK;
  if (!grad_out || !idx) return PCOPS_ERR_INVALID;
  hipLaunchKernelGGL(gather_grad_kernel, dim3(grid_xcd(total, 256)), dim3(256), 0, (hipStream_t)stream, grad_out, idx,
                     C, N, M, total, grad_points);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
