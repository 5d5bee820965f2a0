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
#include <cmath>

#include "common.h"

namespace {

constexpr int kFpsThreads = 512;  // == TOTAL_THREADS (cuda_utils.h:13) for N >= 512
constexpr int kFpsMaxPPT = 32;    // 512 * 32 = 16384 points resident in VGPRs

// uniform-index register pick: `i` is wave-uniform (readfirstlane), so the
// switch lowers to scalar branches and the arrays stay in VGPRs.
template <int PPT>
__device__ __forceinline__ void pick3(const float (&ax)[PPT], const float (&ay)[PPT], const float (&az)[PPT], int i,
                                      float &x, float &y, float &z) {
  x = ax[0];
  y = ay[0];
  z = az[0];
#pragma unroll
  for (int c = 1; c < PPT; ++c) {
    if (i == c) {
      x = ax[c];
      y = ay[c];
      z = az[c];
    }
  }
}

struct __align__(16) FpsSlot {
  float d, x, y, z;
  int k;
  unsigned r;
  int pad0, pad1;
};

template <int PPT>
__global__ __launch_bounds__(kFpsThreads) void fps_reg_kernel(const float *__restrict__ xyz, int N, int M, int T,
                                                               int L, int *__restrict__ idx) {
  const int b = blockIdx.x;
  const float *p = xyz + (size_t)b * N * 3;
  int *out = idx + (size_t)b * M;
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int nw = blockDim.x >> 6;

  float px[PPT], py[PPT], pz[PPT], tmp[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int k = t + T * i;
    if (t < T && k < N) {
      px[i] = p[3 * k];
      py[i] = p[3 * k + 1];
      pz[i] = p[3 * k + 2];
      const float mag = sqd3(px[i], py[i], pz[i]);
      tmp[i] = ((double)mag <= 1e-3) ? -1.f : 1e10f;  // -1: never selected (sampling_gpu.cu:100-101)
    } else {
      px[i] = py[i] = pz[i] = 0.f;
      tmp[i] = -1.f;
    }
  }
  __shared__ FpsSlot slots[2][kFpsThreads / 64];

  const float x0 = p[0], y0 = p[1], z0 = p[2];
  float ox = x0, oy = y0, oz = z0;
  if (t == 0 && M > 0) out[0] = 0;
  int par = 0;
  for (int j = 1; j < M; ++j) {
    float best = -1.f;
    int bi = 0;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const float d = sqd3(px[i] - ox, py[i] - oy, pz[i] - oz);
      const float d2 = fminf(d, tmp[i]);
      tmp[i] = d2;
      if (d2 > best) {
        best = d2;
        bi = i;
      }
    }
    const float wmax = wave_max_f32(best);
    const uint64_t tied = __ballot(best == wmax);
    const int wl = min_bitrev_lane(tied);
    const int wbi = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(bi, wl));
    float cx, cy, cz;
    pick3<PPT>(px, py, pz, wbi, cx, cy, cz);
    cx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cx), wl));
    cy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cy), wl));
    cz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cz), wl));
    if (lane == 0) {
      const int tw = w * 64 + wl;
      FpsSlot s;
      s.d = wmax;
      s.x = cx;
      s.y = cy;
      s.z = cz;
      s.k = tw + T * wbi;
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
    } else {  // no valid point at all: the reference's dists_i[0] == 0
      k = 0;
      ox = x0;
      oy = y0;
      oz = z0;
    }
    if (t == 0) out[j] = k;
    par ^= 1;
  }
}

// Large clouds (N > 16384): same reduction, points streamed from global memory
// (L2-resident after the first round) and running distances in the workspace.
__global__ __launch_bounds__(kFpsThreads) void fps_stream_kernel(const float *__restrict__ xyz, int N, int M, int T,
                                                                  int L, float *__restrict__ temp,
                                                                  int *__restrict__ idx) {
  const int b = blockIdx.x;
  const float *p = xyz + (size_t)b * N * 3;
  float *tm = temp + (size_t)b * N;
  int *out = idx + (size_t)b * M;
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int nw = blockDim.x >> 6;
  for (int k = t; k < N; k += blockDim.x) {
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
      for (int k = t; k < N; k += T) {
        const float d = sqd3(p[3 * k] - ox, p[3 * k + 1] - oy, p[3 * k + 2] - oz);
        const float d2 = fminf(d, tm[k]);
        tm[k] = d2;
        if (d2 > best) {
          best = d2;
          bk = k;
        }
      }
    }
    const float wmax = wave_max_f32(best);
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

__global__ void gather_kernel(const float *__restrict__ points, const int *__restrict__ idx, int C, int N, int M,
                              size_t total, float *__restrict__ out) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int m = (int)(e % M);
    const size_t bc = e / M;
    const size_t b = bc / C;
    const int a = idx[b * M + m];
    out[e] = ((unsigned)a < (unsigned)N) ? points[bc * N + a] : 0.f;
  }
}

__global__ void gather_grad_kernel(const float *__restrict__ grad_out, const int *__restrict__ idx, int C, int N,
                                   int M, size_t total, float *__restrict__ grad_points) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
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

unsigned grid_for(size_t total, int block) {
  size_t g = (total + block - 1) / block;
  if (g > 8192) g = 8192;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" unsigned long long pcops_fps_workspace_bytes(int B, int N) {
  if (B <= 0 || N <= 0) return 0;
  return (N > kFpsThreads * kFpsMaxPPT) ? (unsigned long long)B * N * sizeof(float) : 0ull;
}

extern "C" int pcops_furthest_point_sampling(const float *xyz, int B, int N, int M, int *idx, void *workspace,
                                             unsigned long long workspace_bytes, pcops_stream_t stream) {
  if (B < 0 || M < 0 || (M > 0 && N <= 0)) return PCOPS_ERR_INVALID;
  if (B == 0 || M == 0) return PCOPS_OK;
  if (!xyz || !idx) return PCOPS_ERR_INVALID;
  const int T = opt_n_threads(N);
  int L = 0;
  while ((1 << L) < T) ++L;
  const int nthreads = T < 64 ? 64 : T;
  const int ppt = (N + T - 1) / T;
  hipStream_t s = (hipStream_t)stream;
  if (ppt <= kFpsMaxPPT) {
#define FPS_CASE(P)                                                                              \
  if (ppt <= P) {                                                                                \
    hipLaunchKernelGGL(fps_reg_kernel<P>, dim3(B), dim3(nthreads), 0, s, xyz, N, M, T, L, idx); \
    PC_CHECK_LAUNCH();                                                                           \
    return PCOPS_OK;                                                                             \
  }
    FPS_CASE(1)
    FPS_CASE(2)
    FPS_CASE(4)
    FPS_CASE(8)
    FPS_CASE(16)
    FPS_CASE(32)
#undef FPS_CASE
  }
  if (!workspace || workspace_bytes < pcops_fps_workspace_bytes(B, N)) return PCOPS_ERR_WORKSPACE;
  hipLaunchKernelGGL(fps_stream_kernel, dim3(B), dim3(nthreads), 0, s, xyz, N, M, T, L, (float *)workspace, idx);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_gather_points(const float *points, const int *idx, int B, int C, int N, int M, float *out,
                                   pcops_stream_t stream) {
  if (B < 0 || C < 0 || N < 0 || M < 0) return PCOPS_ERR_INVALID;
  const size_t total = (size_t)B * C * M;
  if (total == 0) return PCOPS_OK;
  if (!points || !idx || !out) return PCOPS_ERR_INVALID;
  hipLaunchKernelGGL(gather_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, points, idx, C,
                     N, M, total, out);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_gather_points_grad(const float *grad_out, const int *idx, int B, int C, int N, int M,
                                        float *grad_points, pcops_stream_t stream) {
  if (B < 0 || C < 0 || N < 0 || M < 0) return PCOPS_ERR_INVALID;
  if ((size_t)B * C * N == 0) return PCOPS_OK;
  if (!grad_points) return PCOPS_ERR_INVALID;
  if (hipMemsetAsync(grad_points, 0, sizeof(float) * (size_t)B * C * N, (hipStream_t)stream) != hipSuccess)
    return PCOPS_ERR_LAUNCH;
  const size_t total = (size_t)B * C * M;
  if (total == 0) return PCOPS_OK;
  if (!grad_out || !idx) return PCOPS_ERR_INVALID;
  hipLaunchKernelGGL(gather_grad_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, grad_out, idx,
                     C, N, M, total, grad_points);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
