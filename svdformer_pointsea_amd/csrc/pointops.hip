// group_points, ball_query, three_nn, three_interpolate (+ grads) for gfx950
// (pointnet2_ops group_points_gpu.cu, ball_query_gpu.cu, interpolate_gpu.cu).
//
// The reference launches these with grid = B only (group_points_gpu.cu:34,
// interpolate_gpu.cu:107) -- B workgroups for the whole chip.  Here every
// element-wise op is a flat grid-stride launch over all outputs (coalesced
// writes, >= 256 workgroups), and the search ops map one query per lane.
#include "common.h"

namespace {

unsigned grid_for(size_t total, int block) {
  size_t g = (total + block - 1) / block;
  if (g > 8192) g = 8192;
  return (unsigned)(g < 1 ? 1 : g);
}

// out[b,c,s,k] = points[b,c,idx[b,s,k]]
__global__ void group_kernel(const float *__restrict__ points, const int *__restrict__ idx, int C, int N, int SK,
                             size_t total, float *__restrict__ out) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int sk = (int)(e % SK);
    const size_t bc = e / SK;
    const size_t b = bc / C;
    const int a = idx[b * SK + sk];
    out[e] = ((unsigned)a < (unsigned)N) ? points[bc * N + a] : 0.f;
  }
}

__global__ void group_grad_kernel(const float *__restrict__ grad_out, const int *__restrict__ idx, int C, int N,
                                  int SK, size_t total, float *__restrict__ grad_points) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int sk = (int)(e % SK);
    const size_t bc = e / SK;
    const size_t b = bc / C;
    const int a = idx[b * SK + sk];
    if ((unsigned)a < (unsigned)N) atomicAdd(grad_points + bc * N + a, grad_out[e]);
  }
}

// ball_query_gpu.cu:9-44: first nsample hits in index order; the first hit
// fills the whole row; no hit leaves zeros.
__global__ void ball_query_kernel(const float *__restrict__ new_xyz, const float *__restrict__ xyz, int B, int N,
                                  int M, float r2, int nsample, int *__restrict__ idx) {
  const size_t tot = (size_t)B * M;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const size_t b = e / M;
    const float *p = xyz + b * N * 3;
    const float nx = new_xyz[e * 3], ny = new_xyz[e * 3 + 1], nz = new_xyz[e * 3 + 2];
    int *o = idx + e * nsample;
    int cnt = 0;
    for (int k = 0; k < N && cnt < nsample; ++k) {
      const float d2 = sqd3(nx - p[3 * k], ny - p[3 * k + 1], nz - p[3 * k + 2]);
      if (d2 < r2) {
        if (cnt == 0)
          for (int l = 0; l < nsample; ++l) o[l] = k;
        o[cnt] = k;
        ++cnt;
      }
    }
    if (cnt == 0)
      for (int l = 0; l < nsample; ++l) o[l] = 0;
  }
}

// interpolate_gpu.cu:9-59 (compare chain in double as the reference; d is fp32)
__global__ void three_nn_kernel(const float *__restrict__ unknown, const float *__restrict__ known, int B, int N,
                                int M, float *__restrict__ dist2, int *__restrict__ idx) {
  extern __shared__ __attribute__((aligned(16))) float4 kt[];
  constexpr int TN = 1024;
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const float *u = unknown + ((size_t)b * N + (j < N ? j : N - 1)) * 3;
  const float *kn = known + (size_t)b * M * 3;
  const float ux = u[0], uy = u[1], uz = u[2];
  float best1 = INFINITY, best2 = INFINITY, best3 = INFINITY;
  int bi1 = 0, bi2 = 0, bi3 = 0;
  for (int t0 = 0; t0 < M; t0 += TN) {
    const int cnt = min(TN, M - t0);
    for (int e = threadIdx.x; e < cnt; e += blockDim.x)
      kt[e] = make_float4(kn[(size_t)(t0 + e) * 3], kn[(size_t)(t0 + e) * 3 + 1], kn[(size_t)(t0 + e) * 3 + 2], 0.f);
    __syncthreads();
    for (int e = 0; e < cnt; ++e) {
      const float4 c = kt[e];
      const float d = sqd3(ux - c.x, uy - c.y, uz - c.z);
      const int k = t0 + e;
      if (d < best1) {
        best3 = best2; bi3 = bi2;
        best2 = best1; bi2 = bi1;
        best1 = d; bi1 = k;
      } else if (d < best2) {
        best3 = best2; bi3 = bi2;
        best2 = d; bi2 = k;
      } else if (d < best3) {
        best3 = d; bi3 = k;
      }
    }
    __syncthreads();
  }
  if (j < N) {
    // the reference initialises its bests to 1e40 (double) -> float inf
    float *dd = dist2 + ((size_t)b * N + j) * 3;
    int *ii = idx + ((size_t)b * N + j) * 3;
    dd[0] = best1; dd[1] = best2; dd[2] = best3;
    ii[0] = bi1; ii[1] = bi2; ii[2] = bi3;
  }
}

// interpolate_gpu.cu:72-101: out = p1*w1 + p2*w2 + p3*w3 (contraction order)
__global__ void three_interp_kernel(const float *__restrict__ points, const int *__restrict__ idx,
                                    const float *__restrict__ weight, int C, int M, int N, size_t total,
                                    float *__restrict__ out) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int j = (int)(e % N);
    const size_t bc = e / N;
    const size_t b = bc / C;
    const int *ii = idx + (b * N + j) * 3;
    const float *ww = weight + (b * N + j) * 3;
    const float *pp = points + bc * M;
    const int i0 = ii[0], i1 = ii[1], i2 = ii[2];
    const float p0 = (unsigned)i0 < (unsigned)M ? pp[i0] : 0.f;
    const float p1 = (unsigned)i1 < (unsigned)M ? pp[i1] : 0.f;
    const float p2 = (unsigned)i2 < (unsigned)M ? pp[i2] : 0.f;
    out[e] = __builtin_fmaf(p2, ww[2], __builtin_fmaf(p0, ww[0], p1 * ww[1]));
  }
}

__global__ void three_interp_grad_kernel(const float *__restrict__ grad_out, const int *__restrict__ idx,
                                         const float *__restrict__ weight, int C, int N, int M, size_t total,
                                         float *__restrict__ grad_points) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int j = (int)(e % N);
    const size_t bc = e / N;
    const size_t b = bc / C;
    const int *ii = idx + (b * N + j) * 3;
    const float *ww = weight + (b * N + j) * 3;
    const float g = grad_out[e];
    float *gp = grad_points + bc * M;
#pragma unroll
    for (int r = 0; r < 3; ++r)
      if ((unsigned)ii[r] < (unsigned)M) atomicAdd(gp + ii[r], g * ww[r]);
  }
}

// ---- fused SA-module grouping (models/model_utils.py:323-356 sample_and_group_knn
// + the channels_last copy the first 1x1 conv reads).  One thread per output
// element of the (B, S, K, Ct) row-major tensor, Ct = 3 + C: channel c < 3 is
// xyz[idx] - new_xyz (the reference's grouped_xyz -= new_xyz, fp32), channel
// c >= 3 is points_t[b, idx, c - 3] (token-major points: a row copies C
// contiguous floats).  Replaces two grouping launches, the repeat + subtract,
// the channel concat and the NCHW -> channels_last copy (and, under autocast,
// the bf16 cast: out_dtype 1 rounds once, as the cast would).
__global__ void sa_group_kernel(const float *__restrict__ xyz, const float *__restrict__ new_xyz,
                                const float *__restrict__ pts, const int *__restrict__ idx, int N, int S, int K,
                                int C, int Ct, size_t total, void *__restrict__ out, int out_dt) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % Ct);
    const size_t row = e / Ct;            // (b, s, k)
    const size_t bs = row / K;            // (b, s)
    const size_t b = bs / S;
    const int a = idx[row];
    const bool ok = (unsigned)a < (unsigned)N;
    float v;
    if (c < 3)
      v = (ok ? xyz[(b * N + a) * 3 + c] : 0.f) - new_xyz[bs * 3 + c];
    else
      v = ok ? pts[(b * N + a) * C + (c - 3)] : 0.f;
    if (out_dt == 1)
      reinterpret_cast<__bf16 *>(out)[e] = (__bf16)v;
    else
      reinterpret_cast<float *>(out)[e] = v;
  }
}

// grad_points_t[b, idx, c] += grad_out[b, s, k, 3 + c] (the group_points_grad
// scatter-add, token-major; consecutive threads add to consecutive channels of
// one row, so the atomics coalesce)
__global__ void sa_group_grad_kernel(const void *__restrict__ g, int g_dt, const int *__restrict__ idx, int N, int S,
                                     int K, int C, int Ct, size_t total, float *__restrict__ gpts) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    const size_t row = e / C;
    const size_t b = row / ((size_t)S * K);
    const int a = idx[row];
    if ((unsigned)a >= (unsigned)N) continue;
    const size_t src = row * Ct + 3 + c;
    const float v = g_dt == 1 ? (float)reinterpret_cast<const __bf16 *>(g)[src] : reinterpret_cast<const float *>(g)[src];
    atomicAdd(gpts + (b * N + a) * C + c, v);
  }
}

}  // namespace

extern "C" int pcops_sa_group(const float *xyz, const float *new_xyz, const float *points_t, const int *idx, int B,
                              int N, int S, int K, int C, void *out, int out_dtype, pcops_stream_t stream) {
  if (B < 0 || N < 0 || S < 0 || K < 0 || C < 0 || (out_dtype != 0 && out_dtype != 1)) return PCOPS_ERR_INVALID;
  const int Ct = 3 + C;
  const size_t total = (size_t)B * S * K * Ct;
  if (total == 0) return PCOPS_OK;
  if (!xyz || !new_xyz || !idx || !out || (C > 0 && !points_t)) return PCOPS_ERR_INVALID;
  hipLaunchKernelGGL(sa_group_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, xyz, new_xyz,
                     points_t, idx, N, S, K, C, Ct, total, out, out_dtype);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_sa_group_grad(const void *grad_out, int grad_dtype, const int *idx, int B, int N, int S, int K,
                                   int C, float *grad_points_t, pcops_stream_t stream) {
  if (B < 0 || N < 0 || S < 0 || K < 0 || C < 0 || (grad_dtype != 0 && grad_dtype != 1)) return PCOPS_ERR_INVALID;
  if ((size_t)B * N * C == 0) return PCOPS_OK;
  if (!grad_points_t) return PCOPS_ERR_INVALID;
  if (pc_memset_async(grad_points_t, 0, sizeof(float) * (size_t)B * N * C, (hipStream_t)stream) != hipSuccess)
    return PCOPS_ERR_LAUNCH;
  const size_t total = (size_t)B * S * K * C;
  if (total == 0) return PCOPS_OK;
  if (!grad_out || !idx) return PCOPS_ERR_INVALID;
  hipLaunchKernelGGL(sa_group_grad_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, grad_out,
                     grad_dtype, idx, N, S, K, C, 3 + C, total, grad_points_t);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_group_points(const float *points, const int *idx, int B, int C, int N, int S, int K, float *out,
                                  pcops_stream_t stream) {
  if (B < 0 || C < 0 || N < 0 || S < 0 || K < 0) return PCOPS_ERR_INVALID;
  const size_t total = (size_t)B * C * S * K;
  if (total == 0) return PCOPS_OK;
  if (!points || !idx || !out) return PCOPS_ERR_INVALID;
  hipLaunchKernelGGL(group_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, points, idx, C, N,
                     S * K, total, out);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_group_points_grad(const float *grad_out, const int *idx, int B, int C, int N, int S, int K,
                                       float *grad_points, pcops_stream_t stream) {
  if (B < 0 || C < 0 || N < 0 || S < 0 || K < 0) return PCOPS_ERR_INVALID;
  if ((size_t)B * C * N == 0) return PCOPS_OK;
  if (!grad_points) return PCOPS_ERR_INVALID;
  if (pc_memset_async(grad_points, 0, sizeof(float) * (size_t)B * C * N, (hipStream_t)stream) != hipSuccess)
    return PCOPS_ERR_LAUNCH;
  const size_t total = (size_t)B * C * S * K;
  if (total == 0) return PCOPS_OK;
  if (!grad_out || !idx) return PCOPS_ERR_INVALID;
  hipLaunchKernelGGL(group_grad_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, grad_out, idx,
                     C, N, S * K, total, grad_points);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_ball_query(const float *new_xyz, const float *xyz, int B, int N, int M, float radius, int nsample,
                                int *idx, pcops_stream_t stream) {
  if (B < 0 || N < 0 || M < 0 || nsample < 0) return PCOPS_ERR_INVALID;
  const size_t tot = (size_t)B * M;
  if (tot == 0 || nsample == 0) return PCOPS_OK;
  if (!new_xyz || !xyz || !idx) return PCOPS_ERR_INVALID;
  hipLaunchKernelGGL(ball_query_kernel, dim3(grid_for(tot, 64)), dim3(64), 0, (hipStream_t)stream, new_xyz, xyz, B, N,
                     M, radius * radius, nsample, idx);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_three_nn(const float *unknown, const float *known, int B, int N, int M, float *dist2, int *idx,
                              pcops_stream_t stream) {
  if (B < 0 || N < 0 || M < 0) return PCOPS_ERR_INVALID;
  if (B == 0 || N == 0) return PCOPS_OK;
  if (!unknown || !known || !dist2 || !idx) return PCOPS_ERR_INVALID;
  const dim3 grid((N + 255) / 256, B);
  hipLaunchKernelGGL(three_nn_kernel, grid, dim3(256), sizeof(float4) * 1024, (hipStream_t)stream, unknown, known, B,
                     N, M, dist2, idx);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_three_interpolate(const float *points, const int *idx, const float *weight, int B, int C, int M,
                                       int N, float *out, pcops_stream_t stream) {
  if (B < 0 || C < 0 || M < 0 || N < 0) return PCOPS_ERR_INVALID;
  const size_t total = (size_t)B * C * N;
  if (total == 0) return PCOPS_OK;
  if (!points || !idx || !weight || !out) return PCOPS_ERR_INVALID;
  hipLaunchKernelGGL(three_interp_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, points, idx,
                     weight, C, M, N, total, out);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_three_interpolate_grad(const float *grad_out, const int *idx, const float *weight, int B, int C,
                                            int N, int M, float *grad_points, pcops_stream_t stream) {
  if (B < 0 || C < 0 || M < 0 || N < 0) return PCOPS_ERR_INVALID;
  if ((size_t)B * C * M == 0) return PCOPS_OK;
  if (!grad_points) return PCOPS_ERR_INVALID;
  if (pc_memset_async(grad_points, 0, sizeof(float) * (size_t)B * C * M, (hipStream_t)stream) != hipSuccess)
    return PCOPS_ERR_LAUNCH;
  const size_t total = (size_t)B * C * N;
  if (total == 0) return PCOPS_OK;
  if (!grad_out || !idx || !weight) return PCOPS_ERR_INVALID;
  hipLaunchKernelGGL(three_interp_grad_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream,
                     grad_out, idx, weight, C, N, M, total, grad_points);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

// ---------------------------------------------------------------- max over neighbours
// torch.max(x, dim=K)[0] of the SA modules / EdgeConv (models/model_utils.py:354,
// 862-864) on the channels_last memory of the (B, C, S, K) conv output, i.e. a
// contiguous (rows = B*S, K, C) tensor: out[r][c] = max_k x[r][k][c] and the
// first maximising k (NaN counts as the maximum, as torch's max), 8 channels
// per thread with 16-byte accesses.  torch's own reduction over the middle
// dim with indices ran ~10x below HBM bandwidth.  Backward: grad_x[r][k][c] =
// (k == arg[r][c]) ? g[r][c] : 0 in one pass (torch: zeros + scatter).
namespace {
template <int DT>
struct Vec8;
template <>
struct Vec8<0> {
  static __device__ __forceinline__ void ld(float (&v)[8], const void *p, long long e) {
    const float4 a = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(p) + e);
    const float4 b = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(p) + e + 4);
    v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
  }
  static __device__ __forceinline__ void st(void *p, long long e, const float (&v)[8]) {
    *reinterpret_cast<float4 *>(reinterpret_cast<float *>(p) + e) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4 *>(reinterpret_cast<float *>(p) + e + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};
template <>
struct Vec8<1> {
  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ void ld(float (&v)[8], const void *p, long long e) {
    const b8 a = *reinterpret_cast<const b8 *>(reinterpret_cast<const __bf16 *>(p) + e);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (float)a[k];
  }
  static __device__ __forceinline__ void st(void *p, long long e, const float (&v)[8]) {
    b8 a;
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = (__bf16)v[k];  // exact: every value is a bf16 input or 0
    *reinterpret_cast<b8 *>(reinterpret_cast<__bf16 *>(p) + e) = a;
  }
};

template <int DT>
__global__ __launch_bounds__(256) void max_k_kernel(const void *__restrict__ x, long long rows, int K, int C,
                                                    void *__restrict__ out, unsigned char *__restrict__ arg) {
  const int c8 = C / 8;
  const long long total = rows * c8;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long r = e / c8;
    const int c = (int)(e - r * c8) * 8;
    float best[8], v[8];
    unsigned char bk[8];
    Vec8<DT>::ld(best, x, (r * K) * C + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) bk[j] = 0;
    for (int k = 1; k < K; ++k) {
      Vec8<DT>::ld(v, x, (r * K + k) * C + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool take = v[j] > best[j] || (v[j] != v[j] && best[j] == best[j]);  // first max; NaN wins
        best[j] = take ? v[j] : best[j];
        bk[j] = take ? (unsigned char)k : bk[j];
      }
    }
    Vec8<DT>::st(out, r * C + c, best);
    unsigned long long packed = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) packed |= (unsigned long long)bk[j] << (8 * j);
    *reinterpret_cast<unsigned long long *>(arg + r * C + c) = packed;
  }
}

template <int DT>
__global__ __launch_bounds__(256) void max_k_grad_kernel(const void *__restrict__ g, const unsigned char *__restrict__ arg,
                                                         long long rows, int K, int C, void *__restrict__ gx) {
  const int c8 = C / 8;
  const long long total = rows * c8;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long r = e / c8;
    const int c = (int)(e - r * c8) * 8;
    float gv[8], o[8];
    Vec8<DT>::ld(gv, g, r * C + c);
    const unsigned long long packed = *reinterpret_cast<const unsigned long long *>(arg + r * C + c);
    for (int k = 0; k < K; ++k) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = ((packed >> (8 * j)) & 0xFF) == (unsigned long long)k ? gv[j] : 0.f;
      Vec8<DT>::st(gx, (r * K + k) * C + c, o);
    }
  }
}

// ---- EdgeConv edge features (models/model_utils.py:847-881; PointSea's copy
// models_PointSea/model_utils.py:551-585): group_local's kNN gather (:812-845),
// `central - neigh`, torch.cat((edge, central), 1) and the channels_last copy the
// first 1x1 conv reads, as ONE pass after the kNN:
//   out[b,n,k,c]     = x[b,n,c] - x[b,idx[b,n,k],c]    (c < C)
//   out[b,n,k,C + c] = x[b,n,c]
// x (B,N,C) token-major fp32 -- the kNN's own operand -- so a neighbour is one
// contiguous row (the reference's channel-major gather reads C strided floats
// per neighbour).  Differences in fp32, rounded once to out's dtype (the
// autocast cast the first conv would apply).  V = 8: C % 8 == 0, a thread
// writes 8 channels (16-B bf16 / 32-B fp32 stores); V = 1 otherwise (C = 3).
template <int V, int DT>
__global__ __launch_bounds__(256) void edge_group_kernel(const float *__restrict__ x, const int *__restrict__ idx,
                                                         int N, int K, int C, long long rows,
                                                         void *__restrict__ out) {
  const int cv = C / V, per = 2 * cv;  // vector chunks per output row
  const long long total = rows * per;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long row = e / per;           // (b, n, k)
    const int j = (int)(e - row * per);
    const long long bn = row / K;            // (b, n)
    const long long b = bn / N;
    const bool edge = j < cv;
    const int c = (edge ? j : j - cv) * V;
    const float *xi = x + bn * C + c;
    float v[V];
#pragma unroll
    for (int t = 0; t < V; ++t) v[t] = xi[t];
    if (edge) {
      const int a = idx[row];
      if ((unsigned)a < (unsigned)N) {
        const float *xj = x + (b * N + a) * C + c;
#pragma unroll
        for (int t = 0; t < V; ++t) v[t] -= xj[t];
      }
    }
    const long long o = row * 2 * C + (edge ? c : C + c);
    if constexpr (V == 8) {
      Vec8<DT>::st(out, o, v);
    } else if constexpr (DT == 1) {
      reinterpret_cast<__bf16 *>(out)[o] = (__bf16)v[0];
    } else {
      reinterpret_cast<float *>(out)[o] = v[0];
    }
  }
}

// Backward, own term: dx[b,n,c] = sum_k (g[b,n,k,c] + g[b,n,k,C+c])  (the gradient
// through `central`, used by the subtraction and the concat; k ascending, fp32),
// stored -- no zero fill, no atomics.
template <int V, int DT>
__global__ __launch_bounds__(256) void edge_group_grad_own_kernel(const void *__restrict__ g, int K, int C,
                                                                  long long pts, float *__restrict__ dx) {
  const int cv = C / V;
  const long long total = pts * cv;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long bn = e / cv;
    const int c = (int)(e - bn * cv) * V;
    float acc[V], a[V], b2[V];
#pragma unroll
    for (int t = 0; t < V; ++t) acc[t] = 0.f;
    for (int k = 0; k < K; ++k) {
      const long long r = (bn * K + k) * 2 * C;
      if constexpr (V == 8) {
        Vec8<DT>::ld(a, g, r + c);
        Vec8<DT>::ld(b2, g, r + C + c);
      } else {
        a[0] = DT == 1 ? (float)reinterpret_cast<const __bf16 *>(g)[r + c] : reinterpret_cast<const float *>(g)[r + c];
        b2[0] = DT == 1 ? (float)reinterpret_cast<const __bf16 *>(g)[r + C + c]
                        : reinterpret_cast<const float *>(g)[r + C + c];
      }
#pragma unroll
      for (int t = 0; t < V; ++t) acc[t] += a[t] + b2[t];
    }
    if constexpr (V == 8) {
      Vec8<0>::st(dx, bn * C + c, acc);
    } else {
      dx[bn * C + c] = acc[0];
    }
  }
}

// Backward, neighbour term: dx[b,idx[b,n,k],c] -= g[b,n,k,c] (the index_points /
// group_points_grad scatter, token-major).  Launched with V = 1: consecutive lanes
// add to consecutive channels of one destination row, so a wave-instruction's
// atomics form one contiguous 256-B run (the full global-atomic rate); 8 channels
// per lane made every instruction touch 8 rows 32 B apart (a fraction of it).
template <int V, int DT>
__global__ __launch_bounds__(256) void edge_group_grad_scatter_kernel(const void *__restrict__ g,
                                                                      const int *__restrict__ idx, int N, int K, int C,
                                                                      long long rows, float *__restrict__ dx) {
  const int cv = C / V;
  const long long total = rows * cv;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long row = e / cv;
    const int c = (int)(e - row * cv) * V;
    const int a = idx[row];
    if ((unsigned)a >= (unsigned)N) continue;
    const long long b = row / ((long long)N * K);
    float v[V];
    if constexpr (V == 8) {
      Vec8<DT>::ld(v, g, row * 2 * C + c);
    } else {
      v[0] = DT == 1 ? (float)reinterpret_cast<const __bf16 *>(g)[row * 2 * C + c]
                     : reinterpret_cast<const float *>(g)[row * 2 * C + c];
    }
    float *d = dx + (b * N + a) * C + c;
#pragma unroll
    for (int t = 0; t < V; ++t) atomicAdd(d + t, -v[t]);
  }
}

unsigned grid_for_ll(long long total) {
  long long g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  return (unsigned)(g < 1 ? 1 : g);
}
}  // namespace

extern "C" int pcops_max_k(const void *x, int dtype, long long rows, int K, int C, void *out, unsigned char *arg,
                           pcops_stream_t stream) {
  if (rows < 0 || K <= 0 || K > 255 || C <= 0 || (dtype != 0 && dtype != 1)) return PCOPS_ERR_INVALID;
  if (C % 8) return PCOPS_ERR_UNSUPPORTED;
  if (rows == 0) return PCOPS_OK;
  if (!x || !out || !arg) return PCOPS_ERR_INVALID;
  const long long total = rows * (C / 8);
  if (dtype == 0)
    hipLaunchKernelGGL(max_k_kernel<0>, dim3(grid_for_ll(total)), dim3(256), 0, (hipStream_t)stream, x, rows, K, C,
                       out, arg);
  else
    hipLaunchKernelGGL(max_k_kernel<1>, dim3(grid_for_ll(total)), dim3(256), 0, (hipStream_t)stream, x, rows, K, C,
                       out, arg);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_max_k_grad(const void *grad_out, int dtype, const unsigned char *arg, long long rows, int K, int C,
                                void *grad_x, pcops_stream_t stream) {
  if (rows < 0 || K <= 0 || K > 255 || C <= 0 || (dtype != 0 && dtype != 1)) return PCOPS_ERR_INVALID;
  if (C % 8) return PCOPS_ERR_UNSUPPORTED;
  if (rows == 0) return PCOPS_OK;
  if (!grad_out || !arg || !grad_x) return PCOPS_ERR_INVALID;
  const long long total = rows * (C / 8);
  if (dtype == 0)
    hipLaunchKernelGGL(max_k_grad_kernel<0>, dim3(grid_for_ll(total)), dim3(256), 0, (hipStream_t)stream, grad_out,
                       arg, rows, K, C, grad_x);
  else
    hipLaunchKernelGGL(max_k_grad_kernel<1>, dim3(grid_for_ll(total)), dim3(256), 0, (hipStream_t)stream, grad_out,
                       arg, rows, K, C, grad_x);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

namespace {
template <int V>
void edge_group_go(const float *x, const int *idx, int N, int K, int C, long long rows, void *out, int dt,
                   hipStream_t s) {
  const unsigned grid = grid_for_ll(rows * 2 * (C / V));
  if (dt == 1)
    hipLaunchKernelGGL((edge_group_kernel<V, 1>), dim3(grid), dim3(256), 0, s, x, idx, N, K, C, rows, out);
  else
    hipLaunchKernelGGL((edge_group_kernel<V, 0>), dim3(grid), dim3(256), 0, s, x, idx, N, K, C, rows, out);
}

template <int V, int DT>
void edge_group_grad_go(const void *g, const int *idx, int B, int N, int K, int C, float *dx, hipStream_t s) {
  const long long pts = (long long)B * N, rows = pts * K;
  hipLaunchKernelGGL((edge_group_grad_own_kernel<V, DT>), dim3(grid_for_ll(pts * (C / V))), dim3(256), 0, s, g, K, C,
                     pts, dx);
  hipLaunchKernelGGL((edge_group_grad_scatter_kernel<1, DT>), dim3(grid_for_ll(rows * C)), dim3(256), 0, s, g, idx, N,
                     K, C, rows, dx);
}
}  // namespace

extern "C" int pcops_edge_group(const float *x, const int *idx, int B, int N, int K, int C, void *out, int out_dtype,
                                pcops_stream_t stream) {
  if (B < 0 || N < 0 || K < 0 || C < 0 || (out_dtype != 0 && out_dtype != 1)) return PCOPS_ERR_INVALID;
  const long long rows = (long long)B * N * K;
  if (rows == 0 || C == 0) return PCOPS_OK;
  if (!x || !idx || !out) return PCOPS_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  if (C % 8 == 0 && ((uintptr_t)x % 16 == 0) && ((uintptr_t)out % 16 == 0))
    edge_group_go<8>(x, idx, N, K, C, rows, out, out_dtype, s);
  else
    edge_group_go<1>(x, idx, N, K, C, rows, out, out_dtype, s);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_edge_group_grad(const void *grad_out, int grad_dtype, const int *idx, int B, int N, int K, int C,
                                     float *grad_x, pcops_stream_t stream) {
  if (B < 0 || N < 0 || K < 0 || C < 0 || (grad_dtype != 0 && grad_dtype != 1)) return PCOPS_ERR_INVALID;
  if ((long long)B * N * C == 0) return PCOPS_OK;
  if (!grad_x) return PCOPS_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  if (K == 0) {
    if (pc_memset_async(grad_x, 0, sizeof(float) * (size_t)B * N * C, s) != hipSuccess) return PCOPS_ERR_LAUNCH;
    return PCOPS_OK;
  }
  if (!grad_out || !idx) return PCOPS_ERR_INVALID;
  const bool vec = C % 8 == 0 && (uintptr_t)grad_out % 16 == 0 && (uintptr_t)grad_x % 16 == 0;
  if (vec && grad_dtype == 1)
    edge_group_grad_go<8, 1>(grad_out, idx, B, N, K, C, grad_x, s);
  else if (vec)
    edge_group_grad_go<8, 0>(grad_out, idx, B, N, K, C, grad_x, s);
  else if (grad_dtype == 1)
    edge_group_grad_go<1, 1>(grad_out, idx, B, N, K, C, grad_x, s);
  else
    edge_group_grad_go<1, 0>(grad_out, idx, B, N, K, C, grad_x, s);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

// ---- 3x3 / stride 2 / pad 1 max pool on channels_last (N, H, W, C) bf16 / fp32 activations
// (torchvision's resnet stem pool, models_PointSea/PointSea.py:37-61 ResEncoder).  Forward: torch's
// NHWC kernel's rule -- the window scanned row by row, strict '>' keeps the first maximum, a NaN
// always takes the slot (so the last NaN wins) -- and the winner's window offset (0..8) as uint8.
// Backward: per input element the gradients of the windows whose winner it is, summed in fp32 over
// (ph, pw) ascending as torch's max_pool_backward_nhwc does, stored once (no atomics, no zero fill).
namespace {
template <typename T>
__global__ void maxpool3s2_fwd_kernel(const T *__restrict__ x, int N, int H, int W, int C, int OH, int OW,
                                      T *__restrict__ y, unsigned char *__restrict__ arg) {
  const long long total = (long long)N * OH * OW * C;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    long long r = e / C;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int n = (int)(r / OH);
    float best = -INFINITY;
    int bi = -1, first = -1;
    for (int i = 0; i < 3; ++i) {
      const int ih = 2 * oh - 1 + i;
      if (ih < 0 || ih >= H) continue;
      for (int j = 0; j < 3; ++j) {
        const int iw = 2 * ow - 1 + j;
        if (iw < 0 || iw >= W) continue;
        if (first < 0) first = 3 * i + j;
        const float v = (float)x[(((long long)n * H + ih) * W + iw) * C + c];
        if (v > best || v != v) {
          best = v;
          bi = 3 * i + j;
        }
      }
    }
    // a window of -inf only: torch keeps its initial index 0 (image element (0, 0)); here the
    // window's first element (unreachable after the ReLU this pool follows)
    if (bi < 0) bi = first;
    y[e] = (T)best;
    arg[e] = (unsigned char)bi;
  }
}

template <typename T>
__global__ void maxpool3s2_bwd_kernel(const T *__restrict__ gy, const unsigned char *__restrict__ arg, int N, int H,
                                      int W, int C, int OH, int OW, T *__restrict__ gx) {
  const long long total = (long long)N * H * W * C;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    long long r = e / C;
    const int iw = (int)(r % W);
    r /= W;
    const int ih = (int)(r % H);
    const int n = (int)(r / H);
    // windows (ph, pw) with 2 ph - 1 <= ih <= 2 ph + 1 (torch's p_start / p_end for k 3, s 2, p 1)
    const int ph0 = ih + 1 < 3 ? 0 : (ih + 1 - 3) / 2 + 1, ph1 = min((ih + 1) / 2 + 1, OH);
    const int pw0 = iw + 1 < 3 ? 0 : (iw + 1 - 3) / 2 + 1, pw1 = min((iw + 1) / 2 + 1, OW);
    float acc = 0.f;
    for (int ph = ph0; ph < ph1; ++ph)
      for (int pw = pw0; pw < pw1; ++pw) {
        const long long o = (((long long)n * OH + ph) * OW + pw) * C + c;
        const int a = arg[o];
        if (2 * ph - 1 + a / 3 == ih && 2 * pw - 1 + a % 3 == iw) acc += (float)gy[o];
      }
    gx[e] = (T)acc;
  }
}

// 8 channels per thread (C % 8 == 0): 16-byte (bf16) / 32-byte (fp32) window loads and stores, the
// same per-channel rule as the scalar kernels above
template <typename T>
struct PoolVec8 {
  T v[8];
};

template <typename T>
__global__ void maxpool3s2_fwd8_kernel(const T *__restrict__ x, int N, int H, int W, int C, int OH, int OW,
                                       T *__restrict__ y, unsigned char *__restrict__ arg) {
  const int C8 = C / 8;
  const long long total = (long long)N * OH * OW * C8;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C8) * 8;
    long long r = e / C8;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int n = (int)(r / OH);
    float best[8];
    int bi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) best[k] = -INFINITY, bi[k] = -1;
    int first = -1;
    for (int i = 0; i < 3; ++i) {
      const int ih = 2 * oh - 1 + i;
      if (ih < 0 || ih >= H) continue;
      for (int j = 0; j < 3; ++j) {
        const int iw = 2 * ow - 1 + j;
        if (iw < 0 || iw >= W) continue;
        if (first < 0) first = 3 * i + j;
        const PoolVec8<T> t = *reinterpret_cast<const PoolVec8<T> *>(x + (((long long)n * H + ih) * W + iw) * C + c);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float v = (float)t.v[k];
          if (v > best[k] || v != v) {
            best[k] = v;
            bi[k] = 3 * i + j;
          }
        }
      }
    }
    PoolVec8<T> o;
    unsigned long long a = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o.v[k] = (T)best[k];
      a |= (unsigned long long)(unsigned char)(bi[k] < 0 ? first : bi[k]) << (8 * k);
    }
    const long long oe = (((long long)n * OH + oh) * OW + ow) * C + c;
    *reinterpret_cast<PoolVec8<T> *>(y + oe) = o;
    *reinterpret_cast<unsigned long long *>(arg + oe) = a;
  }
}

template <typename T>
__global__ void maxpool3s2_bwd8_kernel(const T *__restrict__ gy, const unsigned char *__restrict__ arg, int N, int H,
                                       int W, int C, int OH, int OW, T *__restrict__ gx) {
  const int C8 = C / 8;
  const long long total = (long long)N * H * W * C8;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C8) * 8;
    long long r = e / C8;
    const int iw = (int)(r % W);
    r /= W;
    const int ih = (int)(r % H);
    const int n = (int)(r / H);
    const int ph0 = ih + 1 < 3 ? 0 : (ih + 1 - 3) / 2 + 1, ph1 = min((ih + 1) / 2 + 1, OH);
    const int pw0 = iw + 1 < 3 ? 0 : (iw + 1 - 3) / 2 + 1, pw1 = min((iw + 1) / 2 + 1, OW);
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    for (int ph = ph0; ph < ph1; ++ph)
      for (int pw = pw0; pw < pw1; ++pw) {
        const long long o = (((long long)n * OH + ph) * OW + pw) * C + c;
        const int want = 3 * (ih - 2 * ph + 1) + (iw - 2 * pw + 1);   // this element's offset in window (ph, pw)
        const unsigned long long a = *reinterpret_cast<const unsigned long long *>(arg + o);
        const PoolVec8<T> g = *reinterpret_cast<const PoolVec8<T> *>(gy + o);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if ((int)((a >> (8 * k)) & 0xFF) == want) acc[k] += (float)g.v[k];
      }
    PoolVec8<T> out;
#pragma unroll
    for (int k = 0; k < 8; ++k) out.v[k] = (T)acc[k];
    *reinterpret_cast<PoolVec8<T> *>(gx + (((long long)n * H + ih) * W + iw) * C + c) = out;
  }
}

unsigned pool_grid(long long total) {
  long long g = (total + 255) / 256;
  return (unsigned)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
}
}  // namespace

extern "C" int pcops_maxpool3s2_fwd(const void *x, int dtype, int N, int H, int W, int C, void *y,
                                    unsigned char *argmax, pcops_stream_t stream) {
  if (N < 0 || H < 0 || W < 0 || C < 0 || (dtype != 0 && dtype != 1)) return PCOPS_ERR_INVALID;
  const int OH = (H + 1) / 2, OW = (W + 1) / 2;   // floor((H + 2 - 3) / 2) + 1
  const long long total = (long long)N * OH * OW * C;
  if (total == 0) return PCOPS_OK;
  if (!x || !y || !argmax) return PCOPS_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  if (C % 8 == 0 && ((uintptr_t)x | (uintptr_t)y) % 16 == 0 && (uintptr_t)argmax % 8 == 0) {
    const long long t8 = total / 8;
    if (dtype == 0)
      hipLaunchKernelGGL(maxpool3s2_fwd8_kernel<float>, dim3(pool_grid(t8)), dim3(256), 0, s, (const float *)x, N, H,
                         W, C, OH, OW, (float *)y, argmax);
    else
      hipLaunchKernelGGL(maxpool3s2_fwd8_kernel<__bf16>, dim3(pool_grid(t8)), dim3(256), 0, s, (const __bf16 *)x, N,
                         H, W, C, OH, OW, (__bf16 *)y, argmax);
    PC_CHECK_LAUNCH();
    return PCOPS_OK;
  }
  if (dtype == 0)
    hipLaunchKernelGGL(maxpool3s2_fwd_kernel<float>, dim3(pool_grid(total)), dim3(256), 0, s, (const float *)x, N, H,
                       W, C, OH, OW, (float *)y, argmax);
  else
    hipLaunchKernelGGL(maxpool3s2_fwd_kernel<__bf16>, dim3(pool_grid(total)), dim3(256), 0, s, (const __bf16 *)x, N,
                       H, W, C, OH, OW, (__bf16 *)y, argmax);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_maxpool3s2_bwd(const void *gy, const unsigned char *argmax, int dtype, int N, int H, int W, int C,
                                    void *gx, pcops_stream_t stream) {
  if (N < 0 || H < 0 || W < 0 || C < 0 || (dtype != 0 && dtype != 1)) return PCOPS_ERR_INVALID;
  const int OH = (H + 1) / 2, OW = (W + 1) / 2;
  const long long total = (long long)N * H * W * C;
  if (total == 0) return PCOPS_OK;
  if (!gy || !argmax || !gx) return PCOPS_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  if (C % 8 == 0 && ((uintptr_t)gy | (uintptr_t)gx) % 16 == 0 && (uintptr_t)argmax % 8 == 0) {
    const long long t8 = total / 8;
    if (dtype == 0)
      hipLaunchKernelGGL(maxpool3s2_bwd8_kernel<float>, dim3(pool_grid(t8)), dim3(256), 0, s, (const float *)gy,
                         argmax, N, H, W, C, OH, OW, (float *)gx);
    else
      hipLaunchKernelGGL(maxpool3s2_bwd8_kernel<__bf16>, dim3(pool_grid(t8)), dim3(256), 0, s, (const __bf16 *)gy,
                         argmax, N, H, W, C, OH, OW, (__bf16 *)gx);
    PC_CHECK_LAUNCH();
    return PCOPS_OK;
  }
  if (dtype == 0)
    hipLaunchKernelGGL(maxpool3s2_bwd_kernel<float>, dim3(pool_grid(total)), dim3(256), 0, s, (const float *)gy,
                       argmax, N, H, W, C, OH, OW, (float *)gx);
  else
    hipLaunchKernelGGL(maxpool3s2_bwd_kernel<__bf16>, dim3(pool_grid(total)), dim3(256), 0, s, (const __bf16 *)gy,
                       argmax, N, H, W, C, OH, OW, (__bf16 *)gx);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
