// Multi-view depth projection (gfx950).
//
// PCViews.get_img (models/model_utils.py:1196-1234 -> points2depth :1080-1115 ->
// distribute :1004-1077 with size_x = size_y = 1): one lane per (point, view)
// transforms, projects and splats (w, z*w) into two image planes with float
// atomics; a second pass forms the harmonic-mean depth.  The projection
// arithmetic follows the reference's fp32 op order exactly (point @ R as an
// fma chain = torch's sgemm order, then /, *, +, ceil), so every point lands
// on the reference's pixel.
//
// PCViews_Real.get_img (models_PointSea/mv_utils_zs.py:97-195): one workgroup
// per image transforms its cloud (two 3x3 products + translation), reduces the
// bounding box in LDS, quantises and scatter-maxes the depth into the 8x224x224
// voxel grid (atomicMax on the bit pattern of the positive depth).  Grid2Image
// then runs tile-wise: 7x7 max-pool and 3x3 Gaussian per depth slice from an
// LDS halo tile, max over depth, and a per-image normalisation pass.
#include "common.h"

namespace {

__device__ __forceinline__ void xform(const float *R, float x, float y, float z, float &ox, float &oy, float &oz) {
  // out_c = sum_k p_k R[k][c] as torch's sgemm fma chain: fma(p2, R2c, fma(p1, R1c, p0*R0c))
  ox = __builtin_fmaf(z, R[6], __builtin_fmaf(y, R[3], x * R[0]));
  oy = __builtin_fmaf(z, R[7], __builtin_fmaf(y, R[4], x * R[1]));
  oz = __builtin_fmaf(z, R[8], __builtin_fmaf(y, R[5], x * R[2]));
}

__global__ void depth_splat_kernel(const float *__restrict__ points, const float *__restrict__ rot,
                                   const float *__restrict__ trans, int B, int N, int V, int H, int W,
                                   float *__restrict__ vsum, float *__restrict__ wsum) {
  const size_t tot = (size_t)B * V * N;
  const float eps = 1e-12f;
  const float aspect = (float)((double)W / (double)H);
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e % N);
    const size_t bv = e / N;
    const int v = (int)(bv % V);
    const size_t b = bv / V;
    const float *p = points + (b * N + i) * 3;
    const float *R = rot + v * 9;
    float qx, qy, qz;
    xform(R, p[0], p[1], p[2], qx, qy, qz);
    qx = qx - trans[v * 3];
    qy = qy - trans[v * 3 + 1];
    qz = qz - trans[v * 3 + 2];
    const float cx = (qx / (qz + eps)) * aspect;
    const float cy = qy / (qz + eps);
    const float xx = ((cx + 1.f) * (float)H) / 2.f;
    const float yy = ((cy + 1.f) * (float)W) / 2.f;
    const float ex = ceilf(xx + -0.5f);
    const float ey = ceilf(yy + -0.5f);
    if (!(ex >= 0.f && ex <= (float)(H - 1) && ey >= 0.f && ey <= (float)(W - 1) && qz >= 0.f)) continue;
    const float w = 1.f / (qz + eps);
    const size_t pix = bv * (size_t)H * W + (size_t)ex * W + (size_t)ey;
    atomicAdd(wsum + pix, w);
    atomicAdd(vsum + pix, qz * w);
  }
}

__global__ void depth_resolve_kernel(float *__restrict__ img, const float *__restrict__ wsum, size_t tot) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const float ws = wsum[e];
    img[e] = img[e] / (ws == 0.f ? ws + 1.f : ws);
  }
}

// ---------------------------------------------------------------- PointSea
constexpr int kGridThreads = 256;

__global__ __launch_bounds__(kGridThreads) void points2grid_kernel(const float *__restrict__ points,
                                                                   const float *__restrict__ rot,
                                                                   const float *__restrict__ rot2,
                                                                   const float *__restrict__ trans, int N, int V,
                                                                   int R, int D, float *__restrict__ grid) {
  const int bv = blockIdx.x;
  const int v = bv % V, b = bv / V;
  const float *p = points + (size_t)b * N * 3;
  const float *R1 = rot + v * 9, *R2 = rot2 + v * 9, *t = trans + v * 3;
  __shared__ float red[6][kGridThreads / 64];
  float mx[3] = {-INFINITY, -INFINITY, -INFINITY}, mn[3] = {INFINITY, INFINITY, INFINITY};
  for (int i = threadIdx.x; i < N; i += kGridThreads) {
    float ax, ay, az, qx, qy, qz;
    xform(R1, p[3 * i], p[3 * i + 1], p[3 * i + 2], ax, ay, az);
    xform(R2, ax, ay, az, qx, qy, qz);
    const float q[3] = {qx - t[0], qy - t[1], qz - t[2]};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      mx[c] = fmaxf(mx[c], q[c]);
      mn[c] = fminf(mn[c], q[c]);
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float a = mx[c], m2 = mn[c];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      a = fmaxf(a, __shfl_xor(a, off, 64));
      m2 = fminf(m2, __shfl_xor(m2, off, 64));
    }
    if (lane == 0) {
      red[c][w] = a;
      red[3 + c][w] = m2;
    }
  }
  __syncthreads();
  float cent[3], rng = -INFINITY;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float a = red[c][0], m2 = red[3 + c][0];
    for (int ww = 1; ww < kGridThreads / 64; ++ww) {
      a = fmaxf(a, red[c][ww]);
      m2 = fminf(m2, red[3 + c][ww]);
    }
    cent[c] = (a + m2) / 2.f;
    rng = fmaxf(rng, a - m2);
  }
  const float obj_ratio = 0.8f, depth_bias = 0.2f;
  const size_t G = (size_t)D * R * R;
  float *g = grid + (size_t)bv * G;
  for (int i = threadIdx.x; i < N; i += kGridThreads) {
    float ax, ay, az, qx, qy, qz;
    xform(R1, p[3 * i], p[3 * i + 1], p[3 * i + 2], ax, ay, az);
    xform(R2, ax, ay, az, qx, qy, qz);
    float q0 = ((qx - t[0]) - cent[0]) / rng * 2.f;
    float q1 = ((qy - t[1]) - cent[1]) / rng * 2.f;
    const float q2 = ((qz - t[2]) - cent[2]) / rng * 2.f;
    q0 = q0 * obj_ratio;
    q1 = q1 * obj_ratio;
    float x = (q0 + 1.f) / 2.f * (float)R;
    float y = (q1 + 1.f) / 2.f * (float)R;
    float z = ((q2 + 1.f) / 2.f + depth_bias) / (float)1.2 * (float)(D - 2);
    x = ceilf(x);
    y = ceilf(y);
    const float zi = ceilf(z);
    x = fminf(fmaxf(x, 1.f), (float)(R - 2));
    y = fminf(fmaxf(y, 1.f), (float)(R - 2));
    z = fminf(fmaxf(z, 1.f), (float)(D - 2));
    const float coord = zi * (float)R * (float)R + y * (float)R + x;
    const long ci = (long)coord;
    if (ci < 0 || (size_t)ci >= G) continue;
    const long zz = ci / ((long)R * R), rem = ci % ((long)R * R), yy = rem / R, xx = rem % R;
    // stored permuted [z][x][y] (mv_utils_zs.py:131); z >= 1 > 0 so int order == float order
    atomicMax(reinterpret_cast<int *>(g + ((size_t)zz * R + xx) * R + yy), __float_as_int(z));
  }
}

constexpr int kTile = 32;
constexpr int kHalo = 4;  // 3 (max-pool) + 1 (conv)
constexpr int kIn = kTile + 2 * kHalo;

// per tile: max over depth of conv3x3(maxpool7x7(grid_z)); per-image max via atomicMax
__global__ __launch_bounds__(256) void grid2image_kernel(const float *__restrict__ grid,
                                                         const float *__restrict__ kern, int D, int R,
                                                         float *__restrict__ img, int *__restrict__ img_max) {
  const int bv = blockIdx.z;
  const int x0 = blockIdx.y * kTile, y0 = blockIdx.x * kTile;
  __shared__ float sin_[kIn][kIn + 1];
  __shared__ float srow[kIn][kTile + 2 + 1];  // row-direction 7-max, cols y0-1 .. y0+kTile
  __shared__ float spool[kTile + 2][kTile + 2 + 1];
  float kw[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) kw[i] = kern[i];
  float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  const size_t RR = (size_t)R * R;
  for (int z = 0; z < D; ++z) {
    const float *g = grid + ((size_t)bv * D + z) * RR;
    for (int e = threadIdx.x; e < kIn * kIn; e += 256) {
      const int ix = e / kIn, iy = e % kIn;
      const int gx = x0 - kHalo + ix, gy = y0 - kHalo + iy;
      sin_[ix][iy] = (gx >= 0 && gx < R && gy >= 0 && gy < R) ? g[(size_t)gx * R + gy] : -INFINITY;
    }
    __syncthreads();
    // max over dy in [-3,3] for columns y0-1 .. y0+kTile (kTile+2 columns)
    for (int e = threadIdx.x; e < kIn * (kTile + 2); e += 256) {
      const int ix = e / (kTile + 2), jy = e % (kTile + 2);
      float m = -INFINITY;
#pragma unroll
      for (int d = 0; d < 7; ++d) m = fmaxf(m, sin_[ix][jy + d]);
      srow[ix][jy] = m;
    }
    __syncthreads();
    // max over dx -> pooled values for pixels x0-1..x0+kTile, y0-1..y0+kTile;
    // outside the image the conv's zero padding applies
    for (int e = threadIdx.x; e < (kTile + 2) * (kTile + 2); e += 256) {
      const int jx = e / (kTile + 2), jy = e % (kTile + 2);
      float m = -INFINITY;
#pragma unroll
      for (int d = 0; d < 7; ++d) m = fmaxf(m, srow[jx + d][jy]);
      const int gx = x0 - 1 + jx, gy = y0 - 1 + jy;
      spool[jx][jy] = (gx >= 0 && gx < R && gy >= 0 && gy < R) ? m : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = threadIdx.x + 256 * k;
      const int ox = e / kTile, oy = e % kTile;
      float s = 0.f;
#pragma unroll
      for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) s += kw[dx * 3 + dy] * spool[ox + dx][oy + dy];
      best[k] = fmaxf(best[k], s);
    }
    __syncthreads();
  }
  float lmax = -INFINITY;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int gx = x0 + e / kTile, gy = y0 + e % kTile;
    if (gx < R && gy < R) {
      img[(size_t)bv * RR + (size_t)gx * R + gy] = best[k];
      lmax = fmaxf(lmax, best[k]);
    }
  }
  lmax = wave_max_f32(lmax);
  // values are >= 0 (grid >= 0, Gaussian weights > 0): int order == float order
  if ((threadIdx.x & 63) == 0) atomicMax(img_max + bv, __float_as_int(lmax));
}

__global__ void image_normalize_kernel(const float *__restrict__ img, const int *__restrict__ img_max, int BV,
                                       size_t RR, float *__restrict__ out) {
  const size_t tot = (size_t)BV * RR;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const size_t bv = e / RR, k = e % RR;
    const float v = 1.f - img[e] / __int_as_float(img_max[bv]);
    out[(bv * 3 + 0) * RR + k] = v;
    out[(bv * 3 + 1) * RR + k] = v;
    out[(bv * 3 + 2) * RR + k] = v;
  }
}

unsigned grid_for(size_t total, int block) {
  size_t g = (total + block - 1) / block;
  if (g > 8192) g = 8192;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" unsigned long long pcops_points2depth_workspace_bytes(int B, int V, int H, int W) {
  if (B <= 0 || V <= 0 || H <= 0 || W <= 0) return 0;
  return (unsigned long long)B * V * H * W * sizeof(float);
}

extern "C" int pcops_points2depth(const float *points, const float *rot, const float *trans, int B, int N, int V,
                                  int H, int W, float *img, void *workspace, unsigned long long workspace_bytes,
                                  pcops_stream_t stream) {
  if (B < 0 || N < 0 || V < 0 || H <= 0 || W <= 0) return PCOPS_ERR_INVALID;
  const size_t tot = (size_t)B * V * H * W;
  if (tot == 0) return PCOPS_OK;
  if (!rot || !trans || !img || (N > 0 && !points)) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_points2depth_workspace_bytes(B, V, H, W)) return PCOPS_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  float *wsum = (float *)workspace;
  if (pc_memset_async(img, 0, tot * sizeof(float), s) || pc_memset_async(wsum, 0, tot * sizeof(float), s))
    return PCOPS_ERR_LAUNCH;
  const size_t np = (size_t)B * V * N;
  if (np) {
    hipLaunchKernelGGL(depth_splat_kernel, dim3(grid_for(np, 256)), dim3(256), 0, s, points, rot, trans, B, N, V, H, W,
                       img, wsum);
    PC_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(depth_resolve_kernel, dim3(grid_for(tot, 256)), dim3(256), 0, s, img, wsum, tot);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_points2grid(const float *points, const float *rot, const float *rot2, const float *trans, int B,
                                 int N, int V, int R, int D, float *grid, pcops_stream_t stream) {
  if (B < 0 || N <= 0 || V < 0 || R < 3 || D < 3) return PCOPS_ERR_INVALID;
  if (B == 0 || V == 0) return PCOPS_OK;
  if (!points || !rot || !rot2 || !trans || !grid) return PCOPS_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  if (pc_memset_async(grid, 0, sizeof(float) * (size_t)B * V * D * R * R, s)) return PCOPS_ERR_LAUNCH;
  hipLaunchKernelGGL(points2grid_kernel, dim3(B * V), dim3(kGridThreads), 0, s, points, rot, rot2, trans, N, V, R, D,
                     grid);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" unsigned long long pcops_grid2image_workspace_bytes(int BV, int D, int R) {
  (void)D;
  if (BV <= 0 || R <= 0) return 0;
  return (((unsigned long long)BV * R * R * sizeof(float) + 63) / 64) * 64 + (unsigned long long)BV * sizeof(int);
}

extern "C" int pcops_grid2image(const float *grid, const float *kern, int BV, int D, int R, float *img,
                                void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream) {
  if (BV < 0 || D <= 0 || R <= 0) return PCOPS_ERR_INVALID;
  if (BV == 0) return PCOPS_OK;
  if (!grid || !kern || !img) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_grid2image_workspace_bytes(BV, D, R)) return PCOPS_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const size_t RR = (size_t)R * R;
  float *raw = (float *)workspace;
  int *mx = (int *)((char *)workspace + ((BV * RR * sizeof(float) + 63) / 64) * 64);
  if (pc_memset_async(mx, 0xff, sizeof(int) * BV, s)) return PCOPS_ERR_LAUNCH;  // -NaN bits < any valid max
  // 0xffffffff as int is -1: below every non-negative float bit pattern
  const dim3 gdim((R + kTile - 1) / kTile, (R + kTile - 1) / kTile, BV);
  hipLaunchKernelGGL(grid2image_kernel, gdim, dim3(256), 0, s, grid, kern, D, R, raw, mx);
  PC_CHECK_LAUNCH();
  hipLaunchKernelGGL(image_normalize_kernel, dim3(grid_for(BV * RR, 256)), dim3(256), 0, s, raw, mx, BV, RR, img);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
