// BatchNorm over channels_last activations, fused with what follows it in the
// reference's image / edge encoders:
//   ResNet BasicBlock  relu(bn1(conv1(x))), relu(bn2(conv2(.)) + identity)   models/resnet.py:56-70
//   stem / downsample  relu(bn(conv(x))), bn(conv1x1(x))                      models/SVDFormer.py:139-146
//   EdgeConv           leaky_relu(bn(conv1x1(edge)), 0.2)                     models/model_utils.py:855-866
//   PointSea ResEncoder (torchvision resnet18 stem + layers)                  models_PointSea/PointSea.py:37-61
// The activation is a row-major (rows, C) matrix: the memory of an NCHW tensor
// in channels_last order (rows = N*H*W), C % 8 == 0, C <= 512.  One 16-B
// vector (8 channels) per lane, every pass reads / writes whole rows.
//
// Forward (training):  stats pass  -> per-chunk shifted sums (x - x[0][c]), (x - x[0][c])^2
//                      final       -> mean, 1/sqrt(var + eps) (double combine), running stats
//                                     (momentum, unbiased var), scale / shift per channel
//                      apply pass  -> y = act(x * scale + shift (+ res))
// Backward:            reduce pass -> per chunk sum g, sum g * (x - mean),  g = act'(dy, y)
//                      final       -> dgamma, dbeta, dx = a g + b x + c per channel
//                      apply pass  -> dx (and g itself: the residual branch's gradient)
// torch runs the same BasicBlock as MIOpen mean/variance + norm + clamp + add
// forward and threshold_backward + dscale/dbias + dx (+ autograd's adds)
// backward: 3 and 4-5 launches, each a full pass over the activation.
#include <atomic>
#include <cstdlib>

#include "common.h"

namespace {

struct V8 {
  float v[8];
};
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

template <int DT>
__device__ __forceinline__ void ld8(V8 &o, const void *p, long long e) {
  if constexpr (DT == 0) {
    const float4 a = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(p) + e);
    const float4 b = *reinterpret_cast<const float4 *>(reinterpret_cast<const float *>(p) + e + 4);
    o.v[0] = a.x, o.v[1] = a.y, o.v[2] = a.z, o.v[3] = a.w, o.v[4] = b.x, o.v[5] = b.y, o.v[6] = b.z, o.v[7] = b.w;
  } else {
    const bf16x8_t a = *reinterpret_cast<const bf16x8_t *>(reinterpret_cast<const __bf16 *>(p) + e);
#pragma unroll
    for (int k = 0; k < 8; ++k) o.v[k] = (float)a[k];
  }
}
template <int DT>
__device__ __forceinline__ void st8(void *p, long long e, const V8 &o) {
  if constexpr (DT == 0) {
    float *q = reinterpret_cast<float *>(p) + e;
    *reinterpret_cast<float4 *>(q) = make_float4(o.v[0], o.v[1], o.v[2], o.v[3]);
    *reinterpret_cast<float4 *>(q + 4) = make_float4(o.v[4], o.v[5], o.v[6], o.v[7]);
  } else {
    bf16x8_t a;
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = (__bf16)o.v[k];
    *reinterpret_cast<bf16x8_t *>(reinterpret_cast<__bf16 *>(p) + e) = a;
  }
}

// activation codes: 0 none, 1 ReLU, 2 LeakyReLU(slope)
template <int ACT>
__device__ __forceinline__ float act_fwd(float v, float slope) {
  if constexpr (ACT == 1) return v < 0.f ? 0.f : v;  // NaN propagates (torch's clamp_min)
  if constexpr (ACT == 2) return v > 0.f ? v : v * slope;
  return v;
}
// gradient through the activation from its OUTPUT y: relu -> threshold_backward
// (y <= 0 -> 0); leaky -> leaky_relu_backward (input > 0, and sign(y) == sign(input))
template <int ACT>
__device__ __forceinline__ float act_bwd(float dy, float y, float slope) {
  if constexpr (ACT == 1) return y <= 0.f ? 0.f : dy;
  if constexpr (ACT == 2) return y > 0.f ? dy : dy * slope;
  return dy;
}

// A/B builds override these with -D (csrc/Makefile EXTRA)
#ifndef PCOPS_BN_CHUNKS
#define PCOPS_BN_CHUNKS 256
#endif
#ifndef PCOPS_BN_WAVES
#define PCOPS_BN_WAVES 16
#endif
#ifndef PCOPS_BN_UNROLL
#define PCOPS_BN_UNROLL 4
#endif
constexpr int kBnMaxChunks = PCOPS_BN_CHUNKS;  // partial rows; one kBnWaves-wave block per chunk
constexpr int kBnWaves = PCOPS_BN_WAVES;
constexpr int kBnUnroll = PCOPS_BN_UNROLL;     // rows whose loads issue together per lane

int bn_v(int C) {  // vector columns per wave: largest power of two <= 64 dividing C / 8
  const int nv = C / 8;
  int V = 64;
  while (nv % V) V >>= 1;
  return V;
}

// chunks per launch: kBnMaxChunks, half that below 2^25 elements (the ResNet's layer3 / layer4
// activations: fewer partial rows for the final; profiles/r5_bn_variants.txt)
int bn_max_chunks(long long rows, int C) {
  return rows * C < (1ll << 25) ? kBnMaxChunks / 2 : kBnMaxChunks;
}

void bn_shape(long long rows, int C, int &chunks, long long &rpc) {
  const int strips = C / 8 / bn_v(C);
  const int maxc = bn_max_chunks(rows, C);
  long long want = (maxc + strips - 1) / strips;
  if (want > (rows + 255) / 256) want = (rows + 255) / 256;  // >= 256 rows per chunk
  if (want < 1) want = 1;
  rpc = (rows + want - 1) / want;
  chunks = (int)((rows + rpc - 1) / rpc);
}

// ---- per-chunk column sums: grid (chunks, C/8/V), 16 waves per block (one block
// per CU streams at HBM rate with 4 rows' loads in flight per lane), V lanes
// across 8-channel vectors, 64/V rows per wave step.  Two C-wide partial rows
// per chunk: [chunk][0][c] and [chunk][1][c].
// MODE 0 (forward statistics): s0 = sum (x - k), s1 = sum (x - k)^2, k = x[0][c]
// MODE 1..3 (backward, ACT = MODE-1): s0 = sum g, s1 = sum g * (x - mean), g = act'(dy, y)
template <int DT, int MODE>
__device__ __forceinline__ void bn_accum(const void *__restrict__ x, const void *__restrict__ dy,
                                         const void *__restrict__ y, long long e, const V8 &k, float slope,
                                         float (&s0)[8], float (&s1)[8]) {
  V8 t;
  ld8<DT>(t, x, e);
  if constexpr (MODE == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = t.v[j] - k.v[j];
      s0[j] += d;
      s1[j] = __builtin_fmaf(d, d, s1[j]);
    }
  } else {
    V8 g, o;
    ld8<DT>(g, dy, e);
    if constexpr (MODE != 1) ld8<DT>(o, y, e);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gg = act_bwd<MODE - 1>(g.v[j], MODE != 1 ? o.v[j] : 0.f, slope);
      s0[j] += gg;
      s1[j] = __builtin_fmaf(gg, t.v[j] - k.v[j], s1[j]);
    }
  }
}

// what the final step writes (forward: statistics, running stats, scale / shift; backward: dgamma,
// dbeta and the dx coefficients)
struct BnFin {
  const void *x;
  const float *gamma, *beta;
  float *rmean, *rvar;
  float momentum, eps;
  float *mean_io, *invstd_io, *dgamma, *dbeta;
  int eval;
  float *coef;
  long long *nbt;
  long long rows;
  int C;
};

// channel c's final from its combined sums s0, s1 (double)
template <int MODE, int DT>
__device__ __forceinline__ void bn_final_col(int c, double s0, double s1, const BnFin &f) {
  const int C = f.C;
  const double n = (double)f.rows;
  const double g = f.gamma ? (double)f.gamma[c] : 1.0;
  if constexpr (MODE == 0) {
    const double k = DT == 0 ? (double)reinterpret_cast<const float *>(f.x)[c]
                             : (double)(float)reinterpret_cast<const __bf16 *>(f.x)[c];
    const double m1 = s0 / n;
    double var = s1 / n - m1 * m1;
    if (var < 0.0) var = 0.0;
    const double mean = k + m1;
    const float invstd = 1.0f / sqrtf((float)var + f.eps);  // torch: 1 / sqrt(var + eps) in fp32
    f.mean_io[c] = (float)mean;
    f.invstd_io[c] = invstd;
    if (f.rmean) {
      f.rmean[c] = (float)(f.momentum * mean + (1.0 - f.momentum) * (double)f.rmean[c]);
      const double unbiased = f.rows > 1 ? var * n / (n - 1.0) : var;
      f.rvar[c] = (float)(f.momentum * unbiased + (1.0 - f.momentum) * (double)f.rvar[c]);
    }
    if (f.nbt && c == 0) f.nbt[0] += 1;  // module.num_batches_tracked (no separate add launch)
    const double sc = g * (double)invstd;
    f.coef[c] = (float)sc;
    f.coef[C + c] = (float)((f.beta ? (double)f.beta[c] : 0.0) - (double)(float)mean * sc);
  } else {
    const double inv = (double)f.invstd_io[c];
    if (f.dgamma) f.dgamma[c] = (float)(s1 * inv);
    if (f.dbeta) f.dbeta[c] = (float)s0;
    const double ca = g * inv;
    double cb = 0.0, cc = 0.0;
    if (!f.eval) {
      cb = -g * inv * inv * inv * s1 / n;
      cc = -ca * s0 / n - cb * (double)f.mean_io[c];
    }
    f.coef[c] = (float)ca;
    f.coef[C + c] = (float)cb;
    f.coef[2 * C + c] = (float)cc;
  }
}

// Arrival counters of the fused final (bn_partial_kernel<.., FUSE = true>): zero at load; every
// launch takes its own `strips` slots (bn_arrive_slots) and the last arriving block of a strip
// resets its slot, so a captured graph replays with every slot back at zero.
constexpr unsigned kBnSlots = 1u << 16;
__device__ unsigned g_bn_arrive[kBnSlots];

template <int DT, int MODE, bool FUSE>
__global__ __launch_bounds__(64 * kBnWaves) void bn_partial_kernel(const void *__restrict__ x,
                                                                   const void *__restrict__ dy,
                                                                   const void *__restrict__ y,
                                                                   const float *__restrict__ mean, long long rows,
                                                                   int C, int V, long long rpc, float slope,
                                                                   float *__restrict__ part, BnFin fin,
                                                                   unsigned slot) {
  extern __shared__ float red[];  // [kBnWaves][2][V*8]; FUSE: also the final's [2][16][V*8] doubles
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rw = 64 / V;
  const int rsub = lane / V, vi = lane - rsub * V;
  const int col = (blockIdx.y * V + vi) * 8;
  const long long r0 = blockIdx.x * rpc, r1 = min(rows, r0 + rpc);
  V8 k;
  if constexpr (MODE == 0) {
    ld8<DT>(k, x, col);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) k.v[j] = mean[col + j];
  }
  float s0[8], s1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s0[j] = s1[j] = 0.f;
  const long long step = (long long)kBnWaves * rw;
  long long r = r0 + w * rw + rsub;
  // kBnUnroll rows per iteration: their loads issue before any of them is consumed
  for (; r + (kBnUnroll - 1) * step < r1; r += kBnUnroll * step) {
    const long long e = r * C + col, es = step * C;
#pragma unroll
    for (int u = 0; u < kBnUnroll; ++u) bn_accum<DT, MODE>(x, dy, y, e + u * es, k, slope, s0, s1);
  }
  for (; r < r1; r += step) bn_accum<DT, MODE>(x, dy, y, r * C + col, k, slope, s0, s1);
  for (int o = V; o < 64; o <<= 1)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s0[j] += __shfl_xor(s0[j], o, 64);
      s1[j] += __shfl_xor(s1[j], o, 64);
    }
  const int W8 = V * 8;
  if (rsub == 0)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(w * 2) * W8 + vi * 8 + j] = s0[j];
      red[(w * 2 + 1) * W8 + vi * 8 + j] = s1[j];
    }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * W8; i += 64 * kBnWaves) {
    const int h = i / W8, c = i - h * W8;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < kBnWaves; ++q) s += red[(q * 2 + h) * W8 + c];
    float *dst = part + (long long)blockIdx.x * 2 * C + h * C + blockIdx.y * W8 + c;
    if constexpr (FUSE)
      __hip_atomic_store(dst, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // sc1: written through
    else
      *dst = s;
  }
  if constexpr (FUSE) {
    // The strip's last block to finish runs bn_final_kernel's step for the strip's W8 channels, in
    // the same order (16 chunk groups summed in double, then the groups in order): one launch less.
    // Hand-off without an L2 write-back (a __threadfence() per block cost more than the launch it
    // saved): the partial rows are stored sc1 (write-through), every storing wave drains its stores,
    // one lane per block counts the block in with an agent-scope add, and the block whose add came
    // last reads every partial with sc1 loads.
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      last = __hip_atomic_fetch_add(&g_bn_arrive[slot + blockIdx.y], 1u, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    const int chunks = gridDim.x;
    double *dred = reinterpret_cast<double *>(red);   // [2][16][W8]
    for (int pi = threadIdx.x; pi < 16 * W8; pi += 64 * kBnWaves) {
      const int grp = pi / W8, cj = pi - grp * W8, c = blockIdx.y * W8 + cj;
      float pa[16], pb[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int k = grp + 16 * i;
        pa[i] = k < chunks ? __hip_atomic_load(part + (long long)k * 2 * C + c, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)
                           : 0.f;
        pb[i] = k < chunks ? __hip_atomic_load(part + (long long)k * 2 * C + C + c, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)
                           : 0.f;
      }
      double a = 0.0, b = 0.0;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        a += (double)pa[i];
        b += (double)pb[i];
      }
      dred[grp * W8 + cj] = a;
      dred[(16 + grp) * W8 + cj] = b;
    }
    __syncthreads();
    for (int cj = threadIdx.x; cj < W8; cj += 64 * kBnWaves) {
      double s0 = 0.0, s1 = 0.0;
      for (int i = 0; i < 16; ++i) {
        s0 += dred[i * W8 + cj];
        s1 += dred[(16 + i) * W8 + cj];
      }
      bn_final_col<MODE == 0 ? 0 : 1, DT>(blockIdx.y * W8 + cj, s0, s1, fin);
    }
    if (threadIdx.x == 0)   // back to zero for the next launch that draws this slot
      __hip_atomic_store(&g_bn_arrive[slot + blockIdx.y], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- one 512-thread block (16 groups of 32 channel lanes) per 32 channels: the
// chunk partials combined in double in a fixed order.
// MODE 0: forward statistics -> save_mean / save_invstd, running stats, coef = (scale, shift)
// MODE 1: backward -> dgamma, dbeta, coef = (a, b, c) with dx = a g + b x + c
//         (batch statistics: the full BN gradient; `eval` = 1: running statistics, dx = a g)
template <int MODE, int DT>
__global__ __launch_bounds__(512) void bn_final_kernel(const float *__restrict__ part, int chunks, BnFin fin) {
  __shared__ double red[2][16][33];
  const int C = fin.C;
  const int cl = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  double a = 0.0, b = 0.0;
  if (c < C) {
    // chunks <= 256: at most 16 per group, all loads issued before the adds
    float pa[16], pb[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int k = grp + 16 * i;
      pa[i] = k < chunks ? part[(long long)k * 2 * C + c] : 0.f;
      pb[i] = k < chunks ? part[(long long)k * 2 * C + C + c] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      a += (double)pa[i];
      b += (double)pb[i];
    }
  }
  red[0][grp][cl] = a;
  red[1][grp][cl] = b;
  __syncthreads();
  if (grp != 0 || c >= C) return;
  double s0 = 0.0, s1 = 0.0;
  for (int i = 0; i < 16; ++i) {
    s0 += red[0][i][cl];
    s1 += red[1][i][cl];
  }
  bn_final_col<MODE, DT>(c, s0, s1, fin);
}

// eval-mode forward coefficients from the running statistics
__global__ void bn_eval_coef_kernel(int C, const float *__restrict__ gamma, const float *__restrict__ beta,
                                    const float *__restrict__ rmean, const float *__restrict__ rvar, float eps,
                                    float *__restrict__ mean_out, float *__restrict__ invstd_out,
                                    float *__restrict__ coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = 1.0f / sqrtf(rvar[c] + eps);
  const float g = gamma ? gamma[c] : 1.f;
  const float sc = g * invstd;
  mean_out[c] = rmean[c];
  invstd_out[c] = invstd;
  coef[c] = sc;
  coef[C + c] = (beta ? beta[c] : 0.f) - rmean[c] * sc;
}

// ---- elementwise passes: 4 vectors per thread, per-channel coefficients in LDS.
// n8 < 2^31 vectors (checked on the host), vector v covers channels (v % (C/8)) * 8 ...
template <int DT, int RT, int ACT>
__global__ __launch_bounds__(256) void bn_apply_kernel(const void *__restrict__ x, const void *__restrict__ res,
                                                       const float *__restrict__ coef, int C, unsigned n8,
                                                       float slope, void *__restrict__ y) {
  extern __shared__ float sc[];  // [2][C]
  for (int i = threadIdx.x; i < 2 * C; i += 256) sc[i] = coef[i];
  __syncthreads();
  const unsigned nv = (unsigned)C >> 3;
  const unsigned base = blockIdx.x * 1024u + threadIdx.x;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const unsigned v = base + 256u * j;
    if (v >= n8) break;
    const int c0 = (int)(v % nv) * 8;
    V8 t, r;
    ld8<DT>(t, x, 8LL * v);
    if constexpr (RT >= 0) ld8<RT>(r, res, 8LL * v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float o = __builtin_fmaf(t.v[k], sc[c0 + k], sc[C + c0 + k]);
      // torch adds the residual to the BN output as stored (bf16-rounded for a bf16 x)
      if constexpr (RT >= 0) o = (DT == 1 ? (float)(__bf16)o : o) + r.v[k];
      t.v[k] = act_fwd<ACT>(o, slope);
    }
    st8<DT>(y, 8LL * v, t);
  }
}

template <int DT, int ACT, bool RES>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const void *__restrict__ dy, const void *__restrict__ y,
                                                           const void *__restrict__ x, const float *__restrict__ coef,
                                                           int C, unsigned n8, float slope, void *__restrict__ dx,
                                                           void *__restrict__ dres) {
  extern __shared__ float sc[];  // [3][C]
  for (int i = threadIdx.x; i < 3 * C; i += 256) sc[i] = coef[i];
  __syncthreads();
  const unsigned nv = (unsigned)C >> 3;
  const unsigned base = blockIdx.x * 1024u + threadIdx.x;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const unsigned v = base + 256u * j;
    if (v >= n8) break;
    const int c0 = (int)(v % nv) * 8;
    V8 g, o, t;
    ld8<DT>(g, dy, 8LL * v);
    if constexpr (ACT != 0) ld8<DT>(o, y, 8LL * v);
    ld8<DT>(t, x, 8LL * v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      g.v[k] = act_bwd<ACT>(g.v[k], ACT != 0 ? o.v[k] : 0.f, slope);
      t.v[k] = __builtin_fmaf(sc[c0 + k], g.v[k], __builtin_fmaf(sc[C + c0 + k], t.v[k], sc[2 * C + c0 + k]));
    }
    st8<DT>(dx, 8LL * v, t);
    if constexpr (RES) st8<DT>(dres, 8LL * v, g);
  }
}

// the fused final (PCOPS_BN_FUSED_FINAL, default on; read per call so a test can compare both forms)
// for strips of <= 64 channels: at 128 (C = 128) the last block's serial final cost more than
// the launch it saves (profiles/r5_bn_variants.txt)
bool bn_fuse(int C) {
  const char *e = getenv("PCOPS_BN_FUSED_FINAL");
  return (!e || atoi(e) != 0) && bn_v(C) * 8 <= 64;
}

// host side: `n` consecutive counters no other launch in flight holds.  A captured graph keeps its
// slots for every replay, so launches made while capturing draw from the lower half and eager launches
// from the upper half: an eager launch can never share a counter with a replay running beside it
// (after the eager half wraps it would otherwise be handed a graph's slots).
unsigned bn_arrive_slots(int n, hipStream_t s) {
  constexpr unsigned half = kBnSlots / 2;
  static std::atomic<unsigned> next[2];
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  const bool cap = hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusActive;
  unsigned b = next[cap ? 0 : 1].fetch_add((unsigned)n) % half;
  if (b + (unsigned)n > half) b = 0;
  return (cap ? 0u : half) + b;
}

template <int DT, bool FUSE>
void launch_partial_t(int mode, const void *x, const void *dy, const void *y, const float *mean, long long rows, int C,
                      float slope, float *part, int chunks, long long rpc, const BnFin &fin, hipStream_t s) {
  const int V = bn_v(C);
  const dim3 grid(chunks, C / 8 / V), block(64 * kBnWaves);
  const size_t lds = FUSE ? (size_t)2 * 16 * V * 8 * sizeof(double) : (size_t)kBnWaves * 2 * V * 8 * sizeof(float);
  const unsigned slot = FUSE ? bn_arrive_slots(C / 8 / V, s) : 0u;
  switch (mode) {
    case 0: hipLaunchKernelGGL((bn_partial_kernel<DT, 0, FUSE>), grid, block, lds, s, x, dy, y, mean, rows, C, V, rpc, slope, part, fin, slot); break;
    case 1: hipLaunchKernelGGL((bn_partial_kernel<DT, 1, FUSE>), grid, block, lds, s, x, dy, y, mean, rows, C, V, rpc, slope, part, fin, slot); break;
    case 2: hipLaunchKernelGGL((bn_partial_kernel<DT, 2, FUSE>), grid, block, lds, s, x, dy, y, mean, rows, C, V, rpc, slope, part, fin, slot); break;
    default: hipLaunchKernelGGL((bn_partial_kernel<DT, 3, FUSE>), grid, block, lds, s, x, dy, y, mean, rows, C, V, rpc, slope, part, fin, slot); break;
  }
}

// partial sums + final: one launch (fused) or two
template <int DT>
void launch_stats(int mode, const void *x, const void *dy, const void *y, const float *mean, long long rows, int C,
                  float slope, float *part, int chunks, long long rpc, const BnFin &fin, hipStream_t s) {
  if (bn_fuse(C)) {
    launch_partial_t<DT, true>(mode, x, dy, y, mean, rows, C, slope, part, chunks, rpc, fin, s);
    return;
  }
  launch_partial_t<DT, false>(mode, x, dy, y, mean, rows, C, slope, part, chunks, rpc, fin, s);
  if (mode == 0)
    hipLaunchKernelGGL((bn_final_kernel<0, DT>), dim3((C + 31) / 32), dim3(512), 0, s, part, chunks, fin);
  else
    hipLaunchKernelGGL((bn_final_kernel<1, DT>), dim3((C + 31) / 32), dim3(512), 0, s, part, chunks, fin);
}

template <int DT, int RT>
void launch_apply(int act, const void *x, const void *res, const float *coef, int C, unsigned n8, float slope, void *y,
                  hipStream_t s) {
  const dim3 grid((n8 + 1023) / 1024);
  const size_t lds = 2 * C * sizeof(float);
  if (act == 1)
    hipLaunchKernelGGL((bn_apply_kernel<DT, RT, 1>), grid, dim3(256), lds, s, x, res, coef, C, n8, slope, y);
  else if (act == 2)
    hipLaunchKernelGGL((bn_apply_kernel<DT, RT, 2>), grid, dim3(256), lds, s, x, res, coef, C, n8, slope, y);
  else
    hipLaunchKernelGGL((bn_apply_kernel<DT, RT, 0>), grid, dim3(256), lds, s, x, res, coef, C, n8, slope, y);
}

template <int DT, int ACT>
void launch_bwd_apply(bool res, const void *dy, const void *y, const void *x, const float *coef, int C, unsigned n8,
                      float slope, void *dx, void *dres, hipStream_t s) {
  const dim3 grid((n8 + 1023) / 1024);
  const size_t lds = 3 * C * sizeof(float);
  if (res)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<DT, ACT, true>), grid, dim3(256), lds, s, dy, y, x, coef, C, n8, slope,
                       dx, dres);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<DT, ACT, false>), grid, dim3(256), lds, s, dy, y, x, coef, C, n8, slope,
                       dx, dres);
}

bool bn_shape_ok(long long rows, int C) {
  return rows > 0 && C > 0 && C % 8 == 0 && C <= 512 && rows * (long long)C / 8 < (1LL << 31);
}

}  // namespace

extern "C" unsigned long long pcops_batchnorm_workspace_bytes(long long rows, int C) {
  if (!bn_shape_ok(rows, C)) return 0;
  int chunks;
  long long rpc;
  bn_shape(rows, C, chunks, rpc);
  return ((unsigned long long)chunks * 2 * C + 3ULL * C) * sizeof(float);
}

extern "C" int pcops_batchnorm_fwd(const void *x, int dtype, const void *res, int res_dtype, long long rows, int C,
                                   const float *gamma, const float *beta, float *running_mean, float *running_var,
                                   float momentum, float eps, int batch_stats, int act, float slope, void *y,
                                   float *save_mean, float *save_invstd, void *workspace,
                                   unsigned long long workspace_bytes, long long *num_batches_tracked,
                                   pcops_stream_t stream) {
  if (rows < 0 || C <= 0 || (dtype != 0 && dtype != 1) || act < 0 || act > 2) return PCOPS_ERR_INVALID;
  if (res && res_dtype != 0 && res_dtype != 1) return PCOPS_ERR_INVALID;
  if (rows == 0) return PCOPS_OK;
  if (!bn_shape_ok(rows, C)) return PCOPS_ERR_UNSUPPORTED;
  if (!x || !y || !save_mean || !save_invstd) return PCOPS_ERR_INVALID;
  if (!batch_stats && (!running_mean || !running_var)) return PCOPS_ERR_INVALID;
  if ((running_mean == nullptr) != (running_var == nullptr)) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_batchnorm_workspace_bytes(rows, C)) return PCOPS_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  int chunks;
  long long rpc;
  bn_shape(rows, C, chunks, rpc);
  float *part = (float *)workspace;
  float *coef = part + (long long)chunks * 2 * C;
  if (batch_stats) {
    BnFin fin{x,         gamma,   beta,    running_mean, running_var, momentum,
              eps,       save_mean, save_invstd, nullptr, nullptr,     0,
              coef,      running_mean ? num_batches_tracked : nullptr, rows, C};
    if (dtype == 0)
      launch_stats<0>(0, x, nullptr, nullptr, nullptr, rows, C, 0.f, part, chunks, rpc, fin, s);
    else
      launch_stats<1>(0, x, nullptr, nullptr, nullptr, rows, C, 0.f, part, chunks, rpc, fin, s);
  } else {
    hipLaunchKernelGGL(bn_eval_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, s, C, gamma, beta, running_mean,
                       running_var, eps, save_mean, save_invstd, coef);
  }
  const unsigned n8 = (unsigned)(rows * C / 8);
  const int rt = res ? res_dtype : -1;
  if (dtype == 0) {
    if (rt < 0) launch_apply<0, -1>(act, x, res, coef, C, n8, slope, y, s);
    else if (rt == 0) launch_apply<0, 0>(act, x, res, coef, C, n8, slope, y, s);
    else launch_apply<0, 1>(act, x, res, coef, C, n8, slope, y, s);
  } else {
    if (rt < 0) launch_apply<1, -1>(act, x, res, coef, C, n8, slope, y, s);
    else if (rt == 0) launch_apply<1, 0>(act, x, res, coef, C, n8, slope, y, s);
    else launch_apply<1, 1>(act, x, res, coef, C, n8, slope, y, s);
  }
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_batchnorm_bwd(const void *dy, const void *y, const void *x, int dtype, long long rows, int C,
                                   const float *gamma, const float *save_mean, const float *save_invstd,
                                   int batch_stats, int act, float slope, void *dx, void *dres, float *dgamma,
                                   float *dbeta, void *workspace, unsigned long long workspace_bytes,
                                   pcops_stream_t stream) {
  if (rows < 0 || C <= 0 || (dtype != 0 && dtype != 1) || act < 0 || act > 2) return PCOPS_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  if (rows == 0) {
    if ((dgamma && pc_memset_async(dgamma, 0, sizeof(float) * C, s) != hipSuccess) ||
        (dbeta && pc_memset_async(dbeta, 0, sizeof(float) * C, s) != hipSuccess))
      return PCOPS_ERR_LAUNCH;
    return PCOPS_OK;
  }
  if (!bn_shape_ok(rows, C)) return PCOPS_ERR_UNSUPPORTED;
  if (!dy || !x || !dx || !save_mean || !save_invstd || (act != 0 && !y)) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_batchnorm_workspace_bytes(rows, C)) return PCOPS_ERR_WORKSPACE;
  int chunks;
  long long rpc;
  bn_shape(rows, C, chunks, rpc);
  float *part = (float *)workspace;
  float *coef = part + (long long)chunks * 2 * C;
  const int mode = 1 + act;
  BnFin fin{x,       gamma,  nullptr, nullptr, nullptr, 0.f, 0.f, (float *)save_mean, (float *)save_invstd, dgamma,
            dbeta,   batch_stats ? 0 : 1, coef, nullptr, rows, C};
  if (dtype == 0)
    launch_stats<0>(mode, x, dy, y, save_mean, rows, C, slope, part, chunks, rpc, fin, s);
  else
    launch_stats<1>(mode, x, dy, y, save_mean, rows, C, slope, part, chunks, rpc, fin, s);
  const unsigned n8 = (unsigned)(rows * C / 8);
  const bool r = dres != nullptr;
  if (dtype == 0) {
    if (act == 1) launch_bwd_apply<0, 1>(r, dy, y, x, coef, C, n8, slope, dx, dres, s);
    else if (act == 2) launch_bwd_apply<0, 2>(r, dy, y, x, coef, C, n8, slope, dx, dres, s);
    else launch_bwd_apply<0, 0>(r, dy, y, x, coef, C, n8, slope, dx, dres, s);
  } else {
    if (act == 1) launch_bwd_apply<1, 1>(r, dy, y, x, coef, C, n8, slope, dx, dres, s);
    else if (act == 2) launch_bwd_apply<1, 2>(r, dy, y, x, coef, C, n8, slope, dx, dres, s);
    else launch_bwd_apply<1, 0>(r, dy, y, x, coef, C, n8, slope, dx, dres, s);
  }
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
