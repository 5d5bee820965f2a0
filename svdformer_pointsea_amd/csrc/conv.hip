// 3x3 / stride 1 / pad 1 convolution of channels_last (NHWC) bf16 activations
// on MFMA (v_mfma_f32_16x16x32_bf16, fp32 accumulation): the ResNet BasicBlock
// convs of SVDFormer's image encoder (models/resnet.py:36-70 via
// models/SVDFormer.py:139-146: C = 16 at 224x224, 32 at 112x112; 96 images per
// PCN batch), where MIOpen's NHWC kernels ran 2.5-6x below HBM speed.
//
// forward / input gradient (implicit GEMM, one kernel):
//   y[p][co] = sum_{tap, ci} x[p + off(tap)][ci] * w[co][tap][ci]      (w: OHWI bf16)
//   as D = A . B with A = w (M = co, K = (tap, ci)) held in registers and
//   B = the input window (K x N = pixels) read from an LDS image of the block's
//   (4 + 2) x (64 + 2) input rows: lane l reads the 8 channels k = 8(l>>4)..+7 of
//   pixel l&15 at one tap -- one ds_read_b128, no transpose.  The input gradient
//   of a stride-1 conv is the same product on dy with w'[ci][tap][co] =
//   w[co][ci][8 - tap] (flipped, transposed: built on the host).
// weight gradient:
//   dW[co][tap][ci] = sum_p dy[p][co] * x[p + off(tap)][ci]
//   K = pixels: both operands are read with ds_read_b64_tr_b16 (4 pixels x 16
//   channels per 16-lane group, delivered channel-major) from LDS images of the
//   dy tile and the haloed x tile; one A fragment serves the 9 taps.  Each block
//   loops over tiles (prefetching the next one), keeps its partial dW in registers and
//   writes it once; two small kernels sum the block partials in a fixed order (deterministic).
#include "common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kTH = 4;        // output rows per tile (one per wave)
constexpr int kTW = 64;       // output columns per tile
[[maybe_unused]] constexpr int kLW = kTW + 2;  // haloed input tile columns (weight gradient)

__device__ __forceinline__ f32x4 mfma16(const bf16x8 &a, const bf16x8 &b, const f32x4 &c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Tile staging, global -> registers -> LDS, split in two halves so a block can
// issue every load of a tile before its first LDS write (one memory latency per
// tile instead of one per 16-B vector) and can prefetch the next tile while it
// computes.  A rectangle of R rows x L columns x C channels starting at (hb, wb)
// of image n is held as [row][col][C] bf16; outside the image reads as zero.
template <int C, int R, int L, int NTH = 256>
struct Stage {
  static constexpr int VPP = C / 8, TOT = R * L * VPP, PER = (TOT + NTH - 1) / NTH;
  bf16x8 v[PER];
  __device__ __forceinline__ void load(const __bf16 *__restrict__ x, int n, int hb, int wb, int H, int W) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = threadIdx.x + NTH * j;
      const int vv = i % VPP, pc = i / VPP, c = pc % L, r = pc / L;
      const int hh = hb + r, ww = wb + c;
      v[j] = bf16x8{};
      if (i < TOT && hh >= 0 && hh < H && ww >= 0 && ww < W)
        v[j] = *reinterpret_cast<const bf16x8 *>(x + (((long long)n * H + hh) * W + ww) * C + 8 * vv);
    }
  }
  __device__ __forceinline__ void store(__bf16 *tile) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = threadIdx.x + NTH * j;
      if (i < TOT) *reinterpret_cast<bf16x8 *>(tile + 8 * i) = v[j];
    }
  }
};

// XCD-aware tile order: block b runs on XCD b % 8 (round-robin dispatch), so tile
// t = (b % 8) * per + b / 8 gives every XCD a contiguous run of tiles -- a tile and the
// one below it (t + tiles-per-row) run back to back on one XCD and the shared halo
// rows hit in that XCD's L2 instead of being fetched from HBM twice.
__device__ __forceinline__ long long xcd_tile(long long b, long long tiles) {
  const long long per = (tiles + 7) / 8;
  return (b % 8) * per + b / 8;
}

// ---------------------------------------------------------------- forward / dgrad
// res != nullptr: y = bf16(float(bf16(conv)) + float(res)) -- the input gradient of a BasicBlock's
// first conv plus the gradient its input also receives through the block's identity branch, added
// exactly as autograd's bf16 accumulation of the two would (both terms rounded to bf16 first)
template <int CI, int CO, int TW>
__global__ __launch_bounds__(256) void conv3x3_fwd_kernel(const __bf16 *__restrict__ x,
                                                          const __bf16 *__restrict__ w, __bf16 *__restrict__ y,
                                                          int H, int W, int N, const __bf16 *__restrict__ res) {
  constexpr int KC = (9 * CI + 31) / 32;  // K chunks of 32 over (tap, ci); the tail has zero weights
  constexpr int MT = CO / 16;
  constexpr int LW = TW + 2;
  __shared__ __attribute__((aligned(16))) __bf16 tile[(kTH + 2) * LW * CI];
  const int tw = (W + TW - 1) / TW, th = (H + kTH - 1) / kTH;
  const long long tiles = (long long)N * th * tw;
  const long long t = xcd_tile(blockIdx.x, tiles);
  if (t >= tiles) return;  // the grid is rounded up to a multiple of 8 blocks
  const int n = (int)(t / ((long long)th * tw)), h0 = (int)((t / tw) % th) * kTH, w0 = (int)(t % tw) * TW;
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6, g = l >> 4, i16 = l & 15;
  // weight fragments and the input tile loads issued together (one memory latency)
  bf16x8 a[MT][KC];
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    const int k0 = 32 * c + 8 * g, tap = k0 / CI, ci0 = k0 % CI;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      a[mt][c] = tap < 9 ? *reinterpret_cast<const bf16x8 *>(w + ((16 * mt + i16) * 9 + tap) * CI + ci0) : bf16x8{};
  }
  {
    Stage<CI, kTH + 2, LW> st;
    st.load(x, n, h0 - 1, w0 - 1, H, W);
    st.store(tile);
  }
  __syncthreads();
  const int orow = h0 + wv;
#pragma unroll
  for (int nt = 0; nt < TW / 16; ++nt) {
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int pc = 16 * nt + i16;  // output column in the tile (this lane's B column)
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int k0 = 32 * c + 8 * g;
      const int tap = k0 / CI < 9 ? k0 / CI : 8;  // K tail: finite data against zero weights
      const int ci0 = k0 % CI, dh = tap / 3, dw = tap % 3;
      const bf16x8 b = *reinterpret_cast<const bf16x8 *>(tile + ((wv + dh) * LW + pc + dw) * CI + ci0);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma16(a[mt][c], b, acc[mt]);
    }
    const int ow = w0 + pc;
    if (orow < H && ow < W) {
      const long long e0 = (((long long)n * H + orow) * W + ow) * CO + 4 * g;
      __bf16 *yp = y + e0;
      bf16x4 rv[MT];
      if (res)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) rv[mt] = *reinterpret_cast<const bf16x4 *>(res + e0 + 16 * mt);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (__bf16)acc[mt][r];
        if (res)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (__bf16)((float)o[r] + (float)rv[mt][r]);
        *reinterpret_cast<bf16x4 *>(yp + 16 * mt) = o;
      }
    }
  }
}

// ---------------------------------------------------------------- weight gradient
// grid: G blocks looping over the N * ceil(H/kTH) * ceil(W/kTW) tiles; partial
// dW per block in part[block][co][tap][ci] (fp32)
template <int CI, int CO>
__global__ __launch_bounds__(256) void conv3x3_wgrad_kernel(const __bf16 *__restrict__ x,
                                                            const __bf16 *__restrict__ dy, int N, int H, int W,
                                                            float *__restrict__ part) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int MT = CO / 16, NT = CI / 16;
  // one LDS arena: the x / dy images while looping, the 9*CO*CI fp32 block partial at the end
  constexpr int kXT = (kTH + 2) * kLW * CI, kGT = kTH * kTW * CO, kE = 9 * CO * CI;
  constexpr int kBytes = (2 * (kXT + kGT) > 4 * kE ? 2 * (kXT + kGT) : 4 * kE);
  __shared__ float4 arena[(kBytes + 15) / 16];
  __bf16 *xt = reinterpret_cast<__bf16 *>(arena);
  __bf16 *gt = xt + kXT;
  typedef __attribute__((address_space(3))) short4v lds_s4;
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6, g = l >> 4, i16 = l & 15, q = i16 >> 2, p = i16 & 3;
  const int tw = (W + kTW - 1) / kTW, th = (H + kTH - 1) / kTH;
  const long long tiles = (long long)N * th * tw;
  f32x4 acc[9][MT][NT];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[t][mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  Stage<CI, kTH + 2, kLW> sx;
  Stage<CO, kTH, kTW> sg;
  auto fetch = [&](long long t) {
    const int bx = (int)(t % tw);
    const long long r = t / tw;
    const int by = (int)(r % th), n = (int)(r / th);
    sx.load(x, n, by * kTH - 1, bx * kTW - 1, H, W);
    sg.load(dy, n, by * kTH, bx * kTW, H, W);
  };
  // XCD x = blockIdx.x % 8 owns tiles [x*per, (x+1)*per), strided by its G/8 blocks
  const long long per = (tiles + 7) / 8, lo = (blockIdx.x % 8) * per, hi = min(tiles, lo + per);
  const long long t0 = lo + blockIdx.x / 8, ts = gridDim.x / 8;
  if (t0 < hi) fetch(t0);
  for (long long t = t0; t < hi; t += ts) {
    __syncthreads();  // the previous tile's LDS reads are done
    sx.store(xt);
    sg.store(gt);
    __syncthreads();
    if (t + ts < hi) fetch(t + ts);  // next tile's loads fly during this tile's MFMAs
#pragma unroll
    for (int kc = 0; kc < kTW / 32; ++kc) {
      // pixels 32kc + 8g + (0..3 | 4..7) of row wv; lane 4q+p addresses row q, channels 4p..4p+3
      const int px0 = 32 * kc + 8 * g + q;
      bf16x8 a[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const __bf16 *base = gt + (wv * kTW + px0) * CO + 16 * mt + 4 * p;
        const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)base);
        const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(base + 4 * CO));
        a[mt] = __builtin_shufflevector(__builtin_bit_cast(bf16x4, lo), __builtin_bit_cast(bf16x4, hi), 0, 1, 2, 3,
                                        4, 5, 6, 7);
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int dh = tap / 3, dw = tap % 3;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const __bf16 *base = xt + ((wv + dh) * kLW + px0 + dw) * CI + 16 * nt + 4 * p;
          const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)base);
          const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(base + 4 * CI));
          const bf16x8 b = __builtin_shufflevector(__builtin_bit_cast(bf16x4, lo), __builtin_bit_cast(bf16x4, hi), 0,
                                                   1, 2, 3, 4, 5, 6, 7);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[tap][mt][nt] = mfma16(a[mt], b, acc[tap][mt][nt]);
        }
      }
    }
  }
  // reduce the four waves' partials through LDS (reusing the x image), then one
  // store per element: part[block][co][tap][ci]
  __syncthreads();
  float *red = reinterpret_cast<float *>(arena);
  constexpr int E = kE;
  for (int i = threadIdx.x; i < E; i += 256) red[i] = 0.f;
  __syncthreads();
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (wv == s) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int co = 16 * mt + 4 * g + r, ci = 16 * nt + i16;
              red[(co * 9 + tap) * CI + ci] += acc[tap][mt][nt][r];
            }
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < E; i += 256) part[(long long)blockIdx.x * E + i] = red[i];
#endif
}

// Weight gradient for C = 32 in 3-wave blocks, wave w = kernel row dh: its 3 taps for
// all 4 tile rows (12 accumulator tiles instead of 36 per wave, so three blocks share a CU
// where the one-row-per-wave form held one 4-wave block at 312 VGPRs).
template <int CI, int CO>
__global__ __launch_bounds__(192) void conv3x3_wgrad3_kernel(const __bf16 *__restrict__ x,
                                                             const __bf16 *__restrict__ dy, int N, int H, int W,
                                                             float *__restrict__ part) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int MT = CO / 16, NT = CI / 16;
  constexpr int kXT = (kTH + 2) * kLW * CI, kGT = kTH * kTW * CO, kE = 9 * CO * CI;
  constexpr int kBytes = (2 * (kXT + kGT) > 4 * kE ? 2 * (kXT + kGT) : 4 * kE);
  __shared__ float4 arena[(kBytes + 15) / 16];
  __bf16 *xt = reinterpret_cast<__bf16 *>(arena);
  __bf16 *gt = xt + kXT;
  typedef __attribute__((address_space(3))) short4v lds_s4;
  const int l = threadIdx.x & 63, dh = threadIdx.x >> 6, g = l >> 4, i16 = l & 15, q = i16 >> 2, p = i16 & 3;
  const int tw = (W + kTW - 1) / kTW, th = (H + kTH - 1) / kTH;
  const long long tiles = (long long)N * th * tw;
  f32x4 acc[3][MT][NT];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[t][mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  Stage<CI, kTH + 2, kLW, 192> sx;
  Stage<CO, kTH, kTW, 192> sg;
  auto fetch = [&](long long t) {
    const int bx = (int)(t % tw);
    const long long r = t / tw;
    const int by = (int)(r % th), n = (int)(r / th);
    sx.load(x, n, by * kTH - 1, bx * kTW - 1, H, W);
    sg.load(dy, n, by * kTH, bx * kTW, H, W);
  };
  const long long per = (tiles + 7) / 8, lo = (blockIdx.x % 8) * per, hi = min(tiles, lo + per);
  const long long t0 = lo + blockIdx.x / 8, ts = gridDim.x / 8;
  if (t0 < hi) fetch(t0);
  for (long long t = t0; t < hi; t += ts) {
    __syncthreads();
    sx.store(xt);
    sg.store(gt);
    __syncthreads();
    if (t + ts < hi) fetch(t + ts);
#pragma unroll
    for (int row = 0; row < kTH; ++row)
#pragma unroll
      for (int kc = 0; kc < kTW / 32; ++kc) {
        const int px0 = 32 * kc + 8 * g + q;
        bf16x8 a[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const __bf16 *base = gt + (row * kTW + px0) * CO + 16 * mt + 4 * p;
          const short4v lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)base);
          const short4v hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(base + 4 * CO));
          a[mt] = __builtin_shufflevector(__builtin_bit_cast(bf16x4, lo4), __builtin_bit_cast(bf16x4, hi4), 0, 1, 2,
                                          3, 4, 5, 6, 7);
        }
#pragma unroll
        for (int dw = 0; dw < 3; ++dw)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) {
            const __bf16 *base = xt + ((row + dh) * kLW + px0 + dw) * CI + 16 * nt + 4 * p;
            const short4v lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)base);
            const short4v hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(base + 4 * CI));
            const bf16x8 b = __builtin_shufflevector(__builtin_bit_cast(bf16x4, lo4), __builtin_bit_cast(bf16x4, hi4),
                                                     0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[dw][mt][nt] = mfma16(a[mt], b, acc[dw][mt][nt]);
          }
      }
  }
  // each wave owns taps 3*dh .. 3*dh+2: disjoint slots, one write each
  __syncthreads();
  float *red = reinterpret_cast<float *>(arena);
#pragma unroll
  for (int dw = 0; dw < 3; ++dw)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = 16 * mt + 4 * g + r, ci = 16 * nt + i16;
          red[(co * 9 + 3 * dh + dw) * CI + ci] = acc[dw][mt][nt][r];
        }
  __syncthreads();
  for (int i = threadIdx.x; i < kE; i += 192) part[(long long)blockIdx.x * kE + i] = red[i];
#endif
}

// dw = sum over blocks of part[b][co][tap][ci] in two fixed-order stages (a
// single pass had each thread walk all block rows: ~1 us of latency per 8 rows):
//   reduce1: part2[s][e] = sum_{b = s, s + kSplit, ...} part[b][e]       grid (E/256, kSplit)
//   reduce2: dw = sum_s part2[s][e], written in the weight's memory order -- OIHW
//            [co][ci][kh][kw] or channels_last OHWI [co][kh][kw][ci] -- as fp32 or bf16
constexpr int kSplit = 32;

__global__ __launch_bounds__(256) void conv3x3_wgrad_reduce1_kernel(const float *__restrict__ part, int blocks, int E,
                                                                    float *__restrict__ part2) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int b = blockIdx.y;
  for (; b + 7 * kSplit < blocks; b += 8 * kSplit)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += part[(long long)(b + j * kSplit) * E + e];
  for (; b < blocks; b += kSplit) acc[0] += part[(long long)b * E + e];
  part2[(long long)blockIdx.y * E + e] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
}

__global__ __launch_bounds__(256) void conv3x3_wgrad_reduce2_kernel(const float *__restrict__ part2, int CO, int CI,
                                                                    void *__restrict__ out, int odt, int ohwi) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int E = 9 * CO * CI;
  if (e >= E) return;
  float v = 0.f;
#pragma unroll
  for (int s2 = 0; s2 < kSplit; ++s2) v += part2[(long long)s2 * E + e];
  const int co = e / (9 * CI), rem = e - co * 9 * CI, tap = rem / CI, ci = rem - tap * CI;
  const int o = ohwi ? e : (co * CI + ci) * 9 + tap;
  if (odt == 0)
    reinterpret_cast<float *>(out)[o] = v;
  else
    reinterpret_cast<__bf16 *>(out)[o] = (__bf16)v;
}

int wgrad_blocks(int C) { return C <= 16 ? 1024 : 768; }

bool conv_ok(int N, int H, int W, int C) { return N > 0 && H > 0 && W > 0 && (C == 16 || C == 32); }

// ---------------------------------------------------------------- single-channel stem
// SVDFormer's image stem nn.Conv2d(1, 16, 3, padding=1, bias=False) on the (3B, 1, 224, 224)
// fp32 depth images (models/SVDFormer.py:139-140): K = 9 is too short for MFMA, so VALU.
// The input is rounded to bf16 as autocast's conv would; products accumulate in fp32.
// fwd: one thread per output pixel, the 3 x 3 window from an LDS image of the block's
// (4 + 2) x (64 + 2) input rows, the 16 x 9 weights uniform (scalar loads), 16 bf16 out.
constexpr int kC1Out = 16;

__device__ __forceinline__ float bf16r(float v) { return (float)(__bf16)v; }

__global__ __launch_bounds__(256) void conv3x3_c1_fwd_kernel(const float *__restrict__ x,
                                                             const float *__restrict__ w, __bf16 *__restrict__ y,
                                                             int H, int W) {
  __shared__ float tile[(kTH + 2) * (kTW + 2)];
  const int n = blockIdx.z, h0 = blockIdx.y * kTH, w0 = blockIdx.x * kTW;
  for (int i = threadIdx.x; i < (kTH + 2) * (kTW + 2); i += 256) {
    const int r = i / (kTW + 2), c = i - r * (kTW + 2);
    const int hh = h0 - 1 + r, ww = w0 - 1 + c;
    tile[i] = (hh >= 0 && hh < H && ww >= 0 && ww < W) ? bf16r(x[((long long)n * H + hh) * W + ww]) : 0.f;
  }
  __syncthreads();
  const int r = threadIdx.x >> 6, c = threadIdx.x & 63;
  const int oh = h0 + r, ow = w0 + c;
  if (oh >= H || ow >= W) return;
  float v[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) v[t] = tile[(r + t / 3) * (kTW + 2) + c + t % 3];
  bf16x8 o[2];
#pragma unroll
  for (int co = 0; co < kC1Out; ++co) {
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) acc = __builtin_fmaf(v[t], bf16r(w[co * 9 + t]), acc);
    o[co >> 3][co & 7] = (__bf16)acc;
  }
  bf16x8 *yp = reinterpret_cast<bf16x8 *>(y + (((long long)n * H + oh) * W + ow) * kC1Out);
  yp[0] = o[0];
  yp[1] = o[1];
}

// wgrad: dW[co][tap] = sum_p dy[p][co] * x[p + off(tap)]; G blocks stride over the
// 4 x 64 output tiles, each thread accumulating its pixels' 144 products in registers;
// wave (DPP) + LDS block reduction, one partial row per block (summed by the reduce
// kernels below, in a fixed order)
__global__ __launch_bounds__(256) void conv3x3_c1_wgrad_kernel(const float *__restrict__ x,
                                                               const __bf16 *__restrict__ dy, int N, int H, int W,
                                                               float *__restrict__ part) {
  __shared__ float tile[(kTH + 2) * (kTW + 2)];
  __shared__ float red[4][kC1Out * 9];
  const int tw = (W + kTW - 1) / kTW, th = (H + kTH - 1) / kTH;
  const long long tiles = (long long)N * th * tw;
  const int r = threadIdx.x >> 6, c = threadIdx.x & 63;
  float acc[kC1Out * 9];
#pragma unroll
  for (int i = 0; i < kC1Out * 9; ++i) acc[i] = 0.f;
  // registers holding the NEXT tile (its loads fly while this tile's products run)
  constexpr int XPER = ((kTH + 2) * (kTW + 2) + 255) / 256;
  float xv[XPER];
  bf16x8 g0 = {}, g1 = {};
  auto fetch = [&](long long t) {
    const int bx = (int)(t % tw);
    const long long rr = t / tw;
    const int by = (int)(rr % th), n = (int)(rr / th);
    const int h0 = by * kTH, w0 = bx * kTW;
#pragma unroll
    for (int j = 0; j < XPER; ++j) {
      const int i = threadIdx.x + 256 * j;
      const int ir = i / (kTW + 2), ic = i - ir * (kTW + 2);
      const int hh = h0 - 1 + ir, ww = w0 - 1 + ic;
      xv[j] = (i < (kTH + 2) * (kTW + 2) && hh >= 0 && hh < H && ww >= 0 && ww < W)
                  ? x[((long long)n * H + hh) * W + ww] : 0.f;
    }
    const int oh = h0 + r, ow = w0 + c;
    g0 = bf16x8{};
    g1 = bf16x8{};
    if (oh < H && ow < W) {
      const bf16x8 *gp = reinterpret_cast<const bf16x8 *>(dy + (((long long)n * H + oh) * W + ow) * kC1Out);
      g0 = gp[0];
      g1 = gp[1];
    }
  };
  // XCD x = blockIdx.x % 8 owns tiles [x*per, (x+1)*per), strided by its G/8 blocks
  const long long per = (tiles + 7) / 8, lo = (blockIdx.x % 8) * per, hi = min(tiles, lo + per);
  const long long t0 = lo + blockIdx.x / 8, ts = gridDim.x / 8;
  if (t0 < hi) fetch(t0);
  for (long long t = t0; t < hi; t += ts) {
    __syncthreads();  // the previous tile's LDS reads are done
#pragma unroll
    for (int j = 0; j < XPER; ++j) {
      const int i = threadIdx.x + 256 * j;
      if (i < (kTH + 2) * (kTW + 2)) tile[i] = bf16r(xv[j]);
    }
    const bf16x8 c0 = g0, c1 = g1;
    __syncthreads();
    if (t + ts < hi) fetch(t + ts);
    float v[9];
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) v[tp] = tile[(r + tp / 3) * (kTW + 2) + c + tp % 3];
#pragma unroll
    for (int co = 0; co < kC1Out; ++co) {
      const float g = (float)(co < 8 ? c0[co] : c1[co - 8]);
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) acc[co * 9 + tp] = __builtin_fmaf(g, v[tp], acc[co * 9 + tp]);
    }
  }
  // wave sums (xor shuffles), then the four waves through LDS in a fixed order
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < kC1Out * 9; ++i) {
    float v = acc[i];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0) red[wv][i] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kC1Out * 9; i += 256)
    part[(long long)blockIdx.x * kC1Out * 9 + i] = ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
}

}  // namespace

namespace {
int conv3x3_fwd_impl(const void *x, const void *w, int N, int H, int W, int C, const void *res, void *y,
                     pcops_stream_t stream) {
  if (N < 0 || H < 0 || W < 0) return PCOPS_ERR_INVALID;
  if (N == 0 || H == 0 || W == 0) return PCOPS_OK;
  if (!conv_ok(N, H, W, C)) return PCOPS_ERR_UNSUPPORTED;
  if (!x || !w || !y) return PCOPS_ERR_INVALID;
  const __bf16 *rp = (const __bf16 *)res;
  hipStream_t s = (hipStream_t)stream;
  // 112-column tiles where they divide W exactly (the 224 / 112 images): no masked N-tiles
  const bool wide = W % 112 == 0;
  const int TW = wide ? 112 : 64;
  const long long tiles = (long long)((W + TW - 1) / TW) * ((H + kTH - 1) / kTH) * N;
  const dim3 grid((unsigned)(((tiles + 7) / 8) * 8));  // 1-D tile space, rounded up to 8 (XCD order)
  const __bf16 *xp = (const __bf16 *)x, *wp = (const __bf16 *)w;
  __bf16 *yp = (__bf16 *)y;
  if (C == 16) {
    if (wide) hipLaunchKernelGGL((conv3x3_fwd_kernel<16, 16, 112>), grid, dim3(256), 0, s, xp, wp, yp, H, W, N, rp);
    else hipLaunchKernelGGL((conv3x3_fwd_kernel<16, 16, 64>), grid, dim3(256), 0, s, xp, wp, yp, H, W, N, rp);
  } else {
    if (wide) hipLaunchKernelGGL((conv3x3_fwd_kernel<32, 32, 112>), grid, dim3(256), 0, s, xp, wp, yp, H, W, N, rp);
    else hipLaunchKernelGGL((conv3x3_fwd_kernel<32, 32, 64>), grid, dim3(256), 0, s, xp, wp, yp, H, W, N, rp);
  }
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
}  // namespace

extern "C" int pcops_conv3x3_fwd(const void *x, const void *w, int N, int H, int W, int C, void *y,
                                 pcops_stream_t stream) {
  return conv3x3_fwd_impl(x, w, N, H, W, C, nullptr, y, stream);
}

extern "C" int pcops_conv3x3_fwd_res(const void *x, const void *w, int N, int H, int W, int C, const void *res,
                                     void *y, pcops_stream_t stream) {
  if (!res) return PCOPS_ERR_INVALID;
  return conv3x3_fwd_impl(x, w, N, H, W, C, res, y, stream);
}

extern "C" unsigned long long pcops_conv3x3_wgrad_workspace_bytes(int C) {
  if (C != 16 && C != 32) return 0;
  return (unsigned long long)(wgrad_blocks(C) + kSplit) * 9 * C * C * sizeof(float);
}

extern "C" int pcops_conv3x3_wgrad(const void *x, const void *dy, int N, int H, int W, int C, void *dw, int dw_dtype,
                                   int dw_ohwi, void *workspace, unsigned long long workspace_bytes,
                                   pcops_stream_t stream) {
  if (N < 0 || H < 0 || W < 0 || !dw || (dw_dtype != 0 && dw_dtype != 1)) return PCOPS_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  if (N == 0 || H == 0 || W == 0) {
    if (pc_memset_async(dw, 0, (dw_dtype == 0 ? 4 : 2) * 9 * C * C, s) != hipSuccess) return PCOPS_ERR_LAUNCH;
    return PCOPS_OK;
  }
  if (!conv_ok(N, H, W, C)) return PCOPS_ERR_UNSUPPORTED;
  if (!x || !dy) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_conv3x3_wgrad_workspace_bytes(C)) return PCOPS_ERR_WORKSPACE;
  const int G = wgrad_blocks(C);
  float *part = (float *)workspace;
  if (C == 16)
    hipLaunchKernelGGL((conv3x3_wgrad_kernel<16, 16>), dim3(G), dim3(256), 0, s, (const __bf16 *)x,
                       (const __bf16 *)dy, N, H, W, part);
  else
    hipLaunchKernelGGL((conv3x3_wgrad3_kernel<32, 32>), dim3(G), dim3(192), 0, s, (const __bf16 *)x,
                       (const __bf16 *)dy, N, H, W, part);
  float *part2 = part + (long long)G * 9 * C * C;
  const int E = 9 * C * C;
  hipLaunchKernelGGL(conv3x3_wgrad_reduce1_kernel, dim3((E + 255) / 256, kSplit), dim3(256), 0, s, part, G, E, part2);
  hipLaunchKernelGGL(conv3x3_wgrad_reduce2_kernel, dim3((E + 255) / 256), dim3(256), 0, s, part2, C, C, dw, dw_dtype,
                     dw_ohwi);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

extern "C" int pcops_conv3x3_c1_fwd(const float *x, const float *w, int N, int H, int W, void *y,
                                    pcops_stream_t stream) {
  if (N < 0 || H < 0 || W < 0) return PCOPS_ERR_INVALID;
  if (N == 0 || H == 0 || W == 0) return PCOPS_OK;
  if (!x || !w || !y) return PCOPS_ERR_INVALID;
  const dim3 grid((W + kTW - 1) / kTW, (H + kTH - 1) / kTH, N);
  hipLaunchKernelGGL(conv3x3_c1_fwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, x, w, (__bf16 *)y, H, W);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}

constexpr int kC1Blocks = 1024;

extern "C" unsigned long long pcops_conv3x3_c1_wgrad_workspace_bytes(void) {
  return (unsigned long long)(kC1Blocks + kSplit) * kC1Out * 9 * sizeof(float);
}

extern "C" int pcops_conv3x3_c1_wgrad(const float *x, const void *dy, int N, int H, int W, void *dw, int dw_dtype,
                                      void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream) {
  if (N < 0 || H < 0 || W < 0 || !dw || (dw_dtype != 0 && dw_dtype != 1)) return PCOPS_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  if (N == 0 || H == 0 || W == 0) {
    if (pc_memset_async(dw, 0, (dw_dtype == 0 ? 4 : 2) * kC1Out * 9, s) != hipSuccess) return PCOPS_ERR_LAUNCH;
    return PCOPS_OK;
  }
  if (!x || !dy) return PCOPS_ERR_INVALID;
  if (!workspace || workspace_bytes < pcops_conv3x3_c1_wgrad_workspace_bytes()) return PCOPS_ERR_WORKSPACE;
  float *part = (float *)workspace, *part2 = part + (long long)kC1Blocks * kC1Out * 9;
  const int E = kC1Out * 9;
  hipLaunchKernelGGL(conv3x3_c1_wgrad_kernel, dim3(kC1Blocks), dim3(256), 0, s, x, (const __bf16 *)dy, N, H, W, part);
  hipLaunchKernelGGL(conv3x3_wgrad_reduce1_kernel, dim3((E + 255) / 256, kSplit), dim3(256), 0, s, part, kC1Blocks,
                     E, part2);
  // CI = 1: OIHW [co][0][kh][kw] and OHWI [co][kh][kw][0] are the same order
  hipLaunchKernelGGL(conv3x3_wgrad_reduce2_kernel, dim3((E + 255) / 256), dim3(256), 0, s, part2, kC1Out, 1, dw,
                     dw_dtype, 1);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
