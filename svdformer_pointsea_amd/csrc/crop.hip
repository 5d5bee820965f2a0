// seprate_point_cloud's crop (utils/helpers.py:96-111): the points of each cloud ordered by their distance
// to the crop centre (torch.argsort ascending), a contiguous range of that order packed to the front of a
// zero-tailed buffer.  The reference loops over the batch and slices `idx[num_crop:]` per sample; the
// batched restatement (data.py) ran torch.argsort (a segmented radix sort: ~20 launches) and a gather /
// mask chain (~10 more) -- this is one launch, one workgroup per cloud:
//   * keys (distance bits << 32 | point index) in LDS: a non-negative float's bits order like the float,
//     NaN sorts last (as torch's sort), and equal distances keep index order (the radix sort torch runs
//     is stable);
//   * a bitonic sort of the next power of two >= N keys (padding keys ~0 sort last), P / 2 compare-exchanges
//     per pass over the block, log2(P) (log2(P) + 1) / 2 passes;
//   * row j of cloud b's output is the point of rank start[b] + j (clamped to N - 1), times 1 for
//     j < count[b] and 0 past it -- data.py's _pack, value for value (a tail row holds x * 0, so -0.0 for a
//     negative coordinate, NaN for a non-finite one, as there).
#include "common.h"

namespace {

constexpr int kCropThreads = 1024;
constexpr int kCropMaxN = 16384;   // 16384 keys x 8 B = 128 KB of LDS

__global__ __launch_bounds__(kCropThreads) void crop_pack_kernel(const float *__restrict__ dist,
                                                                 const float *__restrict__ xyz,
                                                                 const long long *__restrict__ start,
                                                                 const long long *__restrict__ count, int N, int P,
                                                                 int n_max, float *__restrict__ out,
                                                                 int *__restrict__ counts) {
  extern __shared__ unsigned long long crop_keys[];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float *d = dist + (size_t)b * N;
  for (int i = tid; i < P; i += kCropThreads)
    crop_keys[i] = i < N ? ((unsigned long long)__float_as_uint(d[i]) << 32) | (unsigned)i : ~0ull;
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P / 2; i += kCropThreads) {
        const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1)), hi = lo + j;
        const unsigned long long a = crop_keys[lo], c = crop_keys[hi];
        if ((a > c) == ((lo & k) == 0)) {
          crop_keys[lo] = c;
          crop_keys[hi] = a;
        }
      }
      __syncthreads();
    }
  const long long s0 = start[b];
  const int s = (int)(s0 < 0 ? 0 : (s0 > N ? N : s0));
  long long c0 = count ? count[b] : (long long)(N - s);
  const int cnt = (int)(c0 < 0 ? 0 : (c0 > N - s ? N - s : c0));
  if (tid == 0 && counts) counts[b] = cnt;
  const float *p = xyz + (size_t)b * N * 3;
  float *o = out + (size_t)b * n_max * 3;
  for (int j = tid; j < n_max; j += kCropThreads) {
    const int src = min(s + j, N - 1);
    const int k = (int)(unsigned)(crop_keys[src] & 0xffffffffu);
    const float keep = j < cnt ? 1.f : 0.f;
    o[3 * j] = p[3 * k] * keep;
    o[3 * j + 1] = p[3 * k + 1] * keep;
    o[3 * j + 2] = p[3 * k + 2] * keep;
  }
}

}  // namespace

extern "C" int pcops_crop_pack(const float *dist, const float *xyz, const long long *start, const long long *count,
                               int B, int N, int n_max, float *out, int *counts, pcops_stream_t stream) {
  if (B < 0 || N < 0 || n_max < 0 || N > kCropMaxN) return PCOPS_ERR_INVALID;
  if (B == 0 || n_max == 0) return PCOPS_OK;
  if (N == 0 || !dist || !xyz || !start || !out) return PCOPS_ERR_INVALID;
  int P = 1;
  while (P < N) P <<= 1;
  if (P < 2) P = 2;
  const size_t lds = (size_t)P * sizeof(unsigned long long);
  static const hipError_t attr = hipFuncSetAttribute((const void *)crop_pack_kernel,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                                      kCropMaxN * (int)sizeof(unsigned long long));
  if (attr != hipSuccess) return PCOPS_ERR_LAUNCH;
  hipLaunchKernelGGL(crop_pack_kernel, dim3(B), dim3(kCropThreads), lds, (hipStream_t)stream, dist, xyz, start, count,
                     N, P, n_max, out, counts);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
