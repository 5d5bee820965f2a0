// Adam / AdamW over the flat fp32 master buffer (train.FlatParams), the update of
// core/train_pcn.py:57-60 (Adam, weight_decay 0) and core/train_55.py:86-88 (AdamW, 5e-4),
// in one pass that also
//   * reads the bf16-shadow region's gradients as the bf16 bucket autograd filled
//     (FlatParams.grad16), instead of a widened fp32 copy of it, and
//   * writes that region's new bf16 shadow weights (the GEMM operands of the next step),
//     instead of a separate fp32 -> bf16 refresh pass over the master buffer.
// The arithmetic is torch's Adam (torch/optim/adam.py, the fused path's order):
//   AdamW: p *= 1 - lr*wd        Adam: g += wd*p
//   m = beta1*m + (1-beta1)*g    v = beta2*v + (1-beta2)*g*g
//   p -= (lr / (1 - beta1^t)) * m / (sqrt(v) / sqrt(1 - beta2^t) + eps)
// with t the step AFTER this update's increment (read from the optimizer's device step
// tensor, which the caller increments first -- as torch's capturable path does), lr from
// a device scalar when given (the LR schedule writes it between graph replays).
#include "common.h"

namespace {

struct AdamArgs {
  float *p, *m, *v;
  const __bf16 *g16;
  const float *g32;
  __bf16 *shadow;
  long long n16, n;
  const float *lr_dev, *step_dev;
  double lr, beta1, beta2, eps, wd;
  int adamw;
};

// torch's fused Adam element update (ATen FusedAdamMathFunctor): the hyper-parameters are doubles,
// so every product with one of them is formed in double and rounded once to fp32; the final
// step_size * m / denom is fp32
__device__ __forceinline__ void adam_elem(const AdamArgs &a, float &p, float &m, float &v, float g, float step_size,
                                          float bc2_sqrt, double lr) {
  if (a.wd != 0.0) {
    if (a.adamw)
      p = (float)((double)p - lr * a.wd * (double)p);
    else
      g = (float)((double)g + (double)p * a.wd);
  }
  m = (float)(a.beta1 * (double)m + (1.0 - a.beta1) * (double)g);
  v = (float)(a.beta2 * (double)v + (1.0 - a.beta2) * (double)g * (double)g);
  const float denom = (float)((double)(sqrtf(v) / bc2_sqrt) + a.eps);
  p = p - step_size * m / denom;
}

__global__ __launch_bounds__(256) void adam_flat_kernel(AdamArgs a) {
  const double t = *a.step_dev;
  const double lr = a.lr_dev ? (double)*a.lr_dev : a.lr;
  const float bc1 = (float)(1.0 - pow(a.beta1, t));
  const float bc2_sqrt = (float)sqrt(1.0 - pow(a.beta2, t));
  const float step_size = (float)(lr / (double)bc1);
  const long long stride = (long long)gridDim.x * 256 * 4;
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  for (long long i0 = ((long long)blockIdx.x * 256 + threadIdx.x) * 4; i0 < a.n; i0 += stride) {
    const bool in16 = i0 < a.n16;
    if (i0 + 4 <= a.n && (!in16 || i0 + 4 <= a.n16)) {
      // 4 elements in one region: 16-B accesses (8-B for the bf16 gradient / shadow)
      float4 p4 = *reinterpret_cast<const float4 *>(a.p + i0);
      float4 m4 = *reinterpret_cast<const float4 *>(a.m + i0);
      float4 v4 = *reinterpret_cast<const float4 *>(a.v + i0);
      float g[4];
      if (in16 && a.g16) {
        const bf16x4_t h = *reinterpret_cast<const bf16x4_t *>(a.g16 + i0);
#pragma unroll
        for (int k = 0; k < 4; ++k) g[k] = (float)h[k];
      } else {
        const float4 g4 = *reinterpret_cast<const float4 *>(a.g32 + i0);
        g[0] = g4.x, g[1] = g4.y, g[2] = g4.z, g[3] = g4.w;
      }
      adam_elem(a, p4.x, m4.x, v4.x, g[0], step_size, bc2_sqrt, lr);
      adam_elem(a, p4.y, m4.y, v4.y, g[1], step_size, bc2_sqrt, lr);
      adam_elem(a, p4.z, m4.z, v4.z, g[2], step_size, bc2_sqrt, lr);
      adam_elem(a, p4.w, m4.w, v4.w, g[3], step_size, bc2_sqrt, lr);
      *reinterpret_cast<float4 *>(a.p + i0) = p4;
      *reinterpret_cast<float4 *>(a.m + i0) = m4;
      *reinterpret_cast<float4 *>(a.v + i0) = v4;
      if (in16 && a.shadow) {
        bf16x4_t o;
        o[0] = (__bf16)p4.x, o[1] = (__bf16)p4.y, o[2] = (__bf16)p4.z, o[3] = (__bf16)p4.w;
        *reinterpret_cast<bf16x4_t *>(a.shadow + i0) = o;
      }
    } else {
      for (long long i = i0; i < i0 + 4 && i < a.n; ++i) {  // region seam / tail
        float p = a.p[i], m = a.m[i], v = a.v[i];
        const float g = (a.g16 && i < a.n16) ? (float)a.g16[i] : a.g32[i];
        adam_elem(a, p, m, v, g, step_size, bc2_sqrt, lr);
        a.p[i] = p;
        a.m[i] = m;
        a.v[i] = v;
        if (a.shadow && i < a.n16) a.shadow[i] = (__bf16)p;
      }
    }
  }
}

}  // namespace

extern "C" int pcops_adam_flat(float *param, const void *grad16, const float *grad32, long long n16, long long n,
                               float *exp_avg, float *exp_avg_sq, void *shadow16, const float *lr_dev, double lr,
                               const float *step_dev, double beta1, double beta2, double eps, double weight_decay,
                               int adamw, pcops_stream_t stream) {
  if (n < 0 || n16 < 0 || n16 > n) return PCOPS_ERR_INVALID;
  if (n == 0) return PCOPS_OK;
  if (!param || !exp_avg || !exp_avg_sq || !step_dev || (!grad32 && (!grad16 || n16 < n))) return PCOPS_ERR_INVALID;
  AdamArgs a{param, exp_avg, exp_avg_sq, (const __bf16 *)grad16, grad32, (__bf16 *)shadow16, grad16 || shadow16 ? n16 : 0, n,
             lr_dev, step_dev, lr, beta1, beta2, eps, weight_decay, adamw};
  long long g = (n + 1024 - 1) / 1024;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(adam_flat_kernel, dim3((unsigned)(g < 1 ? 1 : g)), dim3(256), 0, (hipStream_t)stream, a);
  PC_CHECK_LAUNCH();
  return PCOPS_OK;
}
