// Timing probe of the dK/dV kernels at the PCN shapes (B*H = 256, L = 2048):
// attention.hip is compiled into this file, so -DPCOPS_DKV3_ABL=<bits> builds
// the ablations of attn_dkv3_kernel (see its header); prints ms per launch.
#include "../svdformer_pointsea_amd/csrc/attention.hip"
#include <cstdio>
#include <vector>

template <typename F>
static float time_ms(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

template <int D>
static void run(const char *tag) {
  const int B = 32, H = 8, L = 2048, E = H * D, BH = B * H;
  const size_t n = (size_t)L * B * E;
  std::vector<__bf16> h(n);
  unsigned s = 12345;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    h[i] = (__bf16)(((s >> 9) & 0xFFFF) / 65536.f - 0.5f);
  }
  __bf16 *q, *k, *v, *g, *dk, *dv;
  float *lse, *dl;
  for (__bf16 **p : {&q, &k, &v, &g, &dk, &dv}) (void)hipMalloc(p, n * 2);
  for (__bf16 *p : {q, k, v, g}) (void)hipMemcpy(p, h.data(), n * 2, hipMemcpyHostToDevice);
  (void)hipMalloc(&lse, (size_t)BH * L * 4);
  (void)hipMalloc(&dl, (size_t)BH * L * 4);
  std::vector<float> hl((size_t)BH * L, 9.f);
  (void)hipMemcpy(lse, hl.data(), hl.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemset(dl, 0, hl.size() * 4);
  // seq-first (L, B, E): sb = E, sh = D, srow = B * E
  const Strides st{E, D, (long long)B * E, E, D, (long long)B * E, E, D, (long long)B * E, E, D, (long long)B * E, H};
  const float scale = 1.f / sqrtf((float)D);
  const float flop = 8.f * BH * (float)L * L * D;
  const float t2 = time_ms([&] { dkv2_dispatch(q, k, v, g, lse, dl, dk, dv, BH, L, L, D, scale, st, 0); }, 10);
  const float t3 = time_ms([&] { launch_dkv3<D, 1>(q, k, v, g, lse, dl, dk, dv, BH, L, L, scale, st, 0); }, 10);
  printf("%s D=%d  dkv2 %.3f ms (%.0f TF)  dkv3 %.3f ms (%.0f TF)\n", tag, D, t2, flop / t2 / 1e9, t3, flop / t3 / 1e9);
  for (void *p : {(void *)q, (void *)k, (void *)v, (void *)g, (void *)dk, (void *)dv, (void *)lse, (void *)dl})
    (void)hipFree(p);
}

int main() {
  char tag[32];
  snprintf(tag, sizeof tag, "abl=%d", PCOPS_DKV3_ABL);
  run<128>(tag);
  run<96>(tag);
  return 0;
}
