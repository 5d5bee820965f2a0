// Diagnostic: FPS per-round segment breakdown (sweep / wave-reduce+pick /
// barrier wait / slot tree) from in-kernel s_memtime stamps, plus the clock.
#define FPS_STAMPS 1
#include "../svdformer_pointsea_amd/csrc/sampling.hip"
#include <cstdio>
#include <vector>

int main() {
  for (int N : {2048, 6144, 8192, 16384}) {
    const int B = 32, M = N >= 6144 ? 2048 : N / 4;
    std::vector<float> h(B * N * 3);
    unsigned s = 12345;
    for (auto &v : h) { s = s * 1664525u + 1013904223u; v = (s >> 8) * (1.0f / 16777216.0f) - 0.5f; }
    float *x; int *idx;
    (void)hipMalloc(&x, h.size() * 4); (void)hipMalloc(&idx, B * M * 4);
    (void)hipMemcpy(x, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep) pcops_furthest_point_sampling(x, B, N, M, idx, nullptr, 0, nullptr);
    (void)hipEventRecord(e0);
    pcops_furthest_point_sampling(x, B, N, M, idx, nullptr, 0, nullptr);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long st[8];
    (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(g_fps_stamps), sizeof(st));
    double tot = 0; for (int i = 0; i < 4; ++i) tot += st[i];
    double ghz = tot / (M - 1) / (ms * 1e6 / (M - 1));
    printf("N=%d M=%d: %.3f ms, %.3f us/round, cycles/round %.0f (sweep %.0f, reduce+pick %.0f, barrier %.0f, tree %.0f), implied clock %.2f GHz\n",
           N, M, ms, ms * 1e3 / (M - 1), tot / (M - 1), st[0] / (double)(M - 1), st[1] / (double)(M - 1),
           st[2] / (double)(M - 1), st[3] / (double)(M - 1), ghz);
    unsigned long long ws[16][4];
    (void)hipMemcpyFromSymbol(ws, HIP_SYMBOL(g_fps_wave_stamps), sizeof(ws));
    for (int w = 0; w < 16; ++w)
      printf("   wave %2d: sweep %5.0f reduce+pick %5.0f barrier %5.0f tree %5.0f\n", w, ws[w][0] / (double)(M - 1),
             ws[w][1] / (double)(M - 1), ws[w][2] / (double)(M - 1), ws[w][3] / (double)(M - 1));
  }
  return 0;
}
