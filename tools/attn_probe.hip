// Diagnostic: exercise Prec<bf16,D>::product1/product2 with exact small-integer
// data and compare with a host matmul.
#include "../svdformer_pointsea_amd/csrc/attention.hip"
#include <cstdio>
#include <vector>

template <int D>
__global__ void p2_kernel(const float *T, const float *X, float *Yout) {
  using P = Prec<__bf16, D>;
  __shared__ __attribute__((aligned(16))) __bf16 lds[32 * P::kStride];
  for (int e = threadIdx.x; e < 32 * D; e += 64) lds[(e / D) * P::kStride + (e % D)] = (__bf16)T[e];
  __syncthreads();
  const int l = threadIdx.x, h = l >> 5;
  f32x16 x;
  for (int r = 0; r < 16; ++r) x[r] = X[acc_row(r, h) * 32 + (l & 31)];
  f32x16 Y[D / 32];
  for (int db = 0; db < D / 32; ++db) Y[db] = f32x16{};
  P::product2(Y, lds, x);
  for (int db = 0; db < D / 32; ++db)
    for (int r = 0; r < 16; ++r) Yout[(db * 32 + acc_row(r, h)) * 32 + (l & 31)] = Y[db][r];
}

int main() {
  const int D = 64;
  std::vector<float> T(32 * D), X(32 * 32), Y(D * 32), R(D * 32, 0.f);
  for (int i = 0; i < 32; ++i) for (int d = 0; d < D; ++d) T[i * D + d] = (float)((i * 7 + d * 3) % 11 - 5);
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) X[i * 32 + j] = (float)((i * 5 + j * 13) % 7 - 3);
  for (int d = 0; d < D; ++d) for (int j = 0; j < 32; ++j) for (int i = 0; i < 32; ++i) R[d * 32 + j] += T[i * D + d] * X[i * 32 + j];
  float *dT, *dX, *dY;
  (void)hipMalloc(&dT, T.size() * 4); (void)hipMalloc(&dX, X.size() * 4); (void)hipMalloc(&dY, Y.size() * 4);
  (void)hipMemcpy(dT, T.data(), T.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice);
  p2_kernel<D><<<1, 64>>>(dT, dX, dY);
  (void)hipMemcpy(Y.data(), dY, Y.size() * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int d = 0; d < D; ++d) for (int j = 0; j < 32; ++j)
    if (Y[d * 32 + j] != R[d * 32 + j]) { if (bad < 8) printf("Y[%d][%d] got %g exp %g\n", d, j, Y[d*32+j], R[d*32+j]); ++bad; }
  printf("product2 bf16 mismatches: %d of %d\n", bad, D * 32);
  return 0;
}
