// Diagnostic: verify the bf16 32x32x16 MFMA operand maps and ds_read_b64_tr_b16
// semantics on gfx950 with exact integer data.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void tr_probe(short *out) {
  __shared__ short lds[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += 64) lds[i] = (short)i;  // value = row*64 + col
  __syncthreads();
  const int l = threadIdx.x, i = l & 15, q = i >> 2, p = i & 3, g = l >> 4;
  // group g reads block rows 4g..4g+3, cols 0..15 (row stride 64)
  typedef __attribute__((address_space(3))) short4v lds_s4;
  short4v v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(lds + (4 * g + q) * 64 + 4 * p));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}

// C = A(32x16) * B(16x32) with A[i][k] = (i==k) ? 1 : 0 ... use integer data
__global__ void mfma_probe(float *out) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * h + j;
    a[j] = (__bf16)(float)(r * 16 + k);     // A[r][k]
    b[j] = (__bf16)(float)((k == r) ? 1 : 0); // B[k][col=r] = I (16x32)
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int e = 0; e < 16; ++e) out[l * 16 + e] = c[e];
}

int main() {
  short *d; float *f;
  (void)hipMalloc(&d, 64 * 4 * 2); (void)hipMalloc(&f, 64 * 16 * 4);
  tr_probe<<<1, 64>>>(d);
  short h[256]; (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("tr_b16: lane -> 4 values (value = row*64+col)\n");
  for (int l = 0; l < 64; l += 5) printf("lane %2d: %4d %4d %4d %4d\n", l, h[l*4], h[l*4+1], h[l*4+2], h[l*4+3]);
  mfma_probe<<<1, 64>>>(f);
  float hf[1024]; (void)hipMemcpy(hf, f, sizeof(hf), hipMemcpyDeviceToHost);
  // expected C[i][j] = sum_k A[i][k] B[k][j] = A[i][j] for j < 16 else 0 = i*16+j
  int bad = 0;
  for (int l = 0; l < 64; ++l) for (int e = 0; e < 16; ++e) {
    const int col = l & 31, row = (e & 3) + 8 * (e >> 2) + 4 * (l >> 5);
    const float exp = col < 16 ? row * 16 + col : 0;
    if (hf[l * 16 + e] != exp) { if (bad < 5) printf("mfma mismatch lane %d e %d got %f exp %f\n", l, e, hf[l*16+e], exp); ++bad; }
  }
  printf("mfma map mismatches: %d\n", bad);
  return 0;
}
