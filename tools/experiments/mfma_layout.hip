// Prints where v_mfma_f64_16x16x4f64 puts D[i][j] (lane, item) for A[i][k] = (lane = i + 16 k) and B[k][j] = (lane =
// j + 16 k) operand conventions: A = unit rows (A[i][k] = (k == 0) * (i + 1)), B[0][j] = 1000 (j + 1) -> D[i][j] =
// (i + 1) * 1000 (j + 1), decoded per lane / item.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(double* out) {
  const int l = threadIdx.x, i = l % 16, kk = l / 16;
  const double a = kk == 0 ? i + 1 : 0.0, b = kk == 0 ? 1000.0 * (i + 1) : 0.0;
  d4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int q = 0; q < 4; q++) out[4 * l + q] = c[q];
}
int main() {
  double* d;
  hipMalloc(&d, 256 * sizeof(double));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  double h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; l++)
    for (int q = 0; q < 4; q++) {
      const double v = h[4 * l + q];
      const int i = (int)(v / 1000.0 + 0.5), j = (int)(v - 1000.0 * i + 0.5);  // v = 1000 (i+1)(j+1)?
      (void)i; (void)j;
      const int ii = 4 * (l / 16) + q, jj = l % 16;
      if (v != 1000.0 * (ii + 1) * (jj + 1)) bad++;
      if (l < 20 || l % 16 == 0) printf("lane %2d item %d: %.0f\n", l, q, v);
    }
  printf("mismatches vs D[4(l/16)+q][l%%16]: %d\n", bad);
  return 0;
}
