// Operand / result lane layout of v_mfma_f64_4x4x4f64 (4 blocks of 4x4x4)
// on gfx950: wave p sets A = one-hot at lane p and B[l] = l + 1; every
// nonzero D lane d then holds B of the lane supplying B_b[k][j] for the
// (block, row) of A lane p.  Prints, per A lane: D lanes <- B lanes.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double *out) {
  const int l = threadIdx.x, p = blockIdx.x;
  const double a = l == p ? 1.0 : 0.0, b = l + 1;
  double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  out[p * 64 + l] = d;
}
int main() {
  double *o;
  (void)hipMalloc(&o, 64 * 64 * 8);
  k<<<64, 64>>>(o);
  double h[64 * 64];
  (void)hipMemcpy(h, o, sizeof h, hipMemcpyDeviceToHost);
  for (int p = 0; p < 64; ++p) {
    printf("A lane %2d:", p);
    for (int d = 0; d < 64; ++d)
      if (h[p * 64 + d] != 0) printf(" D%d<-B%d", d, (int)h[p * 64 + d] - 1);
    printf("\n");
  }
  return 0;
}
