// Checks the lane semantics the time-major K1 relies on (gfx950):
//   permlane32_swap(vdst, src): lanes 32-63 of vdst <-> lanes 0-31 of src
//   permlane16_swap(vdst, src): odd 16-lane rows of vdst <-> even rows of src
// P holds rows {0, 1} x 32 channels (lane l: row l/32, ch l%32), Q rows {2, 3};
// after both swaps lane 16k + c must hold (row k, ch c) in P and (row k,
// ch 16 + c) in Q.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *out) {
  const unsigned l = threadIdx.x;
  unsigned p = (l / 32) * 100 + l % 32, q = (2 + l / 32) * 100 + l % 32;
  auto r = __builtin_amdgcn_permlane32_swap(p, q, false, false);
  auto s = __builtin_amdgcn_permlane16_swap(r[0], r[1], false, false);
  out[l] = s[0];
  out[64 + l] = s[1];
}
int main() {
  unsigned *d, h[128];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
  k<<<1, 64>>>(d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    const unsigned row = l / 16, c = l % 16;
    bad += h[l] != row * 100 + c;
    bad += h[64 + l] != row * 100 + 16 + c;
  }
  printf("permlane layout %s (%d mismatches)\n", bad ? "WRONG" : "ok", bad);
  return bad ? 1 : 0;
}
