// Micro-benchmark: v_mfma_f64_16x16x4_f64 issue rate and dependent latency on
// gfx950 (the block-functional GEMM formulation of K1 runs on it).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_mfma64 tools/ubench_mfma64.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int CHAINS>
__global__ void k_mfma(double *out, int iters, double a0, double b0) {
  d4 acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = d4{0, 0, 0, 0};
  double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CHAINS>
void run(int blocks, int wpb, double *out) {
  const int iters = 4096;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_mfma<CHAINS><<<blocks, 64 * wpb>>>(out, iters, 1.0, 1.0);
  hipEventRecord(e0);
  k_mfma<CHAINS><<<blocks, 64 * wpb>>>(out, iters, 1.0, 1.0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double n_mfma = (double)blocks * wpb * iters * CHAINS;
  const double tflops = n_mfma * 2.0 * 16 * 16 * 4 / (ms * 1e-3) / 1e12;
  // cycles per MFMA per SIMD at 2.4 GHz (waves spread over 1024 SIMDs)
  const double per_simd = n_mfma / 1024.0;
  printf("chains=%d blocks=%d waves/blk=%d: %.3f ms  %.1f TFLOP/s  %.1f cyc/mfma/SIMD\n", CHAINS,
         blocks, wpb, ms, tflops, ms * 1e-3 * 2.4e9 / per_simd);
}

int main() {
  double *out;
  hipMalloc(&out, 1 << 24);
  run<1>(256, 4, out);   // 1 wave / SIMD, 1 chain: dependent latency
  run<2>(256, 4, out);
  run<4>(256, 4, out);
  run<1>(512, 4, out);   // 2 waves / SIMD
  run<2>(512, 4, out);
  run<1>(1024, 4, out);  // 4 waves / SIMD
  run<4>(1024, 4, out);
  hipFree(out);
  return 0;
}
