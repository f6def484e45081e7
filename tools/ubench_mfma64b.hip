// Micro-benchmark (sustained, ~tens of ms per case): fp64 MFMA issue rate on
// gfx950 as a function of the A operand's contents and of the shape.
//  - 16x16x4 with random A in every row, with rows 9..15 a copy of row 8 (K1's
//    padding today), with rows 9..15 zero, and all-zero A;
//  - v_mfma_f64_4x4x4_4b (4 blocks of 4x4x4).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_mfma64b tools/ubench_mfma64b.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

// AMODE 0: random A; 1: rows >= 9 copy row 8; 2: rows >= 9 zero; 3: all zero
template <int AMODE>
__global__ __launch_bounds__(256) void k16(double *out, int iters, double seed) {
  const int lane = threadIdx.x & 63, row = lane & 15;
  d4 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = d4{0, 0, 0, 0};
  // pseudo-random operands (distinct per lane and per step) so nothing folds
  double a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = AMODE == 1 && row >= 9 ? 8 : row;
    a[i] = sin(seed * (r + 1) + 0.37 * i + (lane >> 4));
    if (AMODE == 2 && row >= 9) a[i] = 0.0;
    if (AMODE == 3) a[i] = 0.0;
    b[i] = cos(seed * (lane + 3) + 0.71 * i);
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[i], acc[i & 3], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < 4; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k4(double *out, int iters, double seed) {
  const int lane = threadIdx.x & 63;
  double acc[4] = {0, 0, 0, 0};
  double a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = sin(seed * (lane + 1) + 0.37 * i);
    b[i] = cos(seed * (lane + 3) + 0.71 * i);
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i & 3] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[i], b[i], acc[i & 3], 0, 0, 0);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

template <typename K>
void run(const char *name, K kern, double flops_per_mfma, double *out) {
  const int blocks = 1024, threads = 256, iters = 2048;  // 4 waves / SIMD
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  kern<<<blocks, threads>>>(out, iters, 0.123);
  float best = 1e30f, tot = 0;
  const int reps = 20;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(e0);
    kern<<<blocks, threads>>>(out, iters, 0.123 + r);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
    tot += ms;
  }
  const double n_mfma = (double)blocks * (threads / 64) * iters * 8;
  const double avg = tot / reps;
  printf("%-34s avg %.3f ms best %.3f ms  %.1f TFLOP/s  %.1f cyc/mfma/SIMD @2.4GHz\n", name, avg, best,
         n_mfma * flops_per_mfma / (avg * 1e-3) / 1e12, avg * 1e-3 * 2.4e9 / (n_mfma / 1024.0));
}

int main() {
  double *out;
  hipMalloc(&out, 1 << 24);
  const double f16 = 2.0 * 16 * 16 * 4, f4 = 2.0 * 4 * 4 * 4 * 4;
  for (int pass = 0; pass < 2; ++pass) {
    run("16x16x4 random A", k16<0>, f16, out);
    run("16x16x4 rows 9-15 = row 8", k16<1>, f16, out);
    run("16x16x4 rows 9-15 zero", k16<2>, f16, out);
    run("16x16x4 A all zero", k16<3>, f16, out);
    run("4x4x4_4b random", k4, f4, out);
  }
  hipFree(out);
  return 0;
}
