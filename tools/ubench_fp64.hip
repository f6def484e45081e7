// Micro-benchmark: fp64 / fp32 FMA dependent latency and throughput on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
template <typename T, int CH>
__global__ void k_fma(T *out, T a, T b, int iters) {
  T x[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = (T)(threadIdx.x + c);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = fma(x[c], a, b);
  }
  T s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <typename T, int CH>
void run(const char *name, int blocks, int threads, int iters) {
  T *o;
  hipMalloc(&o, sizeof(T) * blocks * threads);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  k_fma<T, CH><<<blocks, threads>>>(o, (T)0.999, (T)0.001, 10);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  k_fma<T, CH><<<blocks, threads>>>(o, (T)0.999, (T)0.001, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double fmas = (double)blocks * threads * iters * CH;
  int waves_per_simd = (blocks * threads / 64 + 1023) / 1024;
  printf("%-8s chains=%2d blocks=%6d threads=%4d : %8.3f ms  %8.2f TFMA/s  cycles/FMA/wave(@2.4GHz, %d waves/SIMD)=%.2f\n",
         name, CH, blocks, threads, ms, fmas / ms / 1e9, waves_per_simd,
         ms * 1e-3 * 2.4e9 / ((double)iters * CH) );
  hipFree(o);
}
int main() {
  // latency: 1 wave per SIMD, 1 chain
  run<double, 1>("f64", 256, 256, 1 << 20);
  run<double, 4>("f64", 256, 256, 1 << 18);
  run<double, 8>("f64", 256, 256, 1 << 17);
  // throughput: 8 waves per SIMD
  run<double, 1>("f64", 2048, 256, 1 << 18);
  run<double, 4>("f64", 2048, 256, 1 << 16);
  run<double, 8>("f64", 2048, 256, 1 << 15);
  run<float, 1>("f32", 256, 256, 1 << 20);
  run<float, 8>("f32", 256, 256, 1 << 17);
  run<float, 8>("f32", 2048, 256, 1 << 15);
  return 0;
}
