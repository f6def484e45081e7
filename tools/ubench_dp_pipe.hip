// Micro-benchmark: do fp64 MFMAs and VALU instructions of OTHER waves on the
// same SIMD overlap on gfx950, or do they share one issue pipe?
// A 512-thread workgroup = 8 waves, wave w on SIMD w % 4: waves 0-3 run an
// MFMA loop, waves 4-7 a VALU loop (one of each per SIMD).  Timed three ways:
// MFMA waves only (VALU waves exit at once), VALU waves only, both.  If the
// pipes overlap, both ~ max(MFMA, VALU); if they share the issue, ~ sum.
// Also MFMA and VALU interleaved in one wave (independent chains).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_dp_pipe tools/ubench_dp_pipe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

// VALU kinds: 0 f64 fma, 1 f32 fma, 2 u32 add, 3 f32 -> f64 cvt, 4 f64 dpp mov (2 x v_mov_b32_dpp)
template <int VK>
__device__ __forceinline__ void valu8(double (&x)[8], float (&f)[8], unsigned (&u)[8], double a, double b) {
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    if (VK == 0) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x[c]) : "v"(a), "v"(b));
    if (VK == 1) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[c]) : "v"((float)a), "v"((float)b));
    if (VK == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[c]) : "v"(c + 1));
    if (VK == 3) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(x[c]) : "v"(f[c]));
    if (VK == 4) {
      asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(u[c]));
      asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(f[c]));
    }
  }
}

// MFMA kinds: 0 f64 16x16x4 (4 chains), 1 f64 4x4x4_4b (4 chains), 2 f32 16x16x4f32, 3 bf16 16x16x32
template <int MK>
__device__ __forceinline__ void mfma4(d4 (&acc)[4], f4 (&accf)[4], double (&acc1)[4], double a, double b) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (MK == 0) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
    if (MK == 1) acc1[c] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc1[c], 0, 0, 0);
    if (MK == 2) accf[c] = __builtin_amdgcn_mfma_f32_16x16x4f32((float)a, (float)b, accf[c], 0, 0, 0);
    if (MK == 3) {
      bf8 av, bv;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        av[i] = (__bf16)(float)a;
        bv[i] = (__bf16)(float)b;
      }
      accf[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, accf[c], 0, 0, 0);
    }
  }
}

// mode 1: MFMA waves only; 2: VALU waves only; 3: both (separate waves);
// 4: MFMA + VALU interleaved inside every wave (all 8 waves)
template <int MK, int VK>
__global__ __launch_bounds__(512) void k_mix(double *out, int mode, int nm, int nv) {
  const int w = threadIdx.x >> 6;
  d4 acc[4];
  f4 accf[4];
  double acc1[4];
  double x[8];
  float f[8];
  unsigned u[8];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    acc[c] = d4{0, 0, 0, 0};
    accf[c] = f4{0, 0, 0, 0};
    acc1[c] = 0;
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    x[c] = threadIdx.x + c;
    f[c] = (float)x[c];
    u[c] = threadIdx.x + c;
  }
  const double a = 0.999 + threadIdx.x * 1e-9, b = 1e-3;
  const bool mw = w < 4;
  if (mode == 4) {
    for (int i = 0; i < nm; ++i) {
      mfma4<MK>(acc, accf, acc1, a, b);
      for (int j = 0; j < nv / nm; ++j) valu8<VK>(x, f, u, a, b);
    }
  } else if (mw && (mode == 1 || mode == 3)) {
    for (int i = 0; i < nm; ++i) mfma4<MK>(acc, accf, acc1, a, b);
  } else if (!mw && (mode == 2 || mode == 3)) {
    for (int i = 0; i < nv; ++i) valu8<VK>(x, f, u, a, b);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < 4; ++c) s += acc[c][0] + accf[c][0] + acc1[c];
#pragma unroll
  for (int c = 0; c < 8; ++c) s += x[c] + f[c] + u[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MK, int VK>
void run(const char *mk, const char *vk, int blocks, int nm, int nv, double *out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float t[5] = {0};
  for (int mode = 1; mode <= 4; ++mode) {
    k_mix<MK, VK><<<blocks, 512>>>(out, mode, nm, nv);  // warm
    hipEventRecord(e0);
    k_mix<MK, VK><<<blocks, 512>>>(out, mode, nm, nv);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&t[mode], e0, e1);
  }
  printf("%-14s + %-10s blocks=%4d: mfma %.3f ms, valu %.3f ms, both(separate waves) %.3f ms = %.2f x sum, %.2f x max;"
         " interleaved %.3f ms\n",
         mk, vk, blocks, t[1], t[2], t[3], t[3] / (t[1] + t[2]), t[3] / (t[1] > t[2] ? t[1] : t[2]), t[4]);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  double *out;
  hipMalloc(&out, sizeof(double) * 2048 * 512);
  for (int blocks : {256, 512}) {
    // iteration counts chosen so the MFMA-only and VALU-only times are similar
    run<0, 0>("f64 16x16x4", "f64 fma", blocks, 4096, 8192, out);
    run<0, 1>("f64 16x16x4", "f32 fma", blocks, 4096, 8192, out);
    run<0, 2>("f64 16x16x4", "u32 add", blocks, 4096, 8192, out);
    run<0, 3>("f64 16x16x4", "cvt f64", blocks, 4096, 8192, out);
    run<0, 4>("f64 16x16x4", "dpp mov", blocks, 4096, 4096, out);
    run<1, 0>("f64 4x4x4_4b", "f64 fma", blocks, 16384, 8192, out);
    run<1, 2>("f64 4x4x4_4b", "u32 add", blocks, 16384, 8192, out);
    run<2, 0>("f32 16x16x4", "f64 fma", blocks, 4096, 8192, out);
    run<3, 0>("bf16 16x16x32", "f64 fma", blocks, 4096, 8192, out);
    run<3, 2>("bf16 16x16x32", "u32 add", blocks, 4096, 8192, out);
  }
  hipFree(out);
  return 0;
}
