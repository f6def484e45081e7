// Micro-benchmark: plain register loads vs LDS-DMA (global_load_lds_dwordx4,
// default and nt policy) streaming a (channel, time) float32 array of
// 10,000 x 1.8 M samples (cfg3, 72 GB).  A wave owns 16 channel rows and walks
// them in time; each wave-instruction moves 1 KB as R rows x (1024/R) bytes.
// LDS-DMA variants keep D one-KB slots per wave in flight (lane-linear LDS
// image) and consume a slot with one ds_read_b128 per lane after a counted
// vmcnt.  Extra dynamic LDS caps the waves per CU.  Every variant returns the
// same checksum (sum of all samples) so a wrong DMA/wait shows up.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_glds tools/ubench_glds.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int64_t NCH = 10000, NT = 1800000;

// source address of instruction n of a unit (16 rows from row0, time from t0)
template <int R>
__device__ __forceinline__ const float *src_of(const float *x, int64_t row0, int64_t t0, int64_t n,
                                               int lane) {
  constexpr int G = 16 / R;          // row groups
  constexpr int SEG = 256 / R;       // floats per row piece
  constexpr int LPR = 64 / R;        // lanes per row
  const int64_t grp = n % G, ts = n / G;
  const int64_t row = row0 + grp * R + lane / LPR;
  return x + row * NT + t0 + ts * SEG + (lane % LPR) * 4;
}

template <int AUX>
__device__ __forceinline__ void glds16(const float *g, uint32_t lds_byte) {
  unsigned keep;
  if constexpr (AUX == 0)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds_byte) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds_byte) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// MODE 0: register loads (PF instructions ahead); 1: LDS-DMA ring of D slots
template <int R, int MODE, int AUX, int D>
__global__ __launch_bounds__(256) void k_stream(const float *__restrict__ x, double *out,
                                                int64_t span) {
  extern __shared__ f4v lds[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t unit = (int64_t)blockIdx.x * 4 + wave;
  const int64_t n_cg = NCH / 16, runs = NT / span;
  if (unit >= n_cg * runs) return;
  const int64_t cg = unit % n_cg, run = unit / n_cg;
  const int64_t row0 = cg * 16, t0 = run * span;
  const int64_t n_ins = 16 * span / 256;  // 1-KB instructions per unit
  float acc = 0.f;
  if constexpr (MODE == 0) {
    f4v v[D];
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = *reinterpret_cast<const f4v *>(src_of<R>(x, row0, t0, d, lane));
    for (int64_t n = 0; n < n_ins; n += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const f4v c = v[d];
        const int64_t nn = n + D + d < n_ins ? n + D + d : n_ins - 1;
        v[d] = *reinterpret_cast<const f4v *>(src_of<R>(x, row0, t0, nn, lane));
        acc += c.x + c.y + c.z + c.w;
      }
    }
  } else {
    f4v *ring = lds + wave * D * 64;  // D slots of 64 lanes x 16 B
    const uint32_t rb = (uint32_t)(uintptr_t)ring;
#pragma unroll
    for (int d = 0; d < D; ++d) glds16<AUX>(src_of<R>(x, row0, t0, d, lane), rb + d * 1024);
    // n_ins is a multiple of D at the spans used (checked on the host)
    for (int64_t n = 0; n < n_ins; n += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        wait_vm<D - 1>();
        const f4v c = ring[d * 64 + lane];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int64_t nn = n + D + d < n_ins ? n + D + d : n_ins - 1;
        glds16<AUX>(src_of<R>(x, row0, t0, nn, lane), rb + d * 1024);
        acc += c.x + c.y + c.z + c.w;
      }
    }
    wait_vm<0>();
  }
  // checksum: one atomic per wave (only the first n_ins loads count; the
  // clamped re-loads past the end are discarded by the loop structure)
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) atomicAdd(out, (double)acc);
}

__global__ void k_fill(float *x, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 13);
    h ^= h >> 15;
    h *= 2246822519u;
    x[i] = (float)(h & 0xffff) * (1.0f / 65536.0f);
  }
}

template <int R, int MODE, int AUX, int D>
void run(const float *x, double *out, int64_t span, const char *name, size_t extra_lds) {
  const int64_t units = (NCH / 16) * (NT / span);
  if ((16 * span / 256) % D) { printf("bad span\n"); return; }
  const unsigned grid = (unsigned)((units + 3) / 4);
  const size_t lds = (MODE ? 4 * D * 1024 : 0) + extra_lds;
  auto fn = reinterpret_cast<const void *>(&k_stream<R, MODE, AUX, D>);
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipMemset(out, 0, 8);
  k_stream<R, MODE, AUX, D><<<grid, 256, lds>>>(x, out, span);
  double chk = 0;
  (void)hipMemcpy(&chk, out, 8, hipMemcpyDeviceToHost);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) k_stream<R, MODE, AUX, D><<<grid, 256, lds>>>(x, out, span);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 3;
  const double bytes = (double)NCH * (double)(NT / span * span) * 4.0;
  printf("%-40s lds/WG %6zu: %7.3f ms  %6.2f TB/s  chk %.6e\n", name, lds, ms,
         bytes / (ms * 1e-3) / 1e12, chk);
}

int main() {
  float *x;
  double *out;
  if (hipMalloc(&x, sizeof(float) * NCH * NT) != hipSuccess) return 1;
  if (hipMalloc(&out, 64) != hipSuccess) return 1;
  k_fill<<<8192, 256>>>(x, NCH * NT);
  (void)hipDeviceSynchronize();
  const int64_t S = 16000;  // 1000 instructions per unit
  // 16 waves per CU = 4 WGs of 256: LDS per WG <= 40 KB
  run<16, 0, 0, 8>(x, out, S, "reg 16x64B PF8", 0);
  run<4, 0, 0, 8>(x, out, S, "reg 4x256B PF8", 0);
  run<16, 1, 0, 8>(x, out, S, "glds 16x64B D8", 0);
  run<16, 1, 1, 8>(x, out, S, "glds nt 16x64B D8", 0);
  run<4, 1, 0, 8>(x, out, S, "glds 4x256B D8", 0);
  run<4, 1, 1, 8>(x, out, S, "glds nt 4x256B D8", 0);
  run<1, 1, 1, 8>(x, out, S, "glds nt 1x1KB D8", 0);
  run<4, 1, 1, 4>(x, out, S, "glds nt 4x256B D4", 0);
  run<4, 1, 1, 4>(x, out, S, "glds nt 4x256B D4 (8 waves/CU)", 60 * 1024);
  run<4, 1, 1, 8>(x, out, S, "glds nt 4x256B D8 (8 waves/CU)", 50 * 1024);
  run<4, 1, 1, 10>(x, out, S, "glds nt 4x256B D10 (8 waves/CU)", 40 * 1024);
  run<4, 1, 0, 8>(x, out, S, "glds 4x256B D8 (8 waves/CU)", 50 * 1024);
  run<16, 0, 0, 8>(x, out, S, "reg 16x64B PF8 (8 waves/CU)", 70 * 1024);
  (void)hipFree(x);
  (void)hipFree(out);
  return 0;
}
