// Micro-benchmark: HBM read rate of (time, channel) float32 storage
// (cfg3 stored time-major: 1.8 M rows x 10,000 channels, 72 GB) streamed by
// waves that own CW consecutive channels and walk 64-row iterations in time,
// for the wave shapes a time-major K1 can use.  VB bytes per lane per load
// (8: two channels, 16: four): one wave-instruction reads (64 VB / (4 CW))
// rows x 4 CW bytes.  WPG waves per workgroup; `lds_kb` of dummy LDS per
// workgroup caps the waves per CU.  Every pattern sums its loads (result
// discarded), so only the load stream is timed.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_tm tools/ubench_tm.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int64_t NCH = 10000, NT = 1800000;
constexpr int64_t SPAN = 16000;  // rows per unit (32 blocks of 500)

template <int CW, int VB, int PF>
__global__ __launch_bounds__(512) void k_tm(const float *__restrict__ x, float *out) {
  extern __shared__ float dummy[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t unit = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  const int64_t n_strip = (NCH + CW - 1) / CW;
  const int64_t n_grp = NT / SPAN;
  if (unit >= n_strip * n_grp) return;
  const int64_t strip = unit % n_strip, grp = unit / n_strip;
  constexpr int LPR = CW * 4 / VB;     // lanes per row
  constexpr int RPI = 64 / LPR;        // rows per instruction
  constexpr int NI = 64 / RPI;         // instructions per 64-row iteration
  const int r_in = lane / LPR;
  int64_t c = strip * CW + (lane % LPR) * (VB / 4);
  if (c > NCH - VB / 4) c = NCH - VB / 4;
  const float *base = x + (grp * SPAN + r_in) * NCH + c;
  float acc = 0.f;
  typedef float fv __attribute__((ext_vector_type(VB / 4)));
  fv buf[PF + 1][NI];
  int64_t row = 0;
#pragma unroll
  for (int d = 0; d < PF; ++d) {
#pragma unroll
    for (int i = 0; i < NI; ++i) buf[d][i] = *reinterpret_cast<const fv *>(base + (row + i * RPI) * NCH);
    row += 64;
  }
  for (int64_t it = 0; it < SPAN / 64; it += PF + 1) {
#pragma unroll
    for (int u = 0; u <= PF; ++u) {
      const int lb = (u + PF) % (PF + 1);
      const int64_t rr = row < SPAN ? row : SPAN - 64;
#pragma unroll
      for (int i = 0; i < NI; ++i) buf[lb][i] = *reinterpret_cast<const fv *>(base + (rr + i * RPI) * NCH);
      row += 64;
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int e = 0; e < VB / 4; ++e) acc += buf[u][i][e];
    }
  }
  if (acc == 1234.5f) out[unit] = acc + dummy[0];
}

template <int CW, int VB, int PF>
void run(const float *x, float *out, int wpg, int lds_kb, const char *name) {
  const int64_t units = ((NCH + CW - 1) / CW) * (NT / SPAN);
  const unsigned grid = (unsigned)((units + wpg - 1) / wpg);
  const size_t lds = (size_t)lds_kb * 1024;
  hipFuncSetAttribute(reinterpret_cast<const void *>(&k_tm<CW, VB, PF>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      160 * 1024);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k_tm<CW, VB, PF><<<grid, 64 * wpg, lds>>>(x, out);
  hipEventRecord(a);
  for (int r = 0; r < 3; ++r) k_tm<CW, VB, PF><<<grid, 64 * wpg, lds>>>(x, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  ms /= 3;
  const double bytes = (double)NCH * (double)(NT / SPAN * SPAN) * 4.0;
  printf("%-28s CW %3d VB %2d PF %d waves/WG %2d lds %3d KB: %7.3f ms  %6.3f TB/s  frac %.3f\n", name, CW, VB, PF, wpg,
         lds_kb, ms, bytes / ms / 1e9, bytes / ms / 1e9 / 8000.0);
}

int main() {
  float *x, *out;
  const size_t n = (size_t)NCH * NT;
  if (hipMalloc(&x, n * 4) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 2;
  hipMemset(x, 0, n * 4);
  hipDeviceSynchronize();
  run<32, 8, 1>(x, out, 8, 117, "K1-tm now (8 waves/CU)");
  run<32, 8, 1>(x, out, 8, 40, "CW32 VB8 16 waves/CU");
  run<32, 8, 2>(x, out, 8, 40, "CW32 VB8 PF2 16 w/CU");
  run<64, 16, 1>(x, out, 8, 117, "CW64 VB16 8 w/CU");
  run<64, 16, 1>(x, out, 8, 40, "CW64 VB16 16 w/CU");
  run<64, 8, 1>(x, out, 8, 40, "CW64 VB8 (2 rows/instr)");
  run<128, 16, 1>(x, out, 8, 40, "CW128 VB16 16 w/CU");
  run<256, 16, 1>(x, out, 8, 40, "CW256 VB16 16 w/CU");
  run<64, 16, 1>(x, out, 4, 20, "CW64 VB16 wg4 16 w/CU");
  run<32, 8, 1>(x, out, 8, 117, "K1-tm now (again)");
  return 0;
}
