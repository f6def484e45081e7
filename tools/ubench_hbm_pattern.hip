// Micro-benchmark: achievable HBM read rate of the access patterns a
// block-functional kernel can use on a (channel, time) float32 array of
// 10,000 x 1.8 M samples (cfg3, 72 GB).  Each wave-instruction loads 1 KB as
// R rows x (1024/R) contiguous bytes; a wave owns 16 channel rows (R = 16, 4)
// or 1 row (R = 1) and walks them in time, PF instructions in flight.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_hbm_pattern tools/ubench_hbm_pattern.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int64_t NCH = 10000, NT = 1800000;

// R rows per instruction, rows of a wave = 16 channels (R < 16 cycles rows)
template <int R>
__global__ __launch_bounds__(256) void k_pattern(const float *__restrict__ x, float *out,
                                                 int64_t span /* samples per unit */) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t unit = (int64_t)blockIdx.x * 4 + wave;
  constexpr int SEG = 256 / R;  // floats per row piece... (1024 B / R) / 4
  const int64_t n_cg = (R == 1) ? NCH : NCH / 16;
  const int64_t runs = NT / span;
  if (unit >= n_cg * runs) return;
  const int64_t cg = unit % n_cg, run = unit / n_cg;
  const int row_in = lane / (SEG / 4);       // 0..R-1
  const int off_in = (lane % (SEG / 4)) * 4;  // float offset in the piece
  float acc = 0.f;
  if (R == 1) {
    const float *p = x + cg * NT + run * span + off_in;
    for (int64_t t = 0; t < span; t += 8 * 256) {
      f4v v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const f4v *>(p + t + 256 * j);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += v[j].x + v[j].y + v[j].z + v[j].w;
    }
  } else {
    // 16 rows; instruction i of a step covers rows (i*R .. i*R+R-1)
    constexpr int NI = 16 / R;  // instructions per step (16 rows x SEG floats)
    const float *p[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) p[i] = x + (cg * 16 + i * R + row_in) * NT + run * span + off_in;
    for (int64_t t = 0; t < span; t += 2 * SEG) {
      f4v v[2 * NI];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < NI; ++i) v[u * NI + i] = *reinterpret_cast<const f4v *>(p[i] + t + u * SEG);
#pragma unroll
      for (int j = 0; j < 2 * NI; ++j) acc += v[j].x + v[j].y + v[j].z + v[j].w;
    }
  }
  if (acc == 1234.5f) out[unit] = acc;
}

// K1's per-block rows: block k of a unit reads 8 x 64 samples from
// floor4(k*L - 4), i.e. 512 samples per 500-sample block (12 re-read), as
// 16 rows x 64 B per instruction; OVL = 0 reads the same rows back to back
// without the overlap (512-sample blocks) for comparison.
template <int OVL>
__global__ __launch_bounds__(256) void k_blockrows(const float *__restrict__ x, float *out, int bpu) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t unit = (int64_t)blockIdx.x * 4 + wave;
  const int L = OVL ? 500 : 512;
  const int64_t nb = (NT - 16) / L;
  const int64_t n_cg = NCH / 16, runs = nb / bpu;
  if (unit >= n_cg * runs) return;
  const int64_t cg = unit % n_cg, run = unit / n_cg;
  const int col = lane & 15, q = lane >> 4;
  const float *xr = x + (cg * 16 + col) * NT + 4 * q;
  float acc = 0.f;
  for (int64_t k = run * bpu; k < (run + 1) * bpu; ++k) {
    const int64_t a = OVL ? (k * L) & ~(int64_t)3 : k * L;
    f4v v[8][4];
#pragma unroll
    for (int it = 0; it < 8; ++it)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[it][j] = *reinterpret_cast<const f4v *>(xr + a + 64 * it + 16 * j);
#pragma unroll
    for (int it = 0; it < 8; ++it)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc += v[it][j].x + v[it][j].y + v[it][j].z + v[it][j].w;
  }
  if (acc == 1234.5f) out[unit] = acc;
}

template <int OVL>
void run_blockrows(const float *x, float *out, const char *name) {
  const int bpu = 32;
  const int L = OVL ? 500 : 512;
  const int64_t nb = (NT - 16) / L;
  const int64_t units = (NCH / 16) * (nb / bpu);
  const unsigned grid = (unsigned)((units + 3) / 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k_blockrows<OVL><<<grid, 256>>>(x, out, bpu);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) k_blockrows<OVL><<<grid, 256>>>(x, out, bpu);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 3;
  const double alg = (double)NCH * (double)(nb / bpu * bpu) * L * 4.0;  // distinct bytes
  printf("%-34s %7.3f ms  %6.2f TB/s of distinct bytes (%.2f GB)\n", name, ms, alg / (ms * 1e-3) / 1e12, alg / 1e9);
}

__global__ void k_fill(float *x, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 13);
    h ^= h >> 15;
    h *= 2246822519u;
    x[i] = (float)(h & 0xffffff) * (1.0f / 16777216.0f) - 0.5f;
  }
}

// calibration store: one double per lane (64 lanes x 8 B = 512 B contiguous)
__global__ void k_store8(double *y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = (double)i;
}

template <int R>
void run(const float *x, float *out, int64_t span, const char *name, size_t lds = 0) {
  const int64_t n_cg = (R == 1) ? NCH : NCH / 16;
  const int64_t units = n_cg * (NT / span);
  const unsigned grid = (unsigned)((units + 3) / 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k_pattern<R><<<grid, 256, lds>>>(x, out, span);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) k_pattern<R><<<grid, 256, lds>>>(x, out, span);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 3;
  const double bytes = (double)NCH * (double)(NT / span * span) * 4.0;
  printf("%-34s span %7lld lds %6zu: %7.3f ms  %6.2f TB/s\n", name, (long long)span, lds, ms,
         bytes / (ms * 1e-3) / 1e12);
}

int main() {
  float *x, *out;
  if (hipMalloc(&x, sizeof(float) * NCH * NT) != hipSuccess) return 1;
  if (hipMalloc(&out, 1 << 24) != hipSuccess) return 1;
  (void)hipMemset(x, 0, sizeof(float) * NCH * NT);
  (void)hipDeviceSynchronize();
  run<1>(x, out, 18000, "zeros: 1 row x 1 KB");
  run<16>(x, out, 16000, "zeros: 16 rows x 64 B");
  k_fill<<<8192, 256>>>(x, NCH * NT);
  (void)hipDeviceSynchronize();
  run<1>(x, out, 18000, "rand: 1 row x 1 KB");
  run<4>(x, out, 16000, "rand: 4 rows x 256 B");
  run<16>(x, out, 16000, "rand: 16 rows x 64 B");
  run<1>(x, out, 18000, "rand: 1 row x 1 KB", 37 * 1024);
  run<16>(x, out, 16000, "rand: 16 rows x 64 B", 37 * 1024);
  run<16>(x, out, 16000, "rand: 16 rows x 64 B", 70 * 1024);
  run_blockrows<1>(x, out, "blockrows L=500 (512-sample rows)");
  run_blockrows<0>(x, out, "blockrows L=512 (no overlap)");
  // known-size store for WRITE_SIZE calibration: 360 M doubles = 2.88 GB
  k_store8<<<8192, 256>>>(reinterpret_cast<double *>(x), 360000000LL);
  (void)hipDeviceSynchronize();
  printf("k_store8: %lld bytes\n", 360000000LL * 8);
  (void)hipFree(x);
  (void)hipFree(out);
  return 0;
}
