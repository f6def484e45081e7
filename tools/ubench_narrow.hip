// Micro-benchmark: K1's sample stream (16 channel rows x 64 B per wave
// instruction, 8 x 64-sample iterations per 500-sample block, bpu blocks per
// wave unit, channel-group-fastest unit order) over a (channel, time) float32
// array of nch x 1.8 M samples, alone — no MFMA, no tap table, no epilogue.
// The rows are rows [off, off + nch) of an allocation of alloc_ch rows, so a
// narrow shard can be streamed from its own allocation or from inside a wide
// one (placement vs width).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_narrow tools/ubench_narrow.hip
// Run:   tools/ubench_narrow <nch> <alloc_ch> <off> <bpu> [order] [shape]
// shape 0: K1's 16 rows x 64 B per wave instruction; shape 1: 8 rows x 128 B
// (whole lines: lanes 8i..8i+7 read one row's 128 B; the same 16 rows x 256 B
// per 64-sample iteration in 4 instructions)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int64_t NT = 1800000;
constexpr int L = 500;

// order 0: unit = cg + n_cg * time group (K1's); 1: unit = time group + n_tg * cg
template <int SHAPE>
__global__ __launch_bounds__(512) void k_rows(const float *__restrict__ x, float *out, int64_t nch, int bpu,
                                              int order) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t unit = (int64_t)blockIdx.x * 8 + wave;
  const int64_t nb = (NT - 16) / L;
  const int64_t n_cg = nch / 16, n_tg = nb / bpu;
  if (unit >= n_cg * n_tg) return;
  const int64_t cg = order ? unit / n_tg : unit % n_cg, tg = order ? unit % n_tg : unit / n_cg;
  const int col = lane & 15, q = lane >> 4;
  const float *xr = x + (cg * 16 + col) * NT + 4 * q;
  // shape 1: rows lane / 8 (instructions 0, 2) and 8 + lane / 8 (1, 3), piece lane % 8
  const float *xa = x + (cg * 16 + (lane >> 3)) * NT + 4 * (lane & 7);
  const float *xb = xa + 8 * NT;
  float acc = 0.f;
  f4v v[2][4];
  int64_t k = tg * bpu, it = 0;
  auto ld = [&](f4v (&b)[4], int64_t kk, int64_t ii) {
    const int64_t a = (kk * L) & ~(int64_t)3;
    if (SHAPE == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const f4v *>(xr + a + 64 * ii + 16 * j);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = *reinterpret_cast<const f4v *>((j & 1 ? xb : xa) + a + 64 * ii + 32 * (j >> 1));
    }
  };
  ld(v[0], k, 0);
  const int64_t n_it = (int64_t)bpu * 8;
  for (int64_t i = 0; i < n_it; i += 2) {
    const int64_t i1 = i + 1 < n_it ? i + 1 : i;
    ld(v[1], tg * bpu + i1 / 8, i1 % 8);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc += v[0][j].x + v[0][j].y + v[0][j].z + v[0][j].w;
    const int64_t i2 = i + 2 < n_it ? i + 2 : i1;
    ld(v[0], tg * bpu + i2 / 8, i2 % 8);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc += v[1][j].x + v[1][j].y + v[1][j].z + v[1][j].w;
  }
  (void)it;
  if (acc == 1234.5f) out[unit] = acc;
}

__global__ void k_fill(float *x, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 13);
    h ^= h >> 15;
    h *= 2246822519u;
    x[i] = (float)(h & 0xffffff) * (1.0f / 16777216.0f) - 0.5f;
  }
}

int main(int argc, char **argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s nch alloc_ch off bpu [order]\n", argv[0]);
    return 2;
  }
  const int64_t nch = atoll(argv[1]), alloc_ch = atoll(argv[2]), off = atoll(argv[3]);
  const int bpu = atoi(argv[4]), order = argc > 5 ? atoi(argv[5]) : 0, shape = argc > 6 ? atoi(argv[6]) : 0;
  if (nch % 16 || off + nch > alloc_ch || bpu < 1) return 2;
  float *x, *out;
  if (hipMalloc(&x, sizeof(float) * alloc_ch * NT) != hipSuccess) return 1;
  if (hipMalloc(&out, 1 << 24) != hipSuccess) return 1;
  k_fill<<<8192, 256>>>(x, alloc_ch * NT);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  const float *xs = x + off * NT;
  const int64_t nb = (NT - 16) / L;
  const int64_t units = (nch / 16) * (nb / bpu);
  const unsigned grid = (unsigned)((units + 7) / 8);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto launch = [&]() {
    if (shape)
      k_rows<1><<<grid, 512>>>(xs, out, nch, bpu, order);
    else
      k_rows<0><<<grid, 512>>>(xs, out, nch, bpu, order);
  };
  launch();
  float best = 1e30f, sum = 0.f;
  const int reps = 5;
  for (int r = 0; r < reps; ++r) {
    (void)hipEventRecord(e0);
    launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
    sum += ms;
  }
  const double bytes = (double)nch * (double)(nb / bpu * bpu) * L * 4.0;
  printf("shape %d nch %6lld alloc %6lld off %6lld bpu %3d order %d: mean %.3f ms min %.3f ms  %.2f TB/s (%.3f of 8)\n",
         shape, (long long)nch, (long long)alloc_ch, (long long)off, bpu, order, sum / reps, best,
         bytes / (sum / reps * 1e-3) / 1e12, bytes / (sum / reps * 1e-3) / 8e12);
  (void)hipFree(x);
  (void)hipFree(out);
  return 0;
}
