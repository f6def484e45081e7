// gfx950 (MI355X / CDNA4) kernels of the low-frequency DAS hot path.
//
//   k_block_functionals_lds — the HBM-streaming kernel for time-contiguous
//        rows: every input sample is read once (coalesced, LDS-staged); per
//        block of L samples it emits the 2n+1 float64 numbers that summarise
//        the block for the zero-phase (forward + reverse) cascade: forward
//        all-pole state e_f, reverse exit state e_r0 and the reverse output at
//        the block's first sample p0.
//   k_block_functionals_gen — same for any strides (lanes = channels).
//   k_chunk_scan — per (chunk, channel): SciPy's odd-extension padding and
//        steady-state initial conditions at the chunk edges, the FIR-history
//        correction of the chunk's first block, the forward scan
//        S_f(k+1) = PhiF S_f(k) + e_f(k), the backward scan
//        T(k) = PhiR T(k+1) + e_r0(k) + M S_f(k) and the decimated outputs
//        y = p0 + H0 T(k+1) + G0 S_f(k).
//   k_sosfiltfilt_full — full-rate zero-phase filter (Patch.pass_filter alone).
//   k_interp_linear — linear gather (Patch.interpolate on a full-rate array).
//   k_rolling_* — windowed mean at the subsampled output points only.
//
// Reference semantics: scipy/signal/_signaltools.py:4718-4828 (sosfiltfilt),
// _arraytools.py:57-107 (odd_ext), _signaltools.py:4103-4175 (sosfilt_zi),
// scipy/interpolate/_interpolate.py:457-484 (linear interp1d); DASCore rolling.
// The block decomposition and realization R are derived in DESIGN.md §2.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../include/lfdas.h"
#include "lfd_internal.h"

namespace lfd {
namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
// the same vectors at the alignment of their element (4-B / 8-B aligned row
// pieces: rows whose stride is not a multiple of 4 samples).  gfx950 serves
// such accesses with the same global_load_dwordx4 / store (unaligned access
// mode), so one kernel covers every row stride
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
typedef double d2u __attribute__((ext_vector_type(2), aligned(8)));

// Nulls (SciPy semantics): a NaN / inf sample poisons every output of the
// chunks that contain it and nothing else.  A block's functionals also read
// samples outside its own L: J samples of FIR history and, in the MFMA
// kernels, zero-tap padding past the row.  Those reads are finite-masked
// (non-finite -> 0; finite values are unchanged) so that a null right
// beside a chunk boundary cannot leak into the neighbouring chunk; the scan's
// FIR-history correction masks the same samples the same way.
__device__ __forceinline__ float finite_or_zero(float v) { return __builtin_isfinite(v) ? v : 0.0f; }

// wave-uniform 64-bit value into SGPRs (VALU-computed values, e.g. 64-bit
// divisions, otherwise make every dependent branch divergent)
__device__ __forceinline__ int64_t uniform64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Compute units of the current device, cached per device (256 on MI355X;
// host launch sizing only)
int cu_count() {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n == 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
    cache[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

// ---------------------------------------------------------------------------
// TDF-II cascade step, SciPy's `_sosfilt` form (full-rate path only)
// ---------------------------------------------------------------------------
template <int NS>
struct FwdRec {
  double b0[NS], b1[NS], b2[NS], na1[NS], na2[NS];
  __device__ __forceinline__ void load(const SosCoef &c) {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      b0[i] = c.b0[i];
      b1[i] = c.b1[i];
      b2[i] = c.b2[i];
      na1[i] = -c.a1[i];
      na2[i] = -c.a2[i];
    }
  }
  __device__ __forceinline__ double step(double (&z)[2 * NS], double v) const {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const double vi = fma(b0[i], v, z[2 * i]);
      z[2 * i] = fma(b1[i], v, fma(na1[i], vi, z[2 * i + 1]));
      z[2 * i + 1] = fma(b2[i], v, na2[i] * vi);
      v = vi;
    }
    return v;
  }
};

// ---------------------------------------------------------------------------
// Realization R recurrences (see lfd_internal.h)
// ---------------------------------------------------------------------------
template <int NS, bool FIR32>
struct RRec {
  static constexpr int J = 2 * NS;
  double na1[NS], na2[NS], nia2[NS], nra[NS];
  float c32[J + 1];
  double c64[J + 1];
  __device__ __forceinline__ void load(const RCoef &r) {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      na1[i] = r.na1[i];
      na2[i] = r.na2[i];
      nia2[i] = r.nia2[i];
      nra[i] = r.nra[i];
    }
#pragma unroll
    for (int j = 0; j <= J; ++j) {
      c32[j] = r.c32[j];
      c64[j] = r.c64[j];
    }
  }
  // FIR on the newest sample xv with history h[0..J-1] = x[n-1..n-J]
  // (float32 when every tap is non-negative, else float64); shifts h.
  __device__ __forceinline__ double fir(float xv, float (&h)[J]) const {
    double w;
    if (FIR32) {
      float a = xv;
#pragma unroll
      for (int j = 1; j <= J; ++j) a = fmaf(c32[j], h[j - 1], a);
      w = (double)a;
    } else {
      double a = (double)xv;
#pragma unroll
      for (int j = 1; j <= J; ++j) a = fma(c64[j], (double)h[j - 1], a);
      w = a;
    }
#pragma unroll
    for (int j = J - 1; j > 0; --j) h[j] = h[j - 1];
    h[0] = xv;
    return w;
  }
  // all-pole cascade: S[2s] = v_s[n-1], S[2s+1] = v_s[n-2]; returns v_last
  __device__ __forceinline__ double allpole(double (&S)[2 * NS], double v) const {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const double vn = fma(na1[s], S[2 * s], fma(na2[s], S[2 * s + 1], v));
      S[2 * s + 1] = S[2 * s];
      S[2 * s] = vn;
      v = vn;
    }
    return v;
  }
  // inverse-time accumulator u <- A_r^{-1} u + B_r y   (7 ops for NS = 2)
  __device__ __forceinline__ void invacc(double (&u)[2 * NS], double y) const {
    double t[2 * NS];
#pragma unroll
    for (int i = 0; i < 2 * NS; ++i) t[i] = u[i];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      // loop-carried chain through u[2s+1] is a single FMA: the nia2*d
      // product depends only on the previous step's u[2s] (ready earlier)
      const double d = s == 0 ? t[0] : t[2 * s] - t[2 * s - 2];
      u[2 * s] = t[2 * s + 1] + y;
      u[2 * s + 1] = fma(nra[s], t[2 * s + 1], nia2[s] * d);
    }
  }
};

// Full scalar sample step of K1 (FIR -> all-pole -> accumulator).
#define LFD_R_SAMPLE(rec, xv, h, S, u, yv)    \
  do {                                       \
    const double w_ = rec.fir((xv), h);      \
    yv = rec.allpole(S, w_);                 \
    rec.invacc(u, yv);                       \
  } while (0)

// Block epilogue: e_f, e_r0 = T u, p0 = cp.u + dp.y0
template <int NS>
__device__ __forceinline__ void store_functionals(const BlockConst &kc, const double (&S)[2 * NS],
                                                  const double (&u)[2 * NS], double p0y,
                                                  double *F, int64_t k, int64_t ch,
                                                  int64_t nb) {
  constexpr int N = 2 * NS;
  const int64_t nF = 2 * N + 1;
  double *Fo = F + f_index(k, 0, ch, nb, (int)nF);
#pragma unroll
  for (int i = 0; i < N; ++i) Fo[i * F_CSTRIDE] = S[i];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) acc = fma(kc.T[i * MAX_N + j], u[j], acc);
    Fo[(N + i) * F_CSTRIDE] = acc;
  }
  double p0 = p0y;  // sum_m dp[m] y0[m], accumulated during the first samples
#pragma unroll
  for (int j = 0; j < N; ++j) p0 = fma(kc.cp[j], u[j], p0);
  Fo[2 * N * F_CSTRIDE] = p0;
}

// ---------------------------------------------------------------------------
// k_block_functionals_lds — time-contiguous rows, 16-B aligned, L % 4 == 0
// (the DASCore ("distance","time") layout).  Wave = 4 channels x 16
// consecutive blocks (one block per lane; TLB-local; the 4 waves of a
// workgroup complete 128-B lines of F = [k][comp][ch]).  Global loads are
// coalesced: each wave-instruction loads 16 consecutive rows x 64 B (4 lanes
// per row piece) into a wave-private LDS tile [64 rows][TS + 4 floats]; each
// lane then reads its own row with conflict-free ds_read_b128 (row stride 20
// dwords: banks 4*(5*lane mod 16)).  The next slice's loads are in flight in
// registers while the current slice is filtered.  LDS ops of one wave execute
// in order, so no barrier is needed.
// ---------------------------------------------------------------------------
constexpr int TS = 16;       // samples per row per slice
constexpr int TSP = TS + 4;  // padded LDS row stride (floats)

#ifndef LFD_K1_MINW
#define LFD_K1_MINW 4  // waves/SIMD the LDS kernel's register budget must allow
#endif

template <int NS, bool FIR32>
__global__ __launch_bounds__(256, LFD_K1_MINW) void k_block_functionals_lds(
    const float *__restrict__ x, int64_t s_ch, BlockGeom g, const BlockConst kc,
    double *__restrict__ F, int chan_fast) {
  constexpr int N = 2 * NS;
  constexpr int J = 2 * NS;
  static_assert(J <= 4 * (TS / 4), "history must fit one slice");
  __shared__ __attribute__((aligned(16))) float lds_all[4][64 * TSP];
  // tile order: time-fastest (default) keeps the resident workgroups on a few
  // channel groups, so the pages in flight stay few (TLB); channel-fastest
  // spreads them over every channel (LFD_K1_CHAN_FAST=1, for A/B).
  const int64_t n_ct = (g.n_ch + 15) / 16;
  const int64_t n_kt = (g.nb + 15) / 16;
  const int64_t tile = blockIdx.x;
  int64_t ct, kt;
  if (chan_fast) {
    ct = tile % n_ct;
    kt = tile / n_ct;
  } else {
    kt = tile % n_kt;
    ct = tile / n_kt;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float *lds = lds_all[wave];
  const int L = g.L;

  const int64_t ch = ct * 16 + wave * 4 + (lane >> 4);
  const int64_t k = kt * 16 + (lane & 15);
  const bool live = ch < g.n_ch && k < g.nb;
  const int64_t chc = ch < g.n_ch ? ch : g.n_ch - 1;
  const int64_t kc_ = k < g.nb ? k : g.nb - 1;

  // rows this lane stages: instruction i covers channel wave*4+i, block
  // kt*16 + lane/4, samples [t + 4*(lane%4), +4)
  const float *src[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int64_t c = ct * 16 + wave * 4 + i;
    int64_t kk = kt * 16 + (lane >> 2);
    c = c < g.n_ch ? c : g.n_ch - 1;
    kk = kk < g.nb ? kk : g.nb - 1;
    src[i] = x + c * s_ch + g.base + kk * (int64_t)L + 4 * (lane & 3);
  }
  float *wr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) wr[i] = lds + (16 * i + (lane >> 2)) * TSP + 4 * (lane & 3);
  const float *rd = lds + lane * TSP;

  RRec<NS, FIR32> rec;
  rec.load(kc.r);
  double S[N], u[N], p0y = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) S[i] = u[i] = 0.0;
  // FIR history: the J samples before the block (0 before the channel start)
  float h[J];
  {
    const int64_t a = g.base + kc_ * (int64_t)L;
    const float *row = x + chc * s_ch;
#pragma unroll
    for (int j = 0; j < J; ++j) h[j] = (a - 1 - j >= 0) ? finite_or_zero(row[a - 1 - j]) : 0.0f;
  }

  const int nfull = L / TS;              // full slices
  const int rem4 = (L - nfull * TS) >> 2;  // float4s of the partial slice (L % 4 == 0)
  const int last_t = (nfull + (rem4 ? 1 : 0) - 1) * TS;
  // two register stages keep two slices of loads in flight per wave
  f4v stA[4], stB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) stA[i] = *reinterpret_cast<const f4v *>(src[i]);
#pragma unroll
  for (int i = 0; i < 4; ++i) stB[i] = *reinterpret_cast<const f4v *>(src[i] + min(TS, last_t));

#define LFD_QUAD(v)                          \
  do {                                       \
    double yv_;                              \
    LFD_R_SAMPLE(rec, v.x, h, S, u, yv_);    \
    LFD_R_SAMPLE(rec, v.y, h, S, u, yv_);    \
    LFD_R_SAMPLE(rec, v.z, h, S, u, yv_);    \
    LFD_R_SAMPLE(rec, v.w, h, S, u, yv_);    \
  } while (0)
// stage -> LDS, refill the stage with slice sl+2, read this lane's row
#define LFD_STAGE(st, sl)                                                              \
  do {                                                                                 \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) *reinterpret_cast<f4v *>(wr[i]) = st[i]; \
    const int tn_ = min(((sl) + 2) * TS, last_t);                                      \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) st[i] =                              \
        *reinterpret_cast<const f4v *>(src[i] + tn_);                                  \
  } while (0)
#define LFD_FULL_SLICE(st, sl)                                  \
  do {                                                          \
    LFD_STAGE(st, sl);                                          \
    const f4v v0_ = *reinterpret_cast<const f4v *>(rd);         \
    const f4v v1_ = *reinterpret_cast<const f4v *>(rd + 4);     \
    const f4v v2_ = *reinterpret_cast<const f4v *>(rd + 8);     \
    const f4v v3_ = *reinterpret_cast<const f4v *>(rd + 12);    \
    LFD_QUAD(v0_);                                              \
    LFD_QUAD(v1_);                                              \
    LFD_QUAD(v2_);                                              \
    LFD_QUAD(v3_);                                              \
  } while (0)

  // slice 0 (peeled): capture the first J forward outputs for p0
  {
    LFD_STAGE(stA, 0);
    const int nq = nfull ? TS / 4 : rem4;
#pragma unroll
    for (int j = 0; j < TS / 4; ++j) {
      if (j < nq) {
        const f4v v = *reinterpret_cast<const f4v *>(rd + 4 * j);
        double yv;
        LFD_R_SAMPLE(rec, v.x, h, S, u, yv);
        if (4 * j + 0 <= J) p0y = fma(kc.dp[4 * j + 0], yv, p0y);
        LFD_R_SAMPLE(rec, v.y, h, S, u, yv);
        if (4 * j + 1 <= J) p0y = fma(kc.dp[4 * j + 1], yv, p0y);
        LFD_R_SAMPLE(rec, v.z, h, S, u, yv);
        if (4 * j + 2 <= J) p0y = fma(kc.dp[4 * j + 2], yv, p0y);
        LFD_R_SAMPLE(rec, v.w, h, S, u, yv);
        if (4 * j + 3 <= J) p0y = fma(kc.dp[4 * j + 3], yv, p0y);
      }
    }
  }
  // full slices 1..nfull-1, two per iteration (static stage indices)
  int sl = 1;
  for (; sl + 1 < nfull; sl += 2) {
    LFD_FULL_SLICE(stB, sl);
    LFD_FULL_SLICE(stA, sl + 1);
  }
  bool next_in_A = false;  // stage holding slice `sl`
  if (sl < nfull) {
    LFD_FULL_SLICE(stB, sl);
    ++sl;
    next_in_A = true;
  }
  // partial last slice
  if (rem4 && nfull >= 1) {
    if (next_in_A) {
#pragma unroll
      for (int i = 0; i < 4; ++i) *reinterpret_cast<f4v *>(wr[i]) = stA[i];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) *reinterpret_cast<f4v *>(wr[i]) = stB[i];
    }
#pragma unroll
    for (int j = 0; j < TS / 4; ++j) {
      if (j < rem4) {
        const f4v v = *reinterpret_cast<const f4v *>(rd + 4 * j);
        LFD_QUAD(v);
      }
    }
  }
#undef LFD_FULL_SLICE
#undef LFD_STAGE
#undef LFD_QUAD
  if (live) store_functionals<NS>(kc, S, u, p0y, F, k, ch, g.nb);
}

// ---------------------------------------------------------------------------
// k_block_functionals_gen — any strides.  Workgroup = 64 channels x 4 blocks;
// a wave is 64 consecutive channels of one block, so a load is 64 consecutive
// floats when s_ch == 1 (the real-file ("time","distance") layout).  A ring of
// D samples per lane stays in flight (clamped indices, branch-free body).
// ---------------------------------------------------------------------------
template <int NS, bool FIR32>
__global__ __launch_bounds__(256) void k_block_functionals_gen(
    const float *__restrict__ x, int64_t s_ch, int64_t s_t, BlockGeom g, const BlockConst kc,
    double *__restrict__ F) {
  constexpr int N = 2 * NS;
  constexpr int J = 2 * NS;
  constexpr int D = 8;
  const int64_t n_kt = (g.nb + 3) / 4;
  const int64_t tile = blockIdx.x;
  const int64_t kt = tile % n_kt, ct = tile / n_kt;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t ch = ct * 64 + lane;
  const int64_t k = kt * 4 + wave;
  if (ch >= g.n_ch || k >= g.nb) return;
  RRec<NS, FIR32> rec;
  rec.load(kc.r);
  double S[N], u[N], p0y = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) S[i] = u[i] = 0.0;
  const int L = g.L;
  const int64_t a = g.base + k * (int64_t)L;
  const float *row = x + ch * s_ch;
  float h[J];
#pragma unroll
  for (int j = 0; j < J; ++j) h[j] = (a - 1 - j >= 0) ? finite_or_zero(row[(a - 1 - j) * s_t]) : 0.0f;
  const float *p = row + a * s_t;
  float buf[D];
#pragma unroll
  for (int d = 0; d < D; ++d) buf[d] = p[(int64_t)min(d, L - 1) * s_t];
  const int Gn = L / D;
  for (int gi = 0; gi < Gn; ++gi) {
    const int nxt = (gi + 1) * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float v = buf[d];
      buf[d] = p[(int64_t)min(nxt + d, L - 1) * s_t];
      double yv;
      LFD_R_SAMPLE(rec, v, h, S, u, yv);
      if (gi * D + d <= J) p0y = fma(kc.dp[min(gi * D + d, J)], yv, p0y);
    }
  }
  const int rem = L - Gn * D;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    if (d < rem) {
      double yv;
      LFD_R_SAMPLE(rec, buf[d], h, S, u, yv);
      const int m = Gn * D + d;
      if (m <= J) p0y = fma(kc.dp[m <= J ? m : 0], yv, p0y);
    }
  }
  store_functionals<NS>(kc, S, u, p0y, F, k, ch, g.nb);
}

// ---------------------------------------------------------------------------
// k_chunk_scan: one thread per (chunk, channel), channel fastest.
// ---------------------------------------------------------------------------
template <int NS>
struct SeqR {  // sequential realization-R steps in float64 (edges)
  static constexpr int J = 2 * NS;
  const RCoef &r;
  __device__ explicit SeqR(const RCoef &rr) : r(rr) {}
  __device__ __forceinline__ double fwd(double (&S)[2 * NS], double (&h)[J], double xv) const {
    double w = xv;
#pragma unroll
    for (int j = 1; j <= J; ++j) w = fma(r.c64[j], h[j - 1], w);
#pragma unroll
    for (int j = J - 1; j > 0; --j) h[j] = h[j - 1];
    h[0] = xv;
    double v = w;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const double vn = fma(r.na1[s], S[2 * s], fma(r.na2[s], S[2 * s + 1], v));
      S[2 * s + 1] = S[2 * s];
      S[2 * s] = vn;
      v = vn;
    }
    return r.G * v;  // y_f
  }
  __device__ __forceinline__ double rev(double (&T)[2 * NS], double y) const {
    double v = y;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const double qn = fma(r.na1[s], T[2 * s], fma(r.na2[s], T[2 * s + 1], v));
      T[2 * s + 1] = T[2 * s];
      T[2 * s] = qn;
      v = qn;
    }
    return v;  // q_last
  }
  // steady state of the cascade for a constant input c (what SciPy's
  // sosfilt_zi * c encodes): every section at v = c * csum * prod dcg
  __device__ __forceinline__ double steady(double (&S)[2 * NS], double c, bool with_fir) const {
    double v = with_fir ? c * r.csum : c;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      v *= r.dcg[s];
      S[2 * s] = S[2 * s + 1] = v;
    }
    return v;
  }
};

// RUNS: the scans walk runs (lfd_internal.h RunConst) over K1's y0 / run
// aggregates instead of blocks over F (requires NS == 2).
#ifndef SCAN_DF
#define SCAN_DF 4  // runs in flight in the forward scan
#endif
#ifndef SCAN_DB
#define SCAN_DB 2  // runs in flight in the backward scan
#endif
// LFD_SCAN_DIAG (timing experiments only, results invalid): bit 1 skips the
// left pad/head, 2 the forward run scan, 4 the right pad and its reverse,
// 8 the backward run scan, 16 the backward scan's y0 loads (zeros), 32 its
// output stores.
#ifdef LFD_DIAG
__constant__ int g_scan_diag = 0;
#endif
// LFD_DG(v): a diagnostic / A/B value, the constant 0 in the production
// build (-DLFD_DIAG builds liblfdas_diag.so for tools/), so every branch it
// guards is compiled out of liblfdas.so
#ifdef LFD_DIAG
#define LFD_DG(v) (v)
#else
#define LFD_DG(v) 0
#endif

// ---- scan edges (k_chunk_scan and k_scan_fused) ----
// Left edge of chunk G for channel row xc: SciPy's odd extension (formed in
// float32, like numpy on float32 input) from the steady state of ext[0], then
// the chunk's samples before block kb (run mode: or the head skip, see
// ChunkGeom::hskip).  Leaves S = the forward state entering block kb and corr
// = the FIR-history corrections of block kb's functionals (K1 used the raw
// samples before head_end; this chunk saw pad / head values).
template <int NS, bool RUNS>
__device__ __forceinline__ void scan_head(const float *__restrict__ xc, int64_t s_t, const ChunkGeom &G, int L, int E,
                                          const SeqR<NS> &R, const ScanConst &sc, const RunConst *rcl,
                                          const double *__restrict__ AG, const RunGeom &rg, int64_t ch,
                                          double (&S)[2 * NS], double (&corr)[4 * NS + 1]) {
  constexpr int N = 2 * NS, J = 2 * NS, NF = 2 * N + 1;
  constexpr int SB = 8;
  double h[J];
  // ---- left edge: odd extension (float32 like numpy), steady state of ext[0]
  const float xl = xc[G.s0 * s_t];
  // head skip (run mode, ChunkGeom::hskip): the head is block kb-1 without
  // its samples [lo, s0), so the state entering block kb is
  //   PhiF S(lo) + E_f(kb-1) + sum_p KfH[.][p] (pad - raw)(lo - J + p)
  // with S(lo) the state after the pad's samples before lo: K1 already summed
  // the head.  A null in [lo, s0) (outside this chunk) poisons e_f(kb-1), so
  // such a (chunk, channel) walks its head instead.
  const int64_t lo_h = G.head_end - L;
  bool hs = false;
  if constexpr (RUNS) {
    if (G.hskip && E > 0 && !(LFD_DG(g_scan_diag) & 1)) {
      hs = true;
      for (int64_t t = lo_h; t < G.s0; ++t) hs = hs && __builtin_isfinite(xc[t * s_t]);
    }
  }
  {
    const int n_pad = hs ? E - (int)(G.s0 - lo_h) : E;
    const double e0 = E > 0 ? (double)(2.0f * xl - xc[(G.s0 + E) * s_t]) : (double)xl;
    R.steady(S, e0, true);
#pragma unroll
    for (int j = 0; j < J; ++j) h[j] = e0;
    for (int i = 0; i < n_pad && !(LFD_DG(g_scan_diag) & 1); ++i) R.fwd(S, h, (double)(2.0f * xl - xc[(G.s0 + E - i) * s_t]));
  }
  if constexpr (RUNS) {
    if (hs) {
      static_assert(N == RUN_N, "run mode is 4th order");
      const RunConst &rc = *rcl;
      const double *agh = AG + ((((ch >> 4) * rg.n_runs) + (G.r0 - 1)) * 8) * 16 + (ch & 15);
      double ns[N];
#pragma unroll
      for (int i = 0; i < N; ++i) {
        double acc = agh[i * 16];
#pragma unroll
        for (int j = 0; j < N; ++j) acc = fma(rc.PhiFp[1][i * 4 + j], S[j], acc);
        ns[i] = acc;
      }
      const int ncorr = (int)(G.s0 - lo_h) + J;
      for (int pq = 0; pq < ncorr; ++pq) {
        const int64_t pos = lo_h - J + pq;
        const double u = (double)(2.0f * xl - xc[(2 * G.s0 - pos) * s_t]);
        const float xv = pos < 0 ? 0.0f : xc[pos * s_t];
        const double raw = pos < lo_h ? (double)finite_or_zero(xv) : (double)xv;
        const double d = u - raw;
#pragma unroll
        for (int i = 0; i < N; ++i) ns[i] = fma(rc.KfH[i][pq], d, ns[i]);
      }
#pragma unroll
      for (int i = 0; i < N; ++i) S[i] = ns[i];
#pragma unroll
      for (int j = 0; j < J; ++j) h[j] = (double)xc[(G.head_end - 1 - j) * s_t];
    }
  }
  if (!(LFD_DG(g_scan_diag) & 1) && !hs) {
    int64_t t = G.s0;
    for (; t + SB <= G.head_end; t += SB) {
      float xv[SB];
#pragma unroll
      for (int u = 0; u < SB; ++u) xv[u] = xc[(t + u) * s_t];
#pragma unroll
      for (int u = 0; u < SB; ++u) R.fwd(S, h, (double)xv[u]);
    }
    for (; t < G.head_end; ++t) R.fwd(S, h, (double)xc[t * s_t]);
  }

  // ---- FIR-history correction of block kb: K1 used the raw samples before
  // head_end (0 before the channel start); this chunk saw pad / head values.
  {
    double dh[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int64_t t = G.head_end - 1 - j;
      dh[j] = h[j] - (t >= 0 ? (double)finite_or_zero(xc[t * s_t]) : 0.0);
    }
    double dw[J];
#pragma unroll
    for (int m = 0; m < J; ++m) {
      double acc = 0.0;
#pragma unroll
      for (int jj = m + 1; jj <= J; ++jj) acc = fma(sc.r.c64[jj], dh[jj - m - 1], acc);
      dw[m] = acc;
    }
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      double acc = 0.0;
#pragma unroll
      for (int m = 0; m < J; ++m) acc = fma(sc.Kc[i * MAX_J + m], dw[m], acc);
      corr[i] = acc;
    }
  }

}

// Right edge: the tail samples after block ke-1 and SciPy's odd extension,
// forward from S (the state after the chunk's last full block) into tp
// (stride tp_stride), then the reverse pass over them from the steady state
// of the last forward output; the output inside the tail (ChunkGeom::
// tail_out_j) is stored.  Leaves T = the reverse state entering block ke-1
// from the right.
template <int NS>
__device__ __forceinline__ void scan_tail(const float *__restrict__ xc, int64_t s_t, const ChunkGeom &G, int E,
                                          const SeqR<NS> &R, const ScanConst &sc, double (&S)[2 * NS],
                                          double *__restrict__ tp, int64_t tp_stride, double *__restrict__ y,
                                          int64_t ch, int64_t ys_ch, int64_t ys_t, double (&T)[2 * NS],
                                          bool store = true, double *yret = nullptr) {
  constexpr int J = 2 * NS;
  constexpr int SB = 8;
  double h[J];
  // ---- right edge: tail samples + odd extension, forward, stored
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int64_t t = G.tail_begin - 1 - j;
    h[j] = (double)xc[t * s_t];
  }
  int64_t ntp = 0;
  double ylast = 0.0;
  if (!(LFD_DG(g_scan_diag) & 4)) {
    int64_t t = G.tail_begin;
    for (; t + SB <= G.s1 + 1; t += SB) {
      float xv[SB];
#pragma unroll
      for (int u = 0; u < SB; ++u) xv[u] = xc[(t + u) * s_t];
#pragma unroll
      for (int u = 0; u < SB; ++u) {
        ylast = R.fwd(S, h, (double)xv[u]);
        tp[(ntp + u) * tp_stride] = ylast;
      }
      ntp += SB;
    }
    for (; t <= G.s1; ++t) {
      ylast = R.fwd(S, h, (double)xc[t * s_t]);
      tp[(ntp++) * tp_stride] = ylast;
    }
  }
  const float xr = xc[G.s1 * s_t];
  for (int i = 0; i < E && !(LFD_DG(g_scan_diag) & 4); ++i) {
    ylast = R.fwd(S, h, (double)(2.0f * xr - xc[(G.s1 - 1 - i) * s_t]));
    tp[(ntp++) * tp_stride] = ylast;
  }

  // ---- reverse pass over pad + tail from the steady state of y_f[-1]
  double qw[J];  // qw[j] = q_last[m+1+j] (future values for the FIR)
  {
    const double qss = R.steady(T, ylast, false);
#pragma unroll
    for (int j = 0; j < J; ++j) qw[j] = qss;
  }
  double y_next = 0.0;  // zero-phase output one sample after the tail output
  auto rev_step = [&](int64_t i, double v) {
    const double q = R.rev(T, v);
    if (G.tail_out_j >= 0 && (G.tail_begin + i == G.tail_out_pos || G.tail_begin + i == G.tail_out_pos + 1)) {
      double acc = q;  // c[0] = 1
#pragma unroll
      for (int j = 1; j <= J; ++j) acc = fma(sc.r.c64[j], qw[j - 1], acc);
      acc *= sc.r.G;
      if (G.tail_begin + i == G.tail_out_pos + 1) {
        y_next = acc;
      } else {  // interp1d between the two samples (w = sc.ow)
        const double yv = fma(sc.ow, y_next - acc, acc);
        if (yret)
          *yret = yv;  // (k_scan_fused's zero-state edge: the caller adds the state part)
        else if (store)
          y[ch * ys_ch + G.tail_out_j * ys_t] = yv;
      }
    }
#pragma unroll
    for (int j = J - 1; j > 0; --j) qw[j] = qw[j - 1];
    qw[0] = q;
  };
  {
    int64_t i = ntp - 1;
    for (; i + 1 >= SB; i -= SB) {
      double tv[SB];
#pragma unroll
      for (int u = 0; u < SB; ++u) tv[u] = tp[(i - u) * tp_stride];
#pragma unroll
      for (int u = 0; u < SB; ++u) rev_step(i - u, tv[u]);
    }
    for (; i >= 0; --i) rev_step(i, tp[i * tp_stride]);
  }

}

// DEFER (run mode): the backward run scan only carries T and stores the T
// entering every run (TR, laid out like SR) and the chunk's p0 correction
// (CR [chunk][ch64]); k_run_outputs then forms the outputs of every run in
// parallel.  The per-thread chain is then the 4x4 T recurrence alone: with
// the outputs inside the chain a 1,250-channel shard spent 2.3 us per run
// step on one wave per 7 SIMDs.
// SEGM (segmented chains, run mode with DEFER): 1 = the head only: the state
// entering run r0 and the FIR-history corrections go to SC, then return (the
// forward chain is k_seg_fwd's); 2 = the tail only, from the state after the
// chunk's last run (SC, from k_seg_fwd): pad + tail forward, the reverse over
// them, the T entering the last run into SC, then return (the backward chain
// is k_seg_bwd's).  SC layout: [chunk][SC_* slot][ch64].
constexpr int SC_HS = 0, SC_SE = 4, SC_TE = 8, SC_CORR = 12, SC_N = SC_N_HOST;
template <int NS, bool RUNS, bool DEFER = false, int DFT = SCAN_DF, int DBT = SCAN_DB, int SEGM = 0>
__global__ __launch_bounds__(256) void k_chunk_scan(
    const float *__restrict__ x, int64_t s_ch, int64_t s_t, BlockGeom g, int padlen,
    const ScanConst sc, const ChunkGeom *__restrict__ cgs, int64_t n_chunks,
    const double *__restrict__ F, double *__restrict__ SF, double *__restrict__ TP,
    int64_t tp_len, double *__restrict__ y, int64_t ys_ch, int64_t ys_t, RunGeom rg,
    const double *__restrict__ Y0, double *__restrict__ TR = nullptr, double *__restrict__ CR = nullptr,
    double *__restrict__ SC = nullptr) {
  constexpr int N = 2 * NS;
  constexpr int NF = 2 * N + 1;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n_thr = n_chunks * g.n_ch;
  // run mode: the run-algebra constants live in LDS (read every run step;
  // from global they put two dependent load latencies on each step)
  __shared__ RunConst rcs[1];
  // run-mode output staging: a wave's 64 channels x one run's <= 8 outputs,
  // written back as 8 rows x 8 consecutive samples per store instruction
  // instead of 64 scattered 4-B stores (0.2 ms of the cfg3 scan)
  __shared__ double outs[RUNS ? 4 : 1][64][RUN_R + 1];
  if constexpr (RUNS) {
    // the fields this scan reads: PhiFp, PhiRp, C (+ A, B for in-chain
    // outputs) and KfH — not the whole 12 KB RunConst (a 64-thread group of
    // a narrow shard loaded 24 doubles per thread before its first step)
    const double *src = &rg.rc->PhiFp[0][0];
    double *dst = &rcs[0].PhiFp[0][0];
    constexpr int n_head = (int)((offsetof(RunConst, A) - offsetof(RunConst, PhiFp)) / sizeof(double));
    constexpr int n_ab = (int)((offsetof(RunConst, PhiF) - offsetof(RunConst, A)) / sizeof(double));
    constexpr int o_kfh = (int)((offsetof(RunConst, KfH) - offsetof(RunConst, PhiFp)) / sizeof(double));
    constexpr int n_copy = n_head + (DEFER ? 0 : n_ab);
    for (int i = threadIdx.x; i < n_copy; i += blockDim.x) dst[i] = src[i];
    for (int i = threadIdx.x; i < 4 * HSKIP_MAX; i += blockDim.x) dst[o_kfh + i] = src[o_kfh + i];
    __syncthreads();
  }
  // whole wave active and inside one chunk: outputs leave through LDS (above)
  const int lane = threadIdx.x & 63;
  const int64_t tid_w = tid - lane;
  const bool coal = RUNS && tid_w + 63 < n_thr && tid_w / g.n_ch == (tid_w + 63) / g.n_ch;
  const int64_t ch_w = tid_w % g.n_ch;
  if (tid >= n_thr) return;
  const int64_t ch = tid % g.n_ch;
  const int64_t c = tid / g.n_ch;
  const ChunkGeom G = cgs[c];
  const float *xc = x + ch * s_ch;
  const int E = padlen;
  const SeqR<NS> R(sc.r);
  (void)tp_len;
  // output blocks: kout0, kout0 + kstep, ... (kstep > 1: sub-blocks)
  const int kst = (int)G.kstep;
  auto is_out = [&](int64_t k) {
    return k >= G.kout0 && k < G.kout1 && (kst == 1 || (int)(k - G.kout0) % kst == 0);
  };
  auto out_j = [&](int64_t k) -> int64_t {
    return G.jout0 + (kst == 1 ? k - G.kout0 : (int64_t)((int)(k - G.kout0) / kst));
  };

  const int64_t ch64 = (g.n_ch + 63) / 64 * 64;
  auto sc_at = [&](int slot) -> double & { return SC[(c * SC_N + slot) * ch64 + ch]; };
  // (scan_head / scan_tail: the edges' sample walks issue 8 samples' loads
  // together — a per-step load left every step waiting on memory latency)
  double S[N];
  double corr[NF];
  const int64_t nF = NF;
  if constexpr (SEGM == 2) {
    // (segmented chains) the state after the chunk's last run
#pragma unroll
    for (int i = 0; i < N; ++i) S[i] = sc_at(SC_SE + i);
#pragma unroll
    for (int i = 0; i < NF; ++i) corr[i] = 0.0;
  } else {
  scan_head<NS, RUNS>(xc, s_t, G, g.L, E, R, sc, RUNS ? &rcs[0] : nullptr, F, rg, ch, S, corr);
  if (DEFER) CR[c * ((g.n_ch + 63) / 64 * 64) + ch] = corr[2 * N];
  if constexpr (SEGM == 1) {
#pragma unroll
    for (int i = 0; i < N; ++i) sc_at(SC_HS + i) = S[i];
#pragma unroll
    for (int i = 0; i < NF; ++i) sc_at(SC_CORR + i) = corr[i];
    return;
  }
  // ---- forward scan over the full blocks (run mode: over runs; SF holds S_in
  // per run, F holds the run aggregates)
  if constexpr (RUNS) {
    static_assert(N == RUN_N, "run mode is 4th order");
    const RunConst &rc = rcs[0];
    // software-pipelined through a ring of SCAN_DF runs: the aggregates and
    // lengths of runs r+1 .. r+SCAN_DF-1 are in flight while run r is applied
    // (the step is ~150 cycles, a load ~1.5 us)
    constexpr int DF = DFT;
    const double *agb = F + (((ch >> 4) * rg.n_runs) * 8) * 16 + (ch & 15);
    double agq[DF][N];
    int lenq[DF];
#pragma unroll
    for (int u = 0; u < DF; ++u) {
      const int64_t r = G.r0 + u;
      lenq[u] = r < G.r1 ? rg.run_len[r] : 0;
#pragma unroll
      for (int i = 0; i < N; ++i) agq[u][i] = r < G.r1 ? agb[(r * 8 + i) * 16] : 0.0;
    }
    for (int64_t rb = G.r0; rb < G.r1 && !(LFD_DG(g_scan_diag) & 2); rb += DF) {
#pragma unroll
      for (int u = 0; u < DF; ++u) {
        const int64_t r = rb + u;
        if (r >= G.r1) break;
        const int len = lenq[u];
        double *sr = SF + sf_index(G.sr_off + (r - G.r0), 0, ch, rg.n_sr, N);
        const double *P = rc.PhiFp[len];
        double ns[N];
#pragma unroll
        for (int i = 0; i < N; ++i) {
          sr[i * SF_ISTRIDE] = S[i];
          double acc = agq[u][i] + (r == G.r0 ? corr[i] : 0.0);
#pragma unroll
          for (int j = 0; j < N; ++j) acc = fma(P[i * 4 + j], S[j], acc);
          ns[i] = acc;
        }
#pragma unroll
        for (int i = 0; i < N; ++i) S[i] = ns[i];
        {
          // unconditional (clamped) refill of slot u after its last use: a
          // conditional load, or a copy of the slot before refilling it,
          // makes the compiler wait for every load in flight (vmcnt(0))
          const int64_t rn = min(r + DF, G.r1 - 1);
          lenq[u] = rg.run_len[rn];
#pragma unroll
          for (int i = 0; i < N; ++i) agq[u][i] = agb[(rn * 8 + i) * 16];
        }
      }
    }
  }
  for (int64_t k = G.kb; !RUNS && k < G.ke; ++k) {
    double *sf = SF + sf_index(G.sf_off + (k - G.kb), 0, ch, g.n_sf, N);
    const double *f = F + f_index(k, 0, ch, g.nb, nF);
    double ns[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      sf[i * SF_ISTRIDE] = S[i];
      double acc = f[i * F_CSTRIDE] + (k == G.kb ? corr[i] : 0.0);
#pragma unroll
      for (int j = 0; j < N; ++j) acc = fma(sc.PhiF[i * MAX_N + j], S[j], acc);
      ns[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) S[i] = ns[i];
  }
  }  // SEGM != 2

  double T[N];
  scan_tail<NS>(xc, s_t, G, E, R, sc, S, TP + tid, n_thr, y, ch, ys_ch, ys_t, T);

  // ---- backward scan, outputs at block starts
  if constexpr (SEGM == 2) {
#pragma unroll
    for (int i = 0; i < N; ++i) sc_at(SC_TE + i) = T[i];
    return;
  }
  if constexpr (RUNS) {
    const RunConst &rc = rcs[0];
    // software-pipelined like the forward scan: run r-1's inputs (S_in,
    // E_r, y0 of its blocks, length, first block) load while run r is applied
    struct RunIn {
      double sin[N], er[N], y0[RUN_R];
      int len;
      int64_t ks;
    };
    const double *agb = F + (((ch >> 4) * rg.n_runs) * 8) * 16 + (ch & 15);
    const double *y0b = Y0 + ((ch >> 4) * g.nb) * 16 + (ch & 15);
    // a run's geometry (len, first block) is loaded SCAN_DB runs before its
    // inputs: the Y0 addresses depend on it, and vmcnt waits are in order, so
    // loading it together with the inputs drained the whole ring every run
    struct RunGeo {
      int len;
      int64_t ks;
    };
    auto load_geo = [&](int64_t r, RunGeo &o) {
      o.len = rg.run_len[r];
      o.ks = rg.run_ks[r];
    };
    auto load_run = [&](int64_t r, const RunGeo &gg, RunIn &o) {
      o.len = gg.len;
      o.ks = gg.ks;
      const double *sr = SF + sf_index(G.sr_off + (r - G.r0), 0, ch, rg.n_sr, N);
#pragma unroll
      for (int i = 0; i < N; ++i) {
        o.sin[i] = sr[i * SF_ISTRIDE];
        o.er[i] = agb[(r * 8 + 4 + i) * 16];
      }
      // every y0 slot loaded (clamped to the plan's blocks; unused ones are
      // masked where they are consumed): a fixed number of loads per run
      if (!DEFER && !(LFD_DG(g_scan_diag) & 16)) {
#pragma unroll
        for (int pp = 0; pp < RUN_R; ++pp) o.y0[pp] = y0b[min(o.ks + pp, g.nb - 1) * 16];
      } else if (!DEFER) {
#pragma unroll
        for (int pp = 0; pp < RUN_R; ++pp) o.y0[pp] = 0.0;
      }
    };
    // ring of SCAN_DB slots (runs r-1 .. r-SCAN_DB+1 in flight while run r is
    // applied)
    constexpr int DB = DBT;
    // q[u] holds run r's inputs, gq[u] run r-DB's geometry (slot u = r mod DB)
    RunIn q[DB];
    RunGeo gq[DB];
#pragma unroll
    for (int u = 0; u < DB; ++u) {
      if (G.r1 - 1 - u >= G.r0) {
        RunGeo g0;
        load_geo(G.r1 - 1 - u, g0);
        load_run(G.r1 - 1 - u, g0, q[u]);
      }
    }
    // (clamped like the loop's: slot u must hold max(r - DB, r0)'s geometry
    // when run r = r1 - 1 - u is applied)
#pragma unroll
    for (int u = 0; u < DB; ++u) load_geo(max(G.r1 - 1 - u - DB, G.r0), gq[u]);
    for (int64_t rb = G.r1 - 1; rb >= G.r0 && !(LFD_DG(g_scan_diag) & 8); rb -= DB)
#pragma unroll
    for (int u = 0; u < DB; ++u) {
      const int64_t r = rb - u;
      if (r < G.r0) break;
      // slot u is applied in place and refilled after its last use (below):
      // copying it out before the refill made the compiler wait for every
      // load in flight (vmcnt(0)) at each step, so the ring overlapped nothing
      const RunIn &cur = q[u];
      const int len = cur.len;
      const int64_t ks = cur.ks;
      const double *sin = cur.sin;
      if (DEFER) {
        double *tr = TR + sf_index(G.sr_off + (r - G.r0), 0, ch, rg.n_sr, N);
#pragma unroll
        for (int i = 0; i < N; ++i) tr[i * SF_ISTRIDE] = T[i];
      }
      double ov[RUN_R];
#pragma unroll
      for (int pp = 0; pp < RUN_R; ++pp) {
        const int64_t k = ks + pp;
        ov[pp] = 0.0;
        if (DEFER || pp >= len || !is_out(k)) continue;
        double acc = cur.y0[pp] + (k == G.kb ? corr[2 * N] : 0.0);
        const double *A = rc.A[len][pp];
        const double *B = rc.B[len - 1 - pp];
#pragma unroll
        for (int j = 0; j < N; ++j) {
          acc = fma(A[j], sin[j], acc);
          acc = fma(B[j], T[j], acc);
        }
        ov[pp] = acc;
        if (!coal) y[ch * ys_ch + out_j(k) * ys_t] = ov[pp];
      }
      if (coal && !DEFER) {
        double(*wl)[RUN_R + 1] = outs[(threadIdx.x >> 6) & 3];
#pragma unroll
        for (int pp = 0; pp < RUN_R; ++pp) wl[lane][pp] = ov[pp];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int e = lane & 7;
        const int64_t k = ks + e;
        const bool ok = e < len && is_out(k);
        double *yb = y + ch_w * ys_ch + (ok ? out_j(k) : 0) * ys_t;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const int row = m * 8 + (lane >> 3);
          const double v = wl[row][e];
          if (ok && !(LFD_DG(g_scan_diag) & 32)) yb[row * ys_ch] = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      const double *PR = rc.PhiRp[len], *CC = rc.C[len];
      double nr[N];
#pragma unroll
      for (int i = 0; i < N; ++i) {
        double acc = cur.er[i] + (r == G.r0 ? corr[N + i] : 0.0);
#pragma unroll
        for (int j = 0; j < N; ++j) {
          acc = fma(PR[i * 4 + j], T[j], acc);
          acc = fma(CC[i * 4 + j], sin[j], acc);
        }
        nr[i] = acc;
      }
#pragma unroll
      for (int i = 0; i < N; ++i) T[i] = nr[i];
      // unconditional (clamped) refill of slot u, see the forward scan
      load_run(max(r - DB, G.r0), gq[u], q[u]);
      load_geo(max(r - 2 * DB, G.r0), gq[u]);
    }
    return;
  }
  for (int64_t k = G.ke - 1; k >= G.kb; --k) {
    const double *sf = SF + sf_index(G.sf_off + (k - G.kb), 0, ch, g.n_sf, N);
    const double *f = F + f_index(k, 0, ch, g.nb, nF);
    const bool first = (k == G.kb);
    double sfv[N];
#pragma unroll
    for (int i = 0; i < N; ++i) sfv[i] = sf[i * SF_ISTRIDE];
    if (is_out(k)) {
      double acc = f[2 * N * F_CSTRIDE] + (first ? corr[2 * N] : 0.0);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        acc = fma(sc.H0[j], T[j], acc);
        acc = fma(sc.G0[j], sfv[j], acc);
      }
      y[ch * ys_ch + out_j(k) * ys_t] = acc;
    }
    double nr[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      double acc = f[(N + i) * F_CSTRIDE] + (first ? corr[N + i] : 0.0);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        acc = fma(sc.PhiR[i * MAX_N + j], T[j], acc);
        acc = fma(sc.M[i * MAX_N + j], sfv[j], acc);
      }
      nr[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) T[i] = nr[i];
  }
}

// ---------------------------------------------------------------------------
// Full-rate zero-phase filter (lfd_internal.h FRConst): SciPy's TDF-II
// cascade, blocked.  k_fullrate_wave: one wave = one (channel, big block of
// FR_L samples); lane j owns the FR_LS-sample sub-block a + j*FR_LS.  Per
// lane, in registers:
//   1. TDF-II forward over the sub-block from zero state -> y0, exit A_j;
//   2. TDF-II over the reversed y0 from zero state -> r0 (outputs), exit Z0_j;
//   3. wave scan S_{j+1} = PhiP S_j + A_j (log-step over the lanes), S_0 =
//      the state entering the big block (SF; 0 for the functionals);
//   4. Z_j = Z0_j + M32 S_j, wave scan T_j = PhiP T_{j+1} + Z_j from the
//      right (T_64 = ST(k+1); 0 for the functionals);
//   5. (out) y[i] = r0[i] + Rh[i] S_j + H[31 - i] T_{j+1}  (linearity: the
//      forward state's and the reverse state's responses; fp64 MFMA).
// Functional mode writes e_f = S_64 and e_r = T_0.  Every recurrence runs in
// its own direction (stable for any pole radius) and in SciPy's coordinates.
// x comes through LDS (row loads; a 4-float pad per 32 keeps the lanes'
// float4 reads conflict-free) and y leaves through LDS as row stores.
// ---------------------------------------------------------------------------
typedef double fr_d4v __attribute__((ext_vector_type(4)));
// LFD_FR_STAGE_OLD=1 (A/B knob): the big block's loads in groups of 8 dwords
#ifdef LFD_DIAG
__constant__ int g_fr_stage_old = 0;
// LFD_FR_STAGGER (diag A/B): the output pass's first 4,096 waves sleep
// 0-3 x this many 2,048-cycle units (a hashed slot), so the waves sharing a
// SIMD do not run their load / scan / MFMA phases in lock step
__constant__ int g_fr_stagger = 0;
// LFD_FR_TIMES (diag): phase stamps of the output pass's first 16,384 waves
__device__ uint64_t g_fr_times[16384 * 8];
#define FR_STAMP(i)                                                                                   \
  do {                                                                                                \
    if (blockIdx.x < 16384) {                                                                         \
      const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                           \
      if (threadIdx.x == 0) g_fr_times[(size_t)blockIdx.x * 8 + (i)] = t_;                            \
    }                                                                                                 \
  } while (0)
// LFD_FRS_TIMES (diag): phase stamps of k_fullrate_scan_seg's first 256
// workgroups (thread 0, after each workgroup barrier)
__device__ uint64_t g_frs_times[256 * 8];
#define FRS_STAMP(i)                                                                                  \
  do {                                                                                                \
    if (blockIdx.x < 256 && threadIdx.x == 0) g_frs_times[(size_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define FR_STAMP(i) \
  do {              \
  } while (0)
#define FRS_STAMP(i) \
  do {               \
  } while (0)
#endif
#ifndef FRS_Q
// k_fullrate_scan: big blocks per load batch (8: 0.83 ms vs 0.91 at 4 on the
// 2,000 x 600,000 band-pass; a software-pipelined next batch spills and is
// slower, profiles/archive_r01_r03.md (r02_fullrate_scan_ab.txt))
#define FRS_Q 8
#endif
#ifndef FR_WAVES
#define FR_WAVES 4  // waves per SIMD the register budget targets (<= 128 VGPRs)
#endif

// Output stage of the full-rate wave kernel: y_j = r0_j + Q w_j with
// w_j = (S_j, T_{j+1}) and Q[i] = (Rh[i], H[31 - i]): the 32 x 2N by 2N x 64
// product on the fp64 matrix cores (v_mfma_f64_16x16x4: A = Q from
// FRConst::QA, B = w staged through LDS, C = r0 read back in the accumulator
// layout), two passes of 16 samples through a 64 x 16 LDS stage, rows of
// 128 B leaving as 16-B stores.  LDS rows of OSTR = 18 doubles (36 dwords =
// 4 x odd): the MFMA-layout accesses (16 rows x 4 adjacent doubles per
// instruction) hit distinct banks, and the row writes go out as 16-B
// ds_write_b128, conflict-free per 8 lanes (lane stride 36 dwords).
// nsb: sub-blocks (rows of 32 samples) whose outputs are stored (64 = all).
template <int NS>
__device__ __forceinline__ void fr_out_mfma(int lane, const FRConst *__restrict__ fc, const double (&Sj)[2 * NS],
                                            const double (&T)[2 * NS], const double (&r0)[FR_LS], double *lds,
                                            double *__restrict__ yr, int64_t ys_t, int nsb = 64) {
  constexpr int N = 2 * NS, LS = FR_LS, OSTR = 18;
  constexpr int K = 2 * N, KS = K / 4;
  const int col = lane & 15, q = lane >> 4;
  double *W = lds;  // [64][K], stride OSTR (the tile's reads are done: one wave, LDS in order)
#pragma unroll
  for (int n = 0; n < N; ++n) {
    W[lane * OSTR + n] = Sj[n];
    W[lane * OSTR + N + n] = T[n];
  }
  __syncthreads();
  double bop[KS][4], aop[2][KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) bop[ks][nt] = W[(16 * nt + col) * OSTR + 4 * ks + q];
    aop[0][ks] = fc->QA[0][ks][lane];
    aop[1][ks] = fc->QA[1][ks][lane];
  }
  __syncthreads();
  double *ob = lds;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
    for (int i = 0; i < 16; i += 2)
      *reinterpret_cast<double2 *>(ob + lane * OSTR + i) = double2{r0[16 * mt + i], r0[16 * mt + i + 1]};
    __syncthreads();
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      double *o = ob + (16 * nt + col) * OSTR + q;
      fr_d4v acc = {o[0], o[4], o[8], o[12]};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(aop[mt][ks], bop[ks][nt], acc, 0, 0, 0);
      o[0] = acc[0];
      o[4] = acc[1];
      o[8] = acc[2];
      o[12] = acc[3];
    }
    __syncthreads();
    if (ys_t == 1 && (reinterpret_cast<uintptr_t>(yr) & 15) == 0) {
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int r = it * 8 + (lane >> 3), c2 = 2 * (lane & 7);
        if (r < nsb)
          *reinterpret_cast<double2 *>(yr + r * LS + 16 * mt + c2) = *reinterpret_cast<const double2 *>(ob + r * OSTR + c2);
      }
    } else {
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int r = it * 4 + (lane >> 4), c = lane & 15;
        if (r < nsb) yr[(r * LS + 16 * mt + c) * ys_t] = ob[r * OSTR + c];
      }
    }
    __syncthreads();
  }
  FR_STAMP(5);
}

// One DPP lane move of a double inside 16-lane rows (both 32-bit halves;
// lanes whose source leaves the row read 0.0): row_shr:d = 0x110 + d,
// row_shl:d = 0x100 + d.
template <int CTRL>
__device__ __forceinline__ double dpp_row_d(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int l2 = __builtin_amdgcn_update_dpp(0, lo, CTRL, 0xf, 0xf, true);
  const int h2 = __builtin_amdgcn_update_dpp(0, hi, CTRL, 0xf, 0xf, true);
  return __hiloint2double(h2, l2);
}

// (big-block path, option fullrate_bigblock; the medium-block output pass
// is k_fullrate_out_mb)
template <int NS, bool OUT>
__global__ __launch_bounds__(64, FR_WAVES) void k_fullrate_wave(
    const float *__restrict__ x, int64_t s_ch, int64_t s_t, int64_t n_ch, int64_t nb,
    const FRConst *__restrict__ fc, const double *__restrict__ SF, const double *__restrict__ ST,
    double *__restrict__ F, double *__restrict__ y, int64_t ys_ch, int64_t ys_t) {
  constexpr int N = 2 * NS, LS = FR_LS, L = FR_L;
  static_assert(LS == 32, "tile reads assume 32-sample sub-blocks");
  constexpr int TLDS = L + 4 * (L / 32);
  // LDS row strides of 18 doubles (36 dwords = 4 x odd): the MFMA-layout
  // accesses (16 rows x 4 adjacent doubles per instruction) hit distinct banks
  constexpr int OSTR = 18;
  constexpr int NLDS = 64 * OSTR > TLDS / 2 ? 64 * OSTR : TLDS / 2;
  __shared__ __attribute__((aligned(16))) double lds[NLDS];
  float *tile = reinterpret_cast<float *>(lds);
  const int lane = threadIdx.x;
  const int col = lane & 15, q = lane >> 4;
  const int64_t ch = blockIdx.x / nb, k = blockIdx.x % nb;
  const int64_t a = k * L;
  {
    // every load of the big block issued before the first LDS write (8 KB
    // per wave in flight, one memory latency per block); time-contiguous,
    // 16-B aligned rows as float4 (1 KB per instruction)
    const float *row = x + ch * s_ch + a * s_t;
    if (s_t == 1 && (reinterpret_cast<uintptr_t>(row) & 15) == 0 && !LFD_DG(g_fr_stage_old)) {
      float4 v[L / 256];
#pragma unroll
      for (int i = 0; i < L / 256; ++i) v[i] = *reinterpret_cast<const float4 *>(row + 4 * lane + 256 * i);
#pragma unroll
      for (int i = 0; i < L / 256; ++i) {
        const int u = 4 * lane + 256 * i;
        *reinterpret_cast<float4 *>(tile + u + 4 * (u >> 5)) = v[i];
      }
    } else {
#pragma unroll 8
      for (int u = lane; u < L; u += 64) tile[u + 4 * (u >> 5)] = row[u * s_t];
    }
  }
  __syncthreads();
  FwdRec<NS> fr;
  fr.load(fc->cf);
  double r0[OUT ? LS : 1], A[N], Z[N];
  if constexpr (OUT) {
    // ---- 1, 2. zero-state forward, then zero-state reverse over its output
    float xs[LS];
    const float *tr = tile + 36 * lane;
#pragma unroll
    for (int g = 0; g < LS / 4; ++g) {
      const float4 v = *reinterpret_cast<const float4 *>(tr + 4 * g);
      xs[4 * g + 0] = v.x;
      xs[4 * g + 1] = v.y;
      xs[4 * g + 2] = v.z;
      xs[4 * g + 3] = v.w;
    }
#pragma unroll
    for (int n = 0; n < N; ++n) A[n] = Z[n] = 0.0;
#pragma unroll
    for (int i = 0; i < LS; ++i) r0[i] = fr.step(A, (double)xs[i]);
#pragma unroll
    for (int i = LS - 1; i >= 0; --i) r0[i] = fr.step(Z, r0[i]);
  } else {
    // ---- 1, 2 (functionals): only the exit states are needed, and they are
    // linear in the sub-block's samples: (A_j, Z0_j) = KAZ x_j, a 16 x 32 by
    // 32 x 64 product on the fp64 matrix cores (B = samples from the tile)
    fr_d4v acc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = fr_d4v{0.0, 0.0, 0.0, 0.0};
    const float *tb = tile + 36 * col + q;
#pragma unroll
    for (int ks = 0; ks < LS / 4; ++ks) {
      const double av = fc->KAZ[ks][lane];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, (double)tb[36 * 16 * nt + 4 * ks], acc[nt], 0, 0, 0);
    }
    __syncthreads();
    double *az = lds;  // [sub-block][functional], stride OSTR
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) az[(16 * nt + col) * OSTR + q + 4 * r] = acc[nt][r];
    __syncthreads();
#pragma unroll
    for (int n = 0; n < N; ++n) {
      A[n] = az[lane * OSTR + n];
      Z[n] = az[lane * OSTR + N + n];
    }
  }
  // the zero-input transition of a cascade is block lower-triangular (a
  // section's state never feeds an earlier section): PhiP skips those blocks
  auto matvec_add = [&](const double *P, const double (&o)[N], double (&v)[N], bool tri) {
#pragma unroll
    for (int r = 0; r < N; ++r) {
      double acc = v[r];
#pragma unroll
      for (int c = 0; c < N; ++c)
        if (!tri || c / 2 <= r / 2) acc = fma(P[r * MAX_N + c], o[c], acc);
      v[r] = acc;
    }
  };
  // ---- 3. forward wave scan
  double Sin[N], vf[N], Sj[N];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    Sin[n] = OUT ? SF[(k * N + n) * n_ch + ch] : 0.0;
    vf[n] = A[n];
  }
  if (OUT && lane == 0) matvec_add(fc->PhiP[0], Sin, vf, true);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int d = 1 << i;
    double o[N];
#pragma unroll
    for (int n = 0; n < N; ++n) o[n] = __shfl_up(vf[n], d);
    if (lane >= d) matvec_add(fc->PhiP[i], o, vf, true);
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const double u = __shfl_up(vf[n], 1);
    Sj[n] = lane == 0 ? Sin[n] : u;
  }
  // ---- 4. reverse exit with the true forward state, backward wave scan
  double vb[N], Tin[N];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    vb[n] = Z[n];
    Tin[n] = OUT ? ST[((k + 1) * N + n) * n_ch + ch] : 0.0;
  }
  matvec_add(fc->M32, Sj, vb, false);
  if (OUT && lane == 63) matvec_add(fc->PhiP[0], Tin, vb, true);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int d = 1 << i;
    double o[N];
#pragma unroll
    for (int n = 0; n < N; ++n) o[n] = __shfl_down(vb[n], d);
    if (lane + d < 64) matvec_add(fc->PhiP[i], o, vb, true);
  }
  if constexpr (!OUT) {
    if (lane == 63) {
#pragma unroll
      for (int n = 0; n < N; ++n) F[(k * 2 * N + n) * n_ch + ch] = vf[n];
    }
    if (lane == 0) {
#pragma unroll
      for (int n = 0; n < N; ++n) F[(k * 2 * N + N + n) * n_ch + ch] = vb[n];
    }
    return;
  }
  // ---- 5. outputs y_j = r0_j + Q w_j, w_j = (S_j, T_{j+1}), Q[i] = (Rh[i],
  // H[31 - i]): the 32 x 2N by 2N x 64 product runs on the fp64 matrix cores
  // (v_mfma_f64_16x16x4: A = Q from FRConst::QA, B = w staged through LDS,
  // C = r0 read back in the accumulator layout)
  double T[N];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const double u = __shfl_down(vb[n], 1);
    T[n] = lane == 63 ? Tin[n] : u;
  }
  if constexpr (OUT) fr_out_mfma<NS>(lane, fc, Sj, T, r0, lds, y + ch * ys_ch + a * ys_t, ys_t);
}

// 4 x 4 transpose across the 16-lane rows of a wave: register c of row R
// becomes register R of row c (v[c] at row R = E[R][c]  ->  v[c] at row R =
// E[c][R]); two v_permlane32_swap then two v_permlane16_swap per 32-bit half
// (VALU lane exchanges, no LDS).  permlane32_swap(a, b) swaps a's rows 2, 3
// with b's rows 0, 1; permlane16_swap(a, b) swaps a's odd rows with b's even
// rows (tools/check_permlane.hip).
__device__ __forceinline__ void swap32_d(double &a, double &b) {
  const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)__double2loint(a), (uint32_t)__double2loint(b), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)__double2hiint(a), (uint32_t)__double2hiint(b), false, false);
  a = __hiloint2double((int)hi[0], (int)lo[0]);
  b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void swap16_d(double &a, double &b) {
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)__double2loint(a), (uint32_t)__double2loint(b), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)__double2hiint(a), (uint32_t)__double2hiint(b), false, false);
  a = __hiloint2double((int)hi[0], (int)lo[0]);
  b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void rows_transpose4(double &v0, double &v1, double &v2, double &v3) {
  swap32_d(v0, v2);
  swap32_d(v1, v3);
  swap16_d(v0, v1);
  swap16_d(v2, v3);
}

// one k-step of A (this lane's 16x16x4 A value) against four column tiles
// (the 4x4x4_4b form of the same products measured slower,
// profiles/archive_r01_r03.md (r02_ubench_mfma64b.txt))
__device__ __forceinline__ void mfma_k4(double av, const double (&b)[4], fr_d4v (&acc)[4]) {
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) acc[nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b[nt], acc[nt], 0, 0, 0);
}

// ---------------------------------------------------------------------------
// k_fullrate_out_mb — output pass of the medium-block full-rate path, with no
// fp64 recurrence at all: one wave = one big block (FR_L samples, the last
// one partial), lane = 32-sample sub-block, 16-lane row = medium block with
// its entering states SF[m] / ST[m + 1] from k_fullrate_scan_seg.
//   1. (A_j, Z0_j) = KAZ x_j (fp64 MFMA, B from the LDS tile), to the lanes
//      by a permlane transpose;
//   2. row scans on DPP: S_j (forward), T_{j+1} (reverse, with Z + M32 S_j);
//   3. y = Kr x + Q (S_j, T_{j+1}): the zero-state response of the sub-block
//      AND the state responses as fp64 MFMA products into one accumulator
//      (A = KRA / QA tables, B = the tile / the states transposed by permlane),
//      staged through the tile's LDS into rows and stored as 16-B pieces.
// The round-3 output pass ran the zero-state responses as TDF-II recurrences
// (40 fp64 FMAs per sample on the VALU: the pass was fp64-issue bound).
// The tile's sub-block rows are 36 floats apart, written as 16-B pieces; the
// entering states SF / ST load at the kernel start with the tile, so their
// latency hides behind the tile's and the KAZ products (3.92 vs 3.98 ms
// loading them at the scans, profiles/r04ao_fr_ab_early_states.txt).
// (Measured and removed, records in profiles/: stores straight from the MFMA
// layout, the bank-conflict-free 34-float layout — 2.5x fewer LDS conflicts,
// 1 % slower, profiles/r04h_fr_ab_lds_layout.txt — 4x4x4_4b products, the KAZ
// column preloaded.)
template <int NS>
__global__ __launch_bounds__(64, FR_WAVES) void k_fullrate_out_mb(
    const float *__restrict__ x, int64_t s_ch, int64_t n_ch, int64_t nb, int64_t n_mb,
    const FRConst *__restrict__ fc, const double *__restrict__ SF, const double *__restrict__ ST,
    double *__restrict__ y, int64_t ys_ch, int64_t ys_t, int ord = 0) {
  constexpr int N = 2 * NS, LS = FR_LS, L = FR_L, K = 2 * N, KS = K / 4, OSTR = 18;
  static_assert(N % 2 == 0 && K % 4 == 0, "state components in groups of 4");
  // LDS: the tile's sub-block rows TS = 36 floats apart (float4 staging
  // writes); the output stage's rows OSTR = 18 doubles apart (MFMA-layout
  // 8-B writes: 36 col + 2 q distinct mod 64 per half wave)
  constexpr int TS = 36;
  constexpr int TLDS = 64 * TS;
  constexpr int NLDS = 64 * OSTR > TLDS / 2 ? 64 * OSTR : TLDS / 2;
  __shared__ __attribute__((aligned(16))) double lds[NLDS];
  float *tile = reinterpret_cast<float *>(lds);
  const int lane = threadIdx.x;
  const int col = lane & 15, q = lane >> 4, jr = lane & 15;
  // ord: 0 = channel-major (consecutive groups = consecutive big blocks of
  // one channel); 1 = block-major (consecutive groups = the same big block of
  // consecutive channels, whose SF / ST entries share cache lines); 2
  // (production) = block-major with the groups of one XCD contiguous: HBM
  // reads 9.55 -> 5.08 GB per launch at 2,000 x 600,000 (x 4.8 GB + SF / ST
  // 0.3 GB algorithmic; channel-major re-fetched each 128-B line of states
  // once per channel), 3.89 -> 3.84 ms (profiles/r04au_fr_ab_block_order.txt)
  FR_STAMP(0);
#ifdef LFD_DIAG
  if (g_fr_stagger && blockIdx.x < 4096) {
    const int slot = (int)(((uint32_t)blockIdx.x * 2654435761u) >> 30);
    for (int i = 0; i < slot * g_fr_stagger; ++i) __builtin_amdgcn_s_sleep(32);
  }
#endif
  int64_t bid = blockIdx.x;
  if (ord == 2 && (gridDim.x & 7) == 0) bid = (bid & 7) * (gridDim.x >> 3) + (bid >> 3);
  const int64_t ch = ord ? bid % n_ch : bid / nb, k = ord ? bid / n_ch : bid % nb;
  const int64_t a = k * L;
  const int nvs = (int)(n_mb - 4 * k < 4 ? (n_mb - 4 * k) * FR_LB : L);
  const int64_t m_row = 4 * k + (lane >> 4);
  const int64_t m = m_row < n_mb ? m_row : n_mb - 1;  // rows past the last medium block: any valid state
  double SinE[N], TinE[N];
  {
    // wave-uniform bases (medium block 4k) + one 32-bit per-lane byte offset
    // (the row's m - 4k < 4): scalar-base loads, no 64-bit address per load
    const double *sfb = SF + 4 * k * N * n_ch + ch, *stb = ST + (4 * k + 1) * N * n_ch + ch;
    const uint32_t vo = (uint32_t)(m - 4 * k) * (uint32_t)(N * n_ch) * 8u;
#pragma unroll
    for (int n = 0; n < N; ++n) {
      SinE[n] = *reinterpret_cast<const double *>(reinterpret_cast<const char *>(sfb + n * n_ch) + vo);
      TinE[n] = *reinterpret_cast<const double *>(reinterpret_cast<const char *>(stb + n * n_ch) + vo);
    }
  }
  {
    const float *row = x + ch * s_ch + a;
    if (nvs < L) {
#pragma unroll 8
      for (int u = lane; u < L; u += 64) tile[(u >> 5) * TS + (u & 31)] = u < nvs ? row[u] : 0.0f;
    } else {
      // (rows need not be 16-B aligned: f4u pieces)
      f4v v[L / 256];
#pragma unroll
      for (int i = 0; i < L / 256; ++i) v[i] = *reinterpret_cast<const f4u *>(row + 4 * lane + 256 * i);
#pragma unroll
      for (int i = 0; i < L / 256; ++i) {
        const int u = 4 * lane + 256 * i;
        *reinterpret_cast<f4v *>(tile + u + 4 * (u >> 5)) = v[i];
      }
    }
  }
  __syncthreads();
  FR_STAMP(1);
  const float *tb = tile + TS * col + q;  // B[k = q][j = col] of tile nt, k-step ks: tb[TS*16*nt + 4*ks]
  // ---- 1. sub-block exits on the matrix cores
  double A[N], Z[N];
  {
    fr_d4v acc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = fr_d4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < LS / 4; ++ks) {
      const double av = fc->KAZ[ks][lane];
      double bk[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) bk[nt] = (double)tb[TS * 16 * nt + 4 * ks];
      mfma_k4(av, bk, acc);
    }
    // acc[nt][r] at row q = functional q + 4r of sub-block 16 nt + col: per r,
    // transpose (row q <-> register nt) -> at row R, register q' = functional
    // q' + 4r of this lane's sub-block 16 R + col
    double f[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double v0 = acc[0][r], v1 = acc[1][r], v2 = acc[2][r], v3 = acc[3][r];
      rows_transpose4(v0, v1, v2, v3);
      f[r][0] = v0;
      f[r][1] = v1;
      f[r][2] = v2;
      f[r][3] = v3;
    }
#pragma unroll
    for (int n = 0; n < N; ++n) {
      A[n] = f[n / 4][n % 4];
      Z[n] = f[(N + n) / 4][(N + n) % 4];
    }
  }
  FR_STAMP(2);
  auto matvec_add = [&](const double *P, const double (&o)[N], double (&v)[N], bool tri) {
#pragma unroll
    for (int r = 0; r < N; ++r) {
      double acc = v[r];
#pragma unroll
      for (int c = 0; c < N; ++c)
        if (!tri || c / 2 <= r / 2) acc = fma(P[r * MAX_N + c], o[c], acc);
      v[r] = acc;
    }
  };
  // ---- 2. row scans (row = medium block m, lane jr = its sub-block)
  double W[K];  // (S_j, T_{j+1})
  {
    double Sin[N], vf[N];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      Sin[n] = SinE[n];
      vf[n] = A[n];
    }
    if (jr == 0) matvec_add(fc->PhiP[0], Sin, vf, true);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      double o[N];
#pragma unroll
      for (int n = 0; n < N; ++n) {
        if (i == 0) o[n] = dpp_row_d<0x111>(vf[n]);
        if (i == 1) o[n] = dpp_row_d<0x112>(vf[n]);
        if (i == 2) o[n] = dpp_row_d<0x114>(vf[n]);
        if (i == 3) o[n] = dpp_row_d<0x118>(vf[n]);
      }
      matvec_add(fc->PhiP[i], o, vf, true);  // lanes without a source add PhiP 0
    }
    double vb[N];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const double u = dpp_row_d<0x111>(vf[n]);
      W[n] = jr == 0 ? Sin[n] : u;
      vb[n] = Z[n];
    }
    double Sj[N];
#pragma unroll
    for (int n = 0; n < N; ++n) Sj[n] = W[n];
    matvec_add(fc->M32, Sj, vb, false);
    double Tin[N];
#pragma unroll
    for (int n = 0; n < N; ++n) Tin[n] = TinE[n];
    if (jr == 15) matvec_add(fc->PhiP[0], Tin, vb, true);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      double o[N];
#pragma unroll
      for (int n = 0; n < N; ++n) {
        if (i == 0) o[n] = dpp_row_d<0x101>(vb[n]);
        if (i == 1) o[n] = dpp_row_d<0x102>(vb[n]);
        if (i == 2) o[n] = dpp_row_d<0x104>(vb[n]);
        if (i == 3) o[n] = dpp_row_d<0x108>(vb[n]);
      }
      matvec_add(fc->PhiP[i], o, vb, true);
    }
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const double u = dpp_row_d<0x101>(vb[n]);
      W[N + n] = jr == 15 ? Tin[n] : u;
    }
  }
  FR_STAMP(3);
  // ---- 3. y = Kr x + Q w on the matrix cores
  // state product first (W dies as it is consumed), then Kr x from the tile.
  // B operand of the state product: k-step ks, tile nt at row q =
  // W_{sub-block 16 nt + col}[4 ks + q]: per ks a row transpose of W[4ks..]
  fr_d4v yacc[2][4];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) yacc[mt][nt] = fr_d4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    double bop[4] = {W[4 * ks], W[4 * ks + 1], W[4 * ks + 2], W[4 * ks + 3]};
    rows_transpose4(bop[0], bop[1], bop[2], bop[3]);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      mfma_k4(fc->QA[mt][ks][lane], bop, yacc[mt]);
    }
  }
#pragma unroll
  for (int ks = 0; ks < LS / 4; ++ks) {
    double bx[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) bx[nt] = (double)tb[TS * 16 * nt + 4 * ks];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      mfma_k4(fc->KRA[mt][ks][lane], bx, yacc[mt]);
    }
  }
  FR_STAMP(4);
  double *yr = y + ch * ys_ch + a * ys_t;
  const int nsb = nvs / LS;
  __syncthreads();  // the tile's reads are done: its LDS becomes the output stage
  double *ob = lds;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    // yacc[mt][nt][r] = y[sample 16 mt + q + 4 r] of sub-block 16 nt + col
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      double *o = ob + (16 * nt + col) * OSTR + q;
      o[0] = yacc[mt][nt][0];
      o[4] = yacc[mt][nt][1];
      o[8] = yacc[mt][nt][2];
      o[12] = yacc[mt][nt][3];
    }
    __syncthreads();
    if (ys_t == 1 && nsb == 64) {  // whole big block: no per-piece bounds, one base per lane
      double *yp = yr + (lane >> 3) * LS + 16 * mt + 2 * (lane & 7);
      const double *op = ob + (lane >> 3) * OSTR + 2 * (lane & 7);
#pragma unroll
      for (int it = 0; it < 8; ++it)
        *reinterpret_cast<d2u *>(yp + it * 8 * LS) = *reinterpret_cast<const d2u *>(op + it * 8 * OSTR);
    } else if (ys_t == 1) {  // 16-B pieces, 8-B aligned on rows of odd length (d2u)
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int r = it * 8 + (lane >> 3), c2 = 2 * (lane & 7);
        if (r < nsb)
          *reinterpret_cast<d2u *>(yr + r * LS + 16 * mt + c2) = *reinterpret_cast<const d2u *>(ob + r * OSTR + c2);
      }
    } else {
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int r = it * 4 + (lane >> 4), c = lane & 15;
        if (r < nsb) yr[(r * LS + 16 * mt + c) * ys_t] = ob[r * OSTR + c];
      }
    }
    __syncthreads();
  }
}

// k_fullrate_scan: one thread per channel.  SciPy's left edge (odd extension,
// zi * ext[0]) -> S_f at every big block start -> the tail + right pad
// forward (TP) -> reverse from zi * y_f[-1] over pad + tail, writing the
// tail's outputs -> T at every big block start, backward.
template <int NS>
__global__ __launch_bounds__(64) void k_fullrate_scan(
    const float *__restrict__ x, int64_t s_ch, int64_t s_t, int64_t n_ch, int64_t n_t, int64_t nb, int padlen,
    const FRConst *__restrict__ fc, const double *__restrict__ F, double *__restrict__ SF,
    double *__restrict__ ST, double *__restrict__ TP, double *__restrict__ y, int64_t ys_ch, int64_t ys_t) {
  constexpr int N = 2 * NS;
  // PhiL and M (read every step) live in LDS: too many for SGPRs
  __shared__ double cPL[N * N], cMM[N * N];
  for (int i = threadIdx.x; i < N * N; i += blockDim.x) {
    cPL[i] = fc->PhiL[(i / N) * MAX_N + i % N];
    cMM[i] = fc->M[(i / N) * MAX_N + i % N];
  }
  __syncthreads();
  const int64_t ch = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= n_ch) return;
  FwdRec<NS> fr;
  fr.load(fc->cf);
  const float *xc = x + ch * s_ch;
  const int E = padlen;
  const float x0 = xc[0], xn = xc[(n_t - 1) * s_t];
  auto ext = [&](int64_t t) -> double {  // scipy odd extension, float32 like numpy
    if (t < E) return (double)(2.0f * x0 - xc[(E - t) * s_t]);
    if (t < E + n_t) return (double)xc[(t - E) * s_t];
    return (double)(2.0f * xn - xc[(n_t - 2 - (t - E - n_t)) * s_t]);
  };
  double z[N];
  {
    const double e0 = ext(0);
#pragma unroll
    for (int i = 0; i < N; ++i) z[i] = fc->zi.v[i] * e0;
  }
  for (int64_t t = 0; t < E; ++t) (void)fr.step(z, ext(t));
  // The walks below are latency-bound (one thread per channel): full batches
  // of Q blocks / B samples load before they are applied, the next batch's
  // loads in flight; the remainders run one step at a time.
  constexpr int Q = FRS_Q, B = 8;
  const double *PL = cPL, *MM = cMM;
  auto mv = [&](const double *P, const double (&v)[N], double (&o)[N], bool tri) {
    asm volatile("" ::: "memory");  // re-read P from LDS (hoisted, 2 x N*N doubles spill)
#pragma unroll
    for (int r = 0; r < N; ++r) {
      double acc = o[r];
#pragma unroll
      for (int c = 0; c < N; ++c)
        if (!tri || c / 2 <= r / 2) acc = fma(P[r * N + c], v[c], acc);
      o[r] = acc;
    }
  };
  auto fwd_block = [&](int64_t k, double (&f)[N]) {
#pragma unroll
    for (int n = 0; n < N; ++n) SF[(k * N + n) * n_ch + ch] = z[n];
    mv(PL, z, f, true);
#pragma unroll
    for (int n = 0; n < N; ++n) z[n] = f[n];
  };
  // ---- forward over the big blocks
  const int64_t nbq = nb / Q * Q;
  for (int64_t k0 = 0; k0 < nbq; k0 += Q) {
    double fq[Q][N];
#pragma unroll
    for (int u = 0; u < Q; ++u)
#pragma unroll
      for (int n = 0; n < N; ++n) fq[u][n] = F[((k0 + u) * 2 * N + n) * n_ch + ch];
#pragma unroll
    for (int u = 0; u < Q; ++u) fwd_block(k0 + u, fq[u]);
  }
  for (int64_t k = nbq; k < nb; ++k) {
    double f[N];
#pragma unroll
    for (int n = 0; n < N; ++n) f[n] = F[(k * 2 * N + n) * n_ch + ch];
    fwd_block(k, f);
  }
  // ---- tail samples [nb * FR_L, n_t), forward
  const int64_t t_tail = nb * FR_L;  // sample index (ext index + E)
  double *tp = TP + ch;
  double yl = 0.0;
  {
    const int64_t nt = n_t - t_tail, ntb = nt / B * B;
    const float *xt = xc + t_tail * s_t;
    for (int64_t i0 = 0; i0 < ntb; i0 += B) {
      float xv[B];
#pragma unroll
      for (int u = 0; u < B; ++u) xv[u] = xt[(i0 + u) * s_t];
#pragma unroll
      for (int u = 0; u < B; ++u) {
        yl = fr.step(z, (double)xv[u]);
        tp[(i0 + u) * n_ch] = yl;
      }
    }
    for (int64_t i = ntb; i < nt; ++i) {
      yl = fr.step(z, (double)xt[i * s_t]);
      tp[i * n_ch] = yl;
    }
    // right pad (odd extension)
    for (int64_t i = 0; i < E; ++i) {
      yl = fr.step(z, (double)(2.0f * xn - xc[(n_t - 2 - i) * s_t]));
      tp[(nt + i) * n_ch] = yl;
    }
  }
  // ---- reverse over pad + tail
#pragma unroll
  for (int i = 0; i < N; ++i) z[i] = fc->zi.v[i] * yl;
  {
    const int64_t nt = n_t - t_tail, ntp = nt + E;
    for (int64_t i = ntp - 1; i >= nt; --i) (void)fr.step(z, tp[i * n_ch]);
    double *yt = y + ch * ys_ch + t_tail * ys_t;
    const int64_t r = nt % B;  // the tail's last r samples one at a time, then full batches
    for (int64_t i = nt - 1; i >= nt - r; --i) yt[i * ys_t] = fr.step(z, tp[i * n_ch]);
    for (int64_t i1 = nt - r - 1; i1 >= 0; i1 -= B) {
      double tv[B];
#pragma unroll
      for (int u = 0; u < B; ++u) tv[u] = tp[(i1 - u) * n_ch];
#pragma unroll
      for (int u = 0; u < B; ++u) yt[(i1 - u) * ys_t] = fr.step(z, tv[u]);
    }
  }
  // ---- reverse over the big blocks
#pragma unroll
  for (int n = 0; n < N; ++n) ST[(nb * N + n) * n_ch + ch] = z[n];
  auto bwd_block = [&](int64_t k, double (&f)[N], const double (&sf)[N]) {
    mv(PL, z, f, true);
    mv(MM, sf, f, false);
#pragma unroll
    for (int n = 0; n < N; ++n) {
      z[n] = f[n];
      ST[(k * N + n) * n_ch + ch] = z[n];
    }
  };
  const int64_t rb = nb % Q;
  for (int64_t k = nb - 1; k >= nb - rb; --k) {
    double f[N], sf[N];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      f[n] = F[(k * 2 * N + N + n) * n_ch + ch];
      sf[n] = SF[(k * N + n) * n_ch + ch];
    }
    bwd_block(k, f, sf);
  }
  for (int64_t k1 = nb - rb - 1; k1 >= 0; k1 -= Q) {
    double fq[Q][N], sq[Q][N];
#pragma unroll
    for (int u = 0; u < Q; ++u)
#pragma unroll
      for (int n = 0; n < N; ++n) {
        fq[u][n] = F[((k1 - u) * 2 * N + N + n) * n_ch + ch];
        sq[u][n] = SF[((k1 - u) * N + n) * n_ch + ch];
      }
#pragma unroll
    for (int u = 0; u < Q; ++u) bwd_block(k1 - u, fq[u], sq[u]);
  }
}

// ---------------------------------------------------------------------------
// k_fullrate_scan_seg: the scan over MEDIUM blocks (FR_LB samples, 4 per big
// block) whose functionals the matrix-core pass wrote (F2, f_index layout:
// 16 channels contiguous per (block, component); components 0..N-1 = A, the
// forward exit from zero state, N..2N-1 = Z, the zero-state reverse exit of
// the zero-state forward output).  One workgroup = 16 channels x G segments
// of seglen medium blocks (G <= 32; lane = channel, 4 segments per wave):
//   A  each segment's forward aggregate from zero state
//   -> entering states E_s = pseg E_{s-1} + agg_{s-1}, E_0 = SciPy's left edge
//   C  the true S_f at every medium block (SFm); M = (n_t - 1) / FR_LB medium
//      blocks (the tail keeps < FR_LB + 1 samples: the output pass covers
//      the medium blocks past the last whole big block as a partial one);
//      the last segment continues over the tail and right pad and returns
//      from zi * y_f[-1] (T_end, the tail's outputs)
//   A' each segment's reverse aggregate from zero T: T <- PhiB T + Z + MB S_f
//   -> entering T from the right, C' the true T at every medium block (STm).
// The output pass (k_fullrate_out_mb) reads SFm / STm per row.
// 16 x G threads per channel group instead of one thread per channel walking
// every block: the walks are G times shorter (latency-bound chains).
// Edge windows in LDS (xl > 0): the workgroup stages the record's last xl
// samples (tail + what the right pad reflects) and first E + 1 samples of its
// channels at the start, and the tail's forward outputs stay in LDS, so the
// serial edge walks (left pad; tail + right pad forward, then reverse) read
// LDS instead of waiting one global latency per batch of samples (2,000 x
// 600,000, tail 448: 0.484 -> 0.392 ms; profiles/r04ah_fr_scan_lds_edges.txt).
// xl = 0 (windows too large for LDS, or diag knob LFD_FR_TAIL_GLOBAL): the
// global-memory walks through TP.  (Batches of 6 / 3 blocks in the walks
// instead of 4 / 2 measured the same: 0.391 ms.)
template <int NS, int CW = 16>
__global__ __launch_bounds__(512) void k_fullrate_scan_seg(
    const float *__restrict__ x, int64_t s_ch, int64_t s_t, int64_t n_ch, int64_t n_t, int64_t M, int padlen,
    const FRConst *__restrict__ fc, const double *__restrict__ F2, double *__restrict__ SFm,
    double *__restrict__ STm, double *__restrict__ TP, double *__restrict__ y, int64_t ys_ch, int64_t ys_t,
    FRSeg sg, int xl) {
  constexpr int N = 2 * NS;
  __shared__ double cPB[N * N], cMB[N * N], cPS[N * N], cPT[N * N];
  static_assert(CW == 16 || CW == 8, "16 or 8 channels per workgroup");
  __shared__ double slotL[CW][N], slotR[CW][N];
  extern __shared__ double agg[];  // [G][CW][N]
  const int tid = threadIdx.x, col = tid % CW, seg = tid / CW;
  FRS_STAMP(0);
  for (int i = tid; i < N * N; i += blockDim.x) {
    const int r = i / N, c = i % N;
    cPB[i] = fc->PhiP[4][r * MAX_N + c];
    cMB[i] = fc->MB[r * MAX_N + c];
    cPS[i] = sg.pseg[r * MAX_N + c];
    cPT[i] = sg.plast[r * MAX_N + c];
  }
  const int E = padlen;
  const int64_t nt_tail = n_t - M * FR_LB;  // tail samples (1 .. FR_LB)
  // LDS windows after agg: tail outputs yw [nt + E][CW] (double), samples
  // xw [xl][CW] (the record's last xl), head xh [E + 1][CW]
  double *yw = agg + (size_t)sg.G * CW * N;
  float *xw = reinterpret_cast<float *>(yw + (size_t)(nt_tail + E) * CW);
  float *xh = xw + (size_t)xl * CW;
  const int64_t lo_w = n_t - xl;
  if (xl > 0) {
    const int64_t c_base = (int64_t)blockIdx.x * CW;
    for (int i = tid; i < CW * xl; i += blockDim.x) {
      const int c = i / xl, t = i - c * xl;  // consecutive threads: consecutive samples
      const int64_t chn = c_base + c < n_ch ? c_base + c : n_ch - 1;
      xw[t * CW + c] = x[chn * s_ch + (lo_w + t) * s_t];
    }
    for (int i = tid; i < CW * (E + 1); i += blockDim.x) {
      const int c = i / (E + 1), t = i - c * (E + 1);
      const int64_t chn = c_base + c < n_ch ? c_base + c : n_ch - 1;
      xh[t * CW + c] = x[chn * s_ch + t * s_t];
    }
  }
  __syncthreads();
  FRS_STAMP(1);
  const int64_t ch = (int64_t)blockIdx.x * CW + col;
  const bool active = ch < n_ch;
  const int64_t m0 = (int64_t)seg * sg.seglen;
  const int64_t m1 = m0 + sg.seglen < M ? m0 + sg.seglen : M;
  const bool live = active && seg < sg.Gu;
  const int64_t chc = active ? ch : n_ch - 1;
  const double *Fc = F2 + ((chc >> 4) * M * 2 * N) * 16 + (chc & 15);  // + (m * 2N + c) * 16
  FwdRec<NS> fr;
  fr.load(fc->cf);
  auto mv = [&](const double *P, const double (&v)[N], double (&o)[N], bool tri) {
    asm volatile("" ::: "memory");  // matrices re-read from LDS, not held in registers
#pragma unroll
    for (int r = 0; r < N; ++r) {
      double acc = o[r];
#pragma unroll
      for (int c = 0; c < N; ++c)
        if (!tri || c / 2 <= r / 2) acc = fma(P[r * N + c], v[c], acc);
      o[r] = acc;
    }
  };
  double *ag = agg + ((size_t)seg * CW + col) * N;
  // Every walk runs through a ring of QF (forward) / QR (reverse) block
  // slots loaded at clamped indices (unconditional loads: a conditional load
  // made the compiler wait for everything in flight); a slot is applied in
  // place and refilled with the block QF / QR ahead, so the chain waits one
  // memory latency per walk rather than per batch (round 6; the batched form
  // waited once per QF / QR blocks).
  constexpr int QF = 4, QR = 4;
  auto fload = [&](int64_t m, int c0, double (&f)[N]) {
#pragma unroll
    for (int n = 0; n < N; ++n) f[n] = Fc[(m * 2 * N + c0 + n) * 16];
  };
  // ---- A: forward aggregate of the segment from zero state
  double a[N];
#pragma unroll
  for (int n = 0; n < N; ++n) a[n] = 0.0;
  if (live) {
    // ring of QF slots: slot u is applied in place, then refilled with the
    // block QF ahead (clamped), so QF - 1 blocks' loads stay in flight
    double fq[QF][N];
#pragma unroll
    for (int u = 0; u < QF; ++u) fload(m0 + u < m1 ? m0 + u : m1 - 1, 0, fq[u]);
    for (int64_t mb = m0; mb < m1; mb += QF) {
#pragma unroll
      for (int u = 0; u < QF; ++u) {
        const int64_t m = mb + u;
        if (m >= m1) break;
        mv(cPB, a, fq[u], true);
#pragma unroll
        for (int n = 0; n < N; ++n) a[n] = fq[u][n];
        fload(m + QF < m1 ? m + QF : m1 - 1, 0, fq[u]);
      }
    }
  }
#pragma unroll
  for (int n = 0; n < N; ++n) ag[n] = a[n];
  const float *xc = x + chc * s_ch;
  // sample t of this channel: from the LDS windows when staged
  auto xhead = [&](int64_t t) { return xl > 0 ? xh[t * CW + col] : xc[t * s_t]; };
  auto xend = [&](int64_t t) { return xl > 0 ? xw[(t - lo_w) * CW + col] : xc[t * s_t]; };
  const float x0 = xhead(0), xn = xend(n_t - 1);
  if (active && seg == 0) {  // SciPy's left edge: zi * ext[0], then the odd extension
    double z[N];
    const double e0 = (double)(2.0f * x0 - xhead(E));
#pragma unroll
    for (int i = 0; i < N; ++i) z[i] = fc->zi.v[i] * e0;
    for (int t = 0; t < E; ++t) (void)fr.step(z, (double)(2.0f * x0 - xhead(E - t)));
#pragma unroll
    for (int n = 0; n < N; ++n) slotL[col][n] = z[n];
  }
  __syncthreads();
  FRS_STAMP(2);
  // ---- entering state of the segment
  double z[N];
#pragma unroll
  for (int n = 0; n < N; ++n) z[n] = slotL[col][n];
  for (int sp = 0; sp < seg && sp < sg.Gu; ++sp) {
    double o[N];
    const double *as = agg + ((size_t)sp * CW + col) * N;
#pragma unroll
    for (int n = 0; n < N; ++n) o[n] = as[n];
    mv(cPS, z, o, true);
#pragma unroll
    for (int n = 0; n < N; ++n) z[n] = o[n];
  }
  // ---- C: true forward states
  if (live) {
    double fq[QF][N];
#pragma unroll
    for (int u = 0; u < QF; ++u) fload(m0 + u < m1 ? m0 + u : m1 - 1, 0, fq[u]);
    for (int64_t mb = m0; mb < m1; mb += QF) {
#pragma unroll
      for (int u = 0; u < QF; ++u) {
        const int64_t m = mb + u;
        if (m >= m1) break;
#pragma unroll
        for (int n = 0; n < N; ++n) SFm[(m * N + n) * n_ch + ch] = z[n];
        mv(cPB, z, fq[u], true);
#pragma unroll
        for (int n = 0; n < N; ++n) z[n] = fq[u][n];
        fload(m + QF < m1 ? m + QF : m1 - 1, 0, fq[u]);
      }
    }
    if (seg == sg.Gu - 1 && xl > 0) {
      // (LDS windows) tail [M FR_LB, n_t) + right pad forward into yw, then
      // the reverse from zi * y_f[-1] over pad + tail (the tail's outputs)
      const int64_t t_tail = M * FR_LB, nt = nt_tail;
      double yl = 0.0;
      for (int64_t i = 0; i < nt; ++i) {
        yl = fr.step(z, (double)xend(t_tail + i));
        yw[i * CW + col] = yl;
      }
      for (int64_t i = 0; i < E; ++i) {
        yl = fr.step(z, (double)(2.0f * xn - xend(n_t - 2 - i)));
        yw[(nt + i) * CW + col] = yl;
      }
#pragma unroll
      for (int i = 0; i < N; ++i) z[i] = fc->zi.v[i] * yl;
      for (int64_t i = nt + E - 1; i >= nt; --i) (void)fr.step(z, yw[i * CW + col]);
      double *yt = y + ch * ys_ch + t_tail * ys_t;
      for (int64_t i = nt - 1; i >= 0; --i) yt[i * ys_t] = fr.step(z, yw[i * CW + col]);
#pragma unroll
      for (int n = 0; n < N; ++n) {
        slotR[col][n] = z[n];
        STm[(M * N + n) * n_ch + ch] = z[n];
      }
    } else if (seg == sg.Gu - 1) {
      // tail samples [M FR_LB, n_t) and the right pad forward (TP), then the
      // reverse from zi * y_f[-1] over pad + tail (the tail's outputs); the
      // reverse re-reads TP in batches of B (one latency per batch)
      constexpr int B = 8;
      const int64_t t_tail = M * FR_LB, nt = n_t - t_tail;
      double *tp = TP + ch;
      const float *xt = xc + t_tail * s_t;
      double yl = 0.0;
      for (int64_t i0 = 0; i0 < nt; i0 += B) {
        float xv[B];
#pragma unroll
        for (int u = 0; u < B; ++u) xv[u] = xt[(i0 + u < nt ? i0 + u : nt - 1) * s_t];
#pragma unroll
        for (int u = 0; u < B; ++u)
          if (i0 + u < nt) {
            yl = fr.step(z, (double)xv[u]);
            tp[(i0 + u) * n_ch] = yl;
          }
      }
      for (int64_t i = 0; i < E; ++i) {
        yl = fr.step(z, (double)(2.0f * xn - xc[(n_t - 2 - i) * s_t]));
        tp[(nt + i) * n_ch] = yl;
      }
#pragma unroll
      for (int i = 0; i < N; ++i) z[i] = fc->zi.v[i] * yl;
      for (int64_t i = nt + E - 1; i >= nt; --i) (void)fr.step(z, tp[i * n_ch]);
      double *yt = y + ch * ys_ch + t_tail * ys_t;
      for (int64_t i1 = nt - 1; i1 >= 0; i1 -= B) {
        double tv[B];
#pragma unroll
        for (int u = 0; u < B; ++u) tv[u] = tp[(i1 - u >= 0 ? i1 - u : 0) * n_ch];
#pragma unroll
        for (int u = 0; u < B; ++u)
          if (i1 - u >= 0) yt[(i1 - u) * ys_t] = fr.step(z, tv[u]);
      }
#pragma unroll
      for (int n = 0; n < N; ++n) {
        slotR[col][n] = z[n];
        STm[(M * N + n) * n_ch + ch] = z[n];
      }
    }
  }
  __syncthreads();
  FRS_STAMP(3);
  // ---- A': reverse aggregate of the segment from zero T (true S_f coupling)
  auto rload = [&](int64_t m, double (&f)[N], double (&sf)[N]) {
    fload(m, N, f);
#pragma unroll
    for (int n = 0; n < N; ++n) sf[n] = SFm[(m * N + n) * n_ch + ch];
  };
#pragma unroll
  for (int n = 0; n < N; ++n) a[n] = 0.0;
  if (live) {
    double fq[QR][N], sq[QR][N];
#pragma unroll
    for (int u = 0; u < QR; ++u) rload(m1 - 1 - u >= m0 ? m1 - 1 - u : m0, fq[u], sq[u]);
    for (int64_t mb = m1 - 1; mb >= m0; mb -= QR) {
#pragma unroll
      for (int u = 0; u < QR; ++u) {
        const int64_t m = mb - u;
        if (m < m0) break;
        mv(cPB, a, fq[u], true);
        mv(cMB, sq[u], fq[u], false);
#pragma unroll
        for (int n = 0; n < N; ++n) a[n] = fq[u][n];
        rload(m - QR >= m0 ? m - QR : m0, fq[u], sq[u]);
      }
    }
  }
#pragma unroll
  for (int n = 0; n < N; ++n) ag[n] = a[n];
  __syncthreads();
  FRS_STAMP(4);
  // ---- T entering the segment from its right end
#pragma unroll
  for (int n = 0; n < N; ++n) z[n] = slotR[col][n];
  for (int sp = sg.Gu - 1; sp > seg; --sp) {
    double o[N];
    const double *as = agg + ((size_t)sp * CW + col) * N;
#pragma unroll
    for (int n = 0; n < N; ++n) o[n] = as[n];
    mv(sp == sg.Gu - 1 ? cPT : cPS, z, o, true);
#pragma unroll
    for (int n = 0; n < N; ++n) z[n] = o[n];
  }
  // ---- C': true reverse states
  if (live) {
    double fq[QR][N], sq[QR][N];
#pragma unroll
    for (int u = 0; u < QR; ++u) rload(m1 - 1 - u >= m0 ? m1 - 1 - u : m0, fq[u], sq[u]);
    for (int64_t mb = m1 - 1; mb >= m0; mb -= QR) {
#pragma unroll
      for (int u = 0; u < QR; ++u) {
        const int64_t m = mb - u;
        if (m < m0) break;
        mv(cPB, z, fq[u], true);
        mv(cMB, sq[u], fq[u], false);
#pragma unroll
        for (int n = 0; n < N; ++n) {
          z[n] = fq[u][n];
          STm[(m * N + n) * n_ch + ch] = z[n];
        }
        rload(m - QR >= m0 ? m - QR : m0, fq[u], sq[u]);
      }
    }
  }
  FRS_STAMP(5);
}

// ---------------------------------------------------------------------------
// Full-rate sosfiltfilt: one thread per channel; forward outputs staged in a
// float64 workspace laid out [t][ch] (coalesced across channels).
// ---------------------------------------------------------------------------
template <int NS>
__global__ __launch_bounds__(256) void k_sosfiltfilt_full(
    const float *__restrict__ x, int64_t n_ch, int64_t n_t, int64_t s_ch,
    int64_t s_t, const SosCoef cf, const ZiVec zi, int padlen, double *__restrict__ ws, double *__restrict__ y, int64_t ys_ch,
    int64_t ys_t) {
  constexpr int N = 2 * NS;
  const int64_t ch = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= n_ch) return;
  FwdRec<NS> fr;
  fr.load(cf);
  const float *xc = x + ch * s_ch;
  const int E = padlen;
  const int64_t n_ext = n_t + 2 * (int64_t)E;
  const float x0 = xc[0], xn = xc[(n_t - 1) * s_t];
  auto ext = [&](int64_t t) -> double {
    if (t < E) return (double)(2.0f * x0 - xc[(E - t) * s_t]);
    if (t < E + n_t) return (double)xc[(t - E) * s_t];
    return (double)(2.0f * xn - xc[(n_t - 2 - (t - E - n_t)) * s_t]);
  };
  double s[N];
  const double e0 = ext(0);
#pragma unroll
  for (int i = 0; i < N; ++i) s[i] = zi.v[i] * e0;
  double yl = 0.0;
  for (int64_t t = 0; t < n_ext; ++t) {
    yl = fr.step(s, ext(t));
    ws[t * n_ch + ch] = yl;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) s[i] = zi.v[i] * yl;
  for (int64_t t = n_ext - 1; t >= E; --t) {
    const double v = fr.step(s, ws[t * n_ch + ch]);
    if (t < E + n_t) y[ch * ys_ch + (t - E) * ys_t] = v;
  }
}

__global__ __launch_bounds__(256) void k_interp_linear(
    const double *__restrict__ x, int64_t n_ch, int64_t n_t, int64_t s_ch,
    int64_t s_t, const int64_t *__restrict__ lo, const double *__restrict__ w,
    int64_t n_out, double *__restrict__ y, int64_t ys_ch, int64_t ys_t) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ch * n_out) return;
  const int64_t j = i % n_out, ch = i / n_out;
  const int64_t l = lo[j];
  const double a = x[ch * s_ch + l * s_t];
  double v = a;
  if (w[j] != 0.0) v = fma(x[ch * s_ch + (l + 1) * s_t] - a, w[j], a);
  y[ch * ys_ch + j * ys_t] = v;
  (void)n_t;
}

// ---------------------------------------------------------------------------
// Rolling mean
// ---------------------------------------------------------------------------
// One DPP step on a double (both 32-bit halves; lanes without a source, or
// in rows the mask leaves out, read 0.0).  dpp_ctrl: row_shr:n = 0x110 + n,
// row_bcast:15 = 0x142, row_bcast:31 = 0x143 (GFX9 encodings).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int l2 = __builtin_amdgcn_update_dpp(0, lo, CTRL, ROW_MASK, 0xf, false);
  const int h2 = __builtin_amdgcn_update_dpp(0, hi, CTRL, ROW_MASK, 0xf, false);
  return __hiloint2double(h2, l2);
}

// Inclusive wave scan of a double over the 64 lanes on DPP (VALU lane
// moves, no LDS round trips): Kogge-Stone inside each 16-lane row, then the
// row totals broadcast forward (row_bcast:15 into rows 1 and 3, row_bcast:31
// into rows 2 and 3).
__device__ __forceinline__ double wave_incl_scan_dpp(double v) {
  v += dpp_d<0x111, 0xf>(v);
  v += dpp_d<0x112, 0xf>(v);
  v += dpp_d<0x114, 0xf>(v);
  v += dpp_d<0x118, 0xf>(v);
  v += dpp_d<0x142, 0xa>(v);
  v += dpp_d<0x143, 0xc>(v);
  return v;
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l), hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// time-contiguous: one wave per output window, float4 loads on the aligned
// interior of the window, fp64 accumulation, grid-stride over windows.
// lane's share of sum(x[a:b]) (float64), float4 loads on the 16-B aligned
// interior with up to 4 independent 1-KB wave loads in flight per step
__device__ __forceinline__ double window_part(const float *__restrict__ x, int64_t a, int64_t b, int lane,
                                              bool vec) {
  double acc = 0.0;
  const int64_t a4 = (a + 3) & ~(int64_t)3;
  const int64_t b4 = b & ~(int64_t)3;
  if (!vec || a4 >= b4) {
    for (int64_t i = a + lane; i < b; i += 64) acc += (double)x[i];
    return acc;
  }
  if (lane < a4 - a) acc += (double)x[a + lane];
  if (lane < b - b4) acc += (double)x[b4 + lane];
  const float4 *p4 = reinterpret_cast<const float4 *>(x + a4);
  const int64_t n4 = (b4 - a4) >> 2;
  for (int64_t q0 = lane; q0 < n4; q0 += 256) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t q = q0 + 64 * u;
      v[u] = q < n4 ? p4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += ((double)v[u].x + (double)v[u].y) + ((double)v[u].z + (double)v[u].w);
  }
  return acc;
}

// One wave per output window (grid-stride).  Two windows per step: their
// loads are issued together (8 KB per wave in flight at W = 1000).
#ifndef ROLL_H
#define ROLL_H 2  // windows per wave step
#endif
__global__ __launch_bounds__(256) void k_rolling_tc(
    const float *__restrict__ x, int64_t n_ch, int64_t n_t, int64_t s_ch,
    int64_t W, int64_t S, float *__restrict__ y, int64_t ys_ch, int64_t ys_t,
    bool vec) {
  constexpr int H = ROLL_H;
  const int64_t n_out = (n_t + S - 1) / S;
  const int64_t n_win = n_ch * n_out;
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const float nanv = __builtin_nanf("");
  for (int64_t w0 = wave0; w0 < n_win; w0 += H * n_waves) {
    double acc[H];
    float *out[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      acc[h] = 0.0;
      out[h] = nullptr;
    }
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const int64_t wi = w0 + h * n_waves;
      if (wi >= n_win) continue;
      const int64_t ch = wi / n_out, k = wi % n_out;
      const int64_t e = k * S;  // inclusive window end
      out[h] = y + ch * ys_ch + k * ys_t;
      if (e < W - 1) {
        if (lane == 0) *out[h] = nanv;
        out[h] = nullptr;
        continue;
      }
      const int64_t a = ch * s_ch + e - W + 1;  // absolute element index
      acc[h] = window_part(x, a, a + W, lane, vec);
    }
#pragma unroll
    for (int h = 0; h < H; ++h) {
      if (!out[h]) continue;
      const double t = wave_sum(acc[h]);
      if (lane == 0) *out[h] = (float)(t / (double)W);
    }
  }
}

// Running window sum for step < window (every sample read once from HBM; the
// sample leaving the window, x[t - W], is re-read W positions later from L2):
//   Wsum(t) = Wsum(t-1) + m(x[t]) - m(x[t-W]),  m(v) = v if finite else 0,
// float64, with a count of the non-finite samples in the window carried the
// same way.  A window holding a null is summed directly over its raw values
// (NaN / inf exactly as numpy's mean of that window), the rest are
// Wsum / W.  Windows with kS < W - 1 are NaN (pandas right-aligned rolling).
__device__ __forceinline__ float window_direct(const float *__restrict__ row, int64_t e, int64_t W,
                                               int64_t s_t) {
  double acc = 0.0;
  for (int64_t m = e - W + 1; m <= e; ++m) acc += (double)row[m * s_t];
  return (float)(acc / (double)W);
}

// Generic strides (the (time, distance) layout: s_ch = 1): one thread per
// channel and segment of outputs, channels adjacent in a wave so each sample
// row is one coalesced 256-B read; grid-stride over (segment, channel group)
// units, so any n_ch * n_out fits the launch.  S >= W: each output's window
// is summed directly (no sample is read twice); S < W: running sum.
__global__ __launch_bounds__(256) void k_rolling_cols(
    const float *__restrict__ x, int64_t n_ch, int64_t n_t, int64_t s_ch,
    int64_t s_t, int64_t W, int64_t S, float *__restrict__ y, int64_t ys_ch,
    int64_t ys_t, int64_t seg_out) {
  const int64_t n_out = (n_t + S - 1) / S;
  const int64_t n_seg = (n_out + seg_out - 1) / seg_out;
  const int64_t n_units = n_seg * n_ch;
  const float nanv = __builtin_nanf("");
  const int64_t k_first = (W - 1 + S - 1) / S;  // first output with a full window
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n_units;
       u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ch = u % n_ch, seg = u / n_ch;
    const int64_t k0 = seg * seg_out;
    const int64_t k1 = min(n_out, k0 + seg_out);
    const float *row = x + ch * s_ch;
    float *yo = y + ch * ys_ch;
    int64_t k = k0;
    for (; k < k1 && k < k_first; ++k) yo[k * ys_t] = nanv;
    if (k >= k1) continue;
    if (S >= W) {
      for (; k < k1; ++k) {
        const int64_t e = k * S;
        double acc = 0.0;
        int bad = 0;
        for (int64_t m = e - W + 1; m <= e; ++m) {
          const float v = row[m * s_t];
          bad |= !__builtin_isfinite(v);
          acc += (double)v;
        }
        yo[k * ys_t] = bad ? window_direct(row, e, W, s_t) : (float)(acc / (double)W);
      }
      continue;
    }
    // running sum from the window ending at k*S
    int64_t e = k * S;
    double sum = 0.0;
    int64_t cnt = 0;
    for (int64_t m = e - W + 1; m <= e; ++m) {
      const float v = row[m * s_t];
      const bool f = __builtin_isfinite(v);
      sum += f ? (double)v : 0.0;
      cnt += !f;
    }
    yo[k * ys_t] = cnt ? window_direct(row, e, W, s_t) : (float)(sum / (double)W);
    for (++k; k < k1; ++k) {
      const int64_t e1 = k * S;
      for (int64_t t = e + 1; t <= e1; ++t) {
        const float vi = row[t * s_t], vo = row[(t - W) * s_t];
        const bool fi = __builtin_isfinite(vi), fo = __builtin_isfinite(vo);
        sum += (fi ? (double)vi : 0.0) - (fo ? (double)vo : 0.0);
        cnt += (int64_t)!fi - (int64_t)!fo;
      }
      e = e1;
      yo[k * ys_t] = cnt ? window_direct(row, e, W, s_t) : (float)(sum / (double)W);
    }
  }
}

// Time-contiguous rows, step < window: one wave per (channel, segment of
// outputs).  A wave step covers RS_P = 512 consecutive positions, each lane
// RS_E = 8 CONSECUTIVE ones (two float4 loads of x[t] and two of the sample
// leaving the window, x[t - W], an L1/L2 re-read).  Per lane: d = x[t] -
// x[t-W] in float64 and a sequential running sum over its 8 positions; one
// wave exclusive scan of the lane totals per step gives each lane its entry
// window sum.  Outputs are the positions t = kS.  Steps inside the output
// range whose window holds no null take a fast path (no masks, no range
// tests: a null makes the lane total non-finite, which sends the step to
// the general path).  The segment's first window is summed directly (a halo
// of W samples per segment: segments are >= 4W).
#ifndef LFD_RS_E
#define LFD_RS_E 8
#endif
constexpr int RS_E = LFD_RS_E;      // positions per lane per step
constexpr int RS_P = 64 * RS_E;     // positions per wave step
// Null bookkeeping of the running sum: each sample contributes a packed code
// (NaN: 1, +inf: 2^21, -inf: 2^42; finite: 0); a window's summed code holds
// its NaN / +inf / -inf counts (W < 2^21).  numpy's mean over such a window:
// NaN if it holds a NaN or both infinities, else the infinity it holds.
__device__ __forceinline__ int64_t null_code(float v) {
  return __builtin_isfinite(v) ? 0 : (v != v ? 1 : (v > 0.0f ? (int64_t)1 << 21 : (int64_t)1 << 42));
}
__device__ __forceinline__ float null_mean(int64_t code, float mean) {
  const int64_t n_nan = code & ((1 << 21) - 1), n_pinf = (code >> 21) & ((1 << 21) - 1), n_ninf = code >> 42;
  if (n_nan || (n_pinf && n_ninf)) return __builtin_nanf("");
  if (n_pinf) return __builtin_inff();
  if (n_ninf) return -__builtin_inff();
  return mean;
}

// STAGE: 2 = S == 1 outputs leave through a wave-private LDS tile as
// coalesced float4 stores (lane 4l + 256j); 0 = lanes store their 8
// positions directly (unaligned rows).  Loads: lanes read their 8
// consecutive positions directly.
constexpr int RS_ROW = RS_E + 4;    // padded LDS row (floats): conflict-free ds_read_b128
// RING: the samples leaving the window, x[t - W], come from a wave-private
// LDS ring of the last ring_mask + 1 >= W + 512 samples (each step writes
// its 512 new samples there) instead of a second global read: the global
// re-read missed L2 for 40 % of its bytes (PMC, 16.9 GB fetched for 12 GB of
// input at W = 1000, S = 1).
template <bool VEC, int STAGE, int NPF = 1, int MINW = 3, bool RING = false>
__global__ __launch_bounds__(256, MINW) void k_rolling_scan_tc(
    const float *__restrict__ x, int64_t n_ch, int n_t, int64_t s_ch, int W, int S,
    float *__restrict__ y, int64_t ys_ch, int64_t ys_t, int seg_out, bool vec_out, int ring_mask, bool scan_dpp) {
  // positions are row-relative int32 (the launcher checks n_t < 2^31 - 1024)
  __shared__ __attribute__((aligned(16))) float lds_all[(STAGE & 2) ? 4 : 1][(STAGE & 2) ? 64 * RS_ROW : 4];
  extern __shared__ __attribute__((aligned(16))) float rs_ring_all[];
  float *ring = rs_ring_all + (RING ? (threadIdx.x >> 6) * (ring_mask + 1) : 0);
  const int lane = threadIdx.x & 63;
  float *lx = lds_all[(STAGE & 2) ? threadIdx.x >> 6 : 0];
  const int n_out = (n_t + S - 1) / S;
  const int n_seg = (n_out + seg_out - 1) / seg_out;
  const int64_t n_units = (int64_t)n_seg * n_ch;
  const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const float nanv = __builtin_nanf("");
  const int k_first = (W - 1 + S - 1) / S;
  const double inv_w = 1.0 / (double)W;
  for (int64_t u = uniform64(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6); u < n_units;
       u += n_waves) {
    const int useg = (int)(u % n_seg);
    const int64_t ch = u / n_seg;
    const int k0 = useg * seg_out;
    const int k1 = min(n_out, k0 + seg_out);
    const float *row = x + ch * s_ch;
    float *yo = y + ch * ys_ch;
    const int ka = k0 > k_first ? k0 : k_first;
    for (int k = k0 + lane; k < k1 && k < k_first; k += 64) yo[k * ys_t] = nanv;
    if (ka >= k1) continue;
    const int p0 = ka * S, p1 = (k1 - 1) * S;  // output positions [p0, p1]
    // Wsum(p0 - 1): window [p0 - W, p0 - 1] (x[-1] = 0 when p0 = W - 1)
    double carry = 0.0;
    int64_t ccnt = 0;  // packed null counts of the window (null_code)
    auto halo = [&]() {
      double acc = 0.0;
      int64_t cnt = 0;
      for (int m = p0 - W + lane; m < p0; m += 64) {
        const float v = m < 0 ? 0.0f : row[m];
        if (RING) ring[m & ring_mask] = v;  // (x[m < 0] = 0 in the ring)
        acc += __builtin_isfinite(v) ? (double)v : 0.0;
        cnt += null_code(v);
      }
      carry = wave_sum(acc);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
      ccnt = cnt;
    };
    const int tb0 = VEC ? (p0 & ~3) : p0;
    struct Tile {
      float xi[RS_E], xo[RS_E];
    };
    auto load = [&](int tb, Tile &T) {
      const int t = tb + RS_E * lane;
      const bool full = tb + RS_P <= n_t && (RING || tb - W >= 0);
      if (RING) {  // x[t - W] comes from the ring in process()
        if (full) {
#pragma unroll
          for (int h = 0; h < RS_E / 4; ++h) {
            const f4v a = *reinterpret_cast<const f4u *>(row + t + 4 * h);
#pragma unroll
            for (int e = 0; e < 4; ++e) T.xi[4 * h + e] = a[e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < RS_E; ++e) T.xi[e] = t + e < n_t ? row[t + e] : 0.0f;
        }
        return;
      }
      if (VEC && full) {
#pragma unroll
        for (int h = 0; h < RS_E / 4; ++h) {
          const f4v a = *reinterpret_cast<const f4u *>(row + t + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) T.xi[4 * h + e] = a[e];
          if ((W & 3) == 0) {
            const f4v b = *reinterpret_cast<const f4u *>(row + t + 4 * h - W);
#pragma unroll
            for (int e = 0; e < 4; ++e) T.xo[4 * h + e] = b[e];
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) T.xo[4 * h + e] = row[t + 4 * h + e - W];
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < RS_E; ++e) {
          const int ti = t + e;
          T.xi[e] = ti < n_t ? row[ti] : 0.0f;
          T.xo[e] = (ti - W >= 0 && ti < n_t) ? row[ti - W] : 0.0f;
        }
      }
    };
    auto process = [&](int tb, const Tile &Tin) {
      const int t = tb + RS_E * lane;  // this lane's first position
      Tile T = Tin;
      if (RING) {
        // this step's samples into the ring, then x[t - W] out of it (W + 512
        // <= ring size: nothing a later read needs is overwritten)
#pragma unroll
        for (int h = 0; h < RS_E / 4; ++h)
          *reinterpret_cast<f4v *>(ring + ((t + 4 * h) & ring_mask)) =
              f4v{T.xi[4 * h], T.xi[4 * h + 1], T.xi[4 * h + 2], T.xi[4 * h + 3]};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if ((W & 3) == 0) {
#pragma unroll
          for (int h = 0; h < RS_E / 4; ++h) {
            const f4v b = *reinterpret_cast<const f4v *>(ring + ((t + 4 * h - W) & ring_mask));
#pragma unroll
            for (int e = 0; e < 4; ++e) T.xo[4 * h + e] = b[e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < RS_E; ++e) T.xo[e] = ring[(t + e - W) & ring_mask];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      double d[RS_E];
#pragma unroll
      for (int e = 0; e < RS_E; ++e) d[e] = (double)T.xi[e] - (double)T.xo[e];
#pragma unroll
      for (int e = 1; e < RS_E; ++e) d[e] += d[e - 1];
      // general path: steps at the output range's edges, or whose window
      // holds a null (a null makes some lane total non-finite)
      const bool general = !(tb >= p0 && tb + RS_P - 1 <= p1 && ccnt == 0) ||
                           __any(!__builtin_isfinite(d[RS_E - 1]));
      if (general) {
#pragma unroll
        for (int e = 0; e < RS_E; ++e) {
          const int ti = t + e;
          const bool in = ti >= p0 && ti <= p1;
          const float a = T.xi[e], b = T.xo[e];
          d[e] = in ? (__builtin_isfinite(a) ? (double)a : 0.0) - (__builtin_isfinite(b) ? (double)b : 0.0) : 0.0;
        }
#pragma unroll
        for (int e = 1; e < RS_E; ++e) d[e] += d[e - 1];
      }
      double v = d[RS_E - 1];
      if (scan_dpp) {
        v = wave_incl_scan_dpp(v);
      } else {
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const double w_ = __shfl_up(v, o, 64);
          if (lane >= o) v += w_;
        }
      }
      const double excl = carry + (v - d[RS_E - 1]);
      const double tot = readlane_d(v, 63);
      float o8[RS_E];
#pragma unroll
      for (int e = 0; e < RS_E; ++e) o8[e] = (float)((excl + d[e]) * inv_w);
      if (general) {
        // windows holding nulls: the packed counts of NaN / +inf / -inf
        // samples in the window give numpy's mean of the raw values
        int64_t c[RS_E];
        bool any_code = ccnt != 0;
#pragma unroll
        for (int e = 0; e < RS_E; ++e) {
          const int ti = t + e;
          c[e] = ti >= p0 && ti <= p1 ? null_code(T.xi[e]) - null_code(T.xo[e]) : 0;
          any_code |= c[e] != 0;
        }
        if (__any(any_code)) {
#pragma unroll
          for (int e = 1; e < RS_E; ++e) c[e] += c[e - 1];
          int64_t vc = c[RS_E - 1];
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            const int64_t w_ = __shfl_up(vc, o, 64);
            if (lane >= o) vc += w_;
          }
          const int64_t ex = ccnt + (vc - c[RS_E - 1]);
#pragma unroll
          for (int e = 0; e < RS_E; ++e) o8[e] = null_mean(ex + c[e], o8[e]);
          ccnt += __shfl(vc, 63, 64);
        }
      }
      if (S == 1 && vec_out && !general && (STAGE & 2)) {
        // lane-consecutive -> coalesced through LDS: float4 j of lane l =
        // positions 4l + 256j
#pragma unroll
        for (int h = 0; h < RS_E / 4; ++h)
          *reinterpret_cast<f4v *>(lx + lane * RS_ROW + 4 * h) = f4v{o8[4 * h], o8[4 * h + 1], o8[4 * h + 2], o8[4 * h + 3]};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int h = 0; h < RS_E / 4; ++h) {
          const int pos = 4 * lane + 256 * h;
          *reinterpret_cast<f4v *>(yo + tb + pos) = *reinterpret_cast<const f4v *>(lx + (pos / RS_E) * RS_ROW + (pos % RS_E));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      } else if (S == 1 && vec_out && !general) {
#pragma unroll
        for (int h = 0; h < RS_E / 4; ++h)
          *reinterpret_cast<f4v *>(yo + t + 4 * h) = f4v{o8[4 * h], o8[4 * h + 1], o8[4 * h + 2], o8[4 * h + 3]};
      } else {
        // outputs: positions t + e with (t + e) % S == 0
        int ph = t % S;
#pragma unroll
        for (int e = 0; e < RS_E; ++e) {
          const int ti = t + e;
          if (ti >= p0 && ti <= p1 && ph == 0) yo[(int64_t)(ti / S) * ys_t] = o8[e];
          ph = ph + 1 == S ? 0 : ph + 1;
        }
      }
      carry += tot;
    };
    // ring of NPF + 1 tiles: NPF steps of loads in flight behind the step
    // being processed (indices static: the ring is unrolled)
    Tile R[NPF + 1];
    if constexpr (RING) {
      // whole tiles (tb + RS_P <= n_t) through the ring with unconditional
      // buffer loads — wave-uniform row descriptor, tile base in soffset, the
      // prefetch index clamped to the last whole tile — so each step waits
      // only for its own tile (a conditional load made the compiler wait for
      // every load in flight); the partial tiles at the row end afterwards
      const __amdgpu_buffer_rsrc_t rrow =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(row), (short)0, n_t * 4, 0x00020000);
      auto load_i = [&](int tb, Tile &T) {
#pragma unroll
        for (int h = 0; h < RS_E / 4; ++h) {
          const auto a = __builtin_bit_cast(
              f4v, __builtin_amdgcn_raw_buffer_load_b128(rrow, 4u * (uint32_t)(RS_E * lane + 4 * h), 4 * tb, 0));
#pragma unroll
          for (int e = 0; e < 4; ++e) T.xi[4 * h + e] = a[e];
        }
      };
      const int n_tiles = (p1 - tb0) / RS_P + 1;
      const int nI = min(n_tiles, n_t - RS_P - tb0 >= 0 ? (n_t - RS_P - tb0) / RS_P + 1 : 0);
      if (nI > 0) {
#pragma unroll
        for (int d = 0; d < NPF; ++d) load_i(tb0 + min(d, nI - 1) * RS_P, R[d]);
      }
      halo();  // the first window's sum (its loads queue behind the ring's)
      int i = 0;
      while (i < nI) {
#pragma unroll
        for (int u = 0; u <= NPF; ++u) {
          load_i(tb0 + min(i + NPF, nI - 1) * RS_P, R[(u + NPF) % (NPF + 1)]);
          process(tb0 + i * RS_P, R[u]);
          if (++i == nI) break;
        }
      }
      for (; i < n_tiles; ++i) {
        Tile T;
        load(tb0 + i * RS_P, T);
        process(tb0 + i * RS_P, T);
      }
      continue;
    }
    int tb = tb0;
#pragma unroll
    for (int d = 0; d < NPF; ++d)
      if (tb + d * RS_P <= p1) load(tb + d * RS_P, R[d]);
    halo();  // the first window's sum (its loads queue behind the ring's)
    bool fin = false;
    while (!fin) {
#pragma unroll
      for (int u = 0; u <= NPF; ++u) {
        if (tb + NPF * RS_P <= p1) load(tb + NPF * RS_P, R[(u + NPF) % (NPF + 1)]);
        process(tb, R[u]);
        tb += RS_P;
        if (tb > p1) {
          fin = true;
          break;
        }
      }
    }
  }
}


// ---------------------------------------------------------------------------
// k_rolling_seg — rolling mean for 1 < S < W on time-contiguous rows by
// segment prefix sums (g = gcd(W, S) >= 16, M = W / g, Q = S / g).  Segment
// j holds positions ((j - 1) g, j g]; output k is the sum of segments
// kQ - M + 1 .. kQ over W:
//   out[k] = (SP(kQ) - SP(kQ - M)) / W,   SP(j) = sum of x over (jA g, j g]
// with SP relative to the unit's first needed boundary jA = ka Q - M.  A
// wave owns (channel, range of outputs); per tile of 1,024 positions (4
// lane-contiguous 16-B buffer loads per lane, NPF tiles in flight, then a
// wave-private LDS stage to 16 consecutive positions per lane) every lane sums
// its 16 samples in float64 and the sum up to the one segment boundary
// (g >= 16) its positions may hold; one DPP wave scan of the lane sums gives
// SP at every boundary of the tile, written to a wave-private LDS ring of
// segment prefixes.  Outputs read two ring entries each: no per-position
// running sum, no ring of raw samples, the only carried value is the tile
// total.  Nulls: packed counts (null_code) ride along in an int64 ring, so a
// window's NaN / +-inf counts give numpy's mean of it exactly; tiles without
// a non-finite sample skip that bookkeeping.
// ---------------------------------------------------------------------------
constexpr int RG_E = 16;          // positions per lane per tile
constexpr int RG_P = 64 * RG_E;   // positions per tile

__device__ __forceinline__ int64_t wave_incl_scan_i64(int64_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t w = __shfl_up(v, o, 64);
    if (lane >= o) v += w;
  }
  return v;
}

// Loads: lane l, load h reads positions 256 h + 4 l .. + 3 (one 1-KB span
// per wave-instruction, as the W = S kernel reads) and the tile goes through
// a wave-private 4-KB LDS stage to the 16-consecutive-positions-per-lane
// layout; lane l reads its 4 pieces in the rotated order (j + l / 4) & 3,
// which keeps every ds_read_b128 lane group on distinct banks.  (Round 6,
// with the unconditional interior loads below: cfg2 S = 250 0.719 -> 0.733
// of HBM; lanes loading their own 64 B — 64 lines per wave-instruction —
// measured equal or slower.)
template <int NPF>
__global__ __launch_bounds__(256) void k_rolling_seg(const float *__restrict__ x, int64_t n_ch, int n_t, int64_t s_ch,
                                                     int W, int S, int g, float *__restrict__ y, int64_t ys_ch,
                                                     int64_t ys_t, int seg_out, int ring_mask, int ebatch,
                                                     int diag = 0) {
  // (diag, LFD_ROLL_SEG_DIAG, timings only: 1 = loads + lane sums only, 2 = no
  // output pass)
  diag = LFD_DG(diag);
  extern __shared__ double rg_ring_all[];
  const int R = ring_mask + 1;
  double *spr = rg_ring_all + (size_t)(threadIdx.x >> 6) * 2 * R;   // SP(j) at slot j & ring_mask
  int64_t *cdr = reinterpret_cast<int64_t *>(spr + R);              // packed null counts, same slots
  const int lane = threadIdx.x & 63;
  // the wave's 4-KB transpose stage, past the 4 waves' rings
  float *stg = reinterpret_cast<float *>(rg_ring_all + (size_t)8 * R) + (size_t)(threadIdx.x >> 6) * RG_P;
  const int M = W / g, Q = S / g;
  const int n_out = (n_t + S - 1) / S;
  const int n_seg = (n_out + seg_out - 1) / seg_out;
  const int64_t n_units = (int64_t)n_seg * n_ch;
  const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int k_first = (M + Q - 1) / Q;  // first output with a full window (kS >= W - 1 <=> kQ >= M)
  const float nanv = __builtin_nanf("");
  const double inv_w = 1.0 / (double)W;
  for (int64_t u = uniform64(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6); u < n_units; u += n_waves) {
    const int useg = (int)(u % n_seg);
    const int64_t ch = u / n_seg;
    const int k0 = useg * seg_out;
    const int k1 = min(n_out, k0 + seg_out);
    const float *row = x + ch * s_ch;
    float *yo = y + ch * ys_ch;
    for (int k = k0 + lane; k < k1 && k < k_first; k += 64) yo[k * ys_t] = nanv;
    const int ka = max(k0, k_first);
    if (ka >= k1) continue;
    const int jA = ka * Q - M;               // SP(jA) = 0
    const int pos0 = jA * g + 1;             // first accumulated position
    const int pend = (k1 - 1) * S;           // last one (< n_t)
    if (lane == 0) {
      spr[jA & ring_mask] = 0.0;
      cdr[jA & ring_mask] = 0;
    }
    double carry = 0.0;
    int64_t ccarry = 0;
    int kn = ka;  // next output to emit
    struct Tile {
      float v[RG_E];
    };
    // position of element i of a loaded tile (lane-contiguous 16-B pieces)
    auto lpos = [&](int tb, int i) { return tb + 256 * (i >> 2) + 4 * lane + (i & 3); };
    // interior tile (every position in [pos0, pend]): unconditional 16-B
    // buffer loads at the wave-uniform row descriptor, the tile base in
    // soffset and a fixed per-lane voffset — no per-tile address VGPRs, so
    // the ring's waits count only the loads before them (with 64-bit
    // addresses recomputed per tile the register reuse forced vmcnt(0))
    const __amdgpu_buffer_rsrc_t rrow =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(row), (short)0, n_t * 4, 0x00020000);
    auto load_i = [&](int tb, Tile &T) {
#pragma unroll
      for (int h = 0; h < RG_E / 4; ++h) {
        const uint32_t vo = 4u * (uint32_t)(lpos(0, 4 * h));
        const auto a = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rrow, vo, 4 * tb, 0));
#pragma unroll
        for (int e = 0; e < 4; ++e) T.v[4 * h + e] = a[e];
      }
    };
    // edge tile: positions outside [pos0, pend] read as 0
    auto load_g = [&](int tb, Tile &T) {
#pragma unroll
      for (int i = 0; i < RG_E; ++i) {
        const int q = lpos(tb, i);
        T.v[i] = (q >= pos0 && q <= pend) ? row[q] : 0.0f;
      }
    };
    auto process = [&](int tb, const Tile &Tin) {
      const int p = tb + RG_E * lane;
      // this lane's segment boundary (a multiple of g), if any: offset eb
      const int bq = (p + g - 1) / g;
      const int bpos = bq * g;
      const int eb = bpos - p;
      const bool has = eb < RG_E && bpos > jA * g && bpos <= pend;
      // T.v[i] = position p + off(i) (the rotated pieces)
      Tile T;
#pragma unroll
      for (int h = 0; h < RG_E / 4; ++h)
        *reinterpret_cast<f4v *>(stg + 256 * h + 4 * lane) =
            f4v{Tin.v[4 * h], Tin.v[4 * h + 1], Tin.v[4 * h + 2], Tin.v[4 * h + 3]};
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int rot = lane >> 2;
#pragma unroll
      for (int j = 0; j < RG_E / 4; ++j) {
        const f4v b = *reinterpret_cast<const f4v *>(stg + RG_E * lane + 4 * ((j + rot) & 3));
#pragma unroll
        for (int e = 0; e < 4; ++e) T.v[4 * j + e] = b[e];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      auto off = [&](int i) { return 4 * (((i >> 2) + rot) & 3) + (i & 3); };
      double tot = 0.0, part = 0.0;
      bool bad = false;
#pragma unroll
      for (int e = 0; e < RG_E; ++e) {
        const float v = T.v[e];
        const bool f = __builtin_isfinite(v);
        bad |= !f;
        const double d = f ? (double)v : 0.0;
        tot += d;
        part += off(e) <= eb ? d : 0.0;
      }
      if (diag & 1) {
        if (tot + part == 1234.5 && !bad) yo[0] = 0.f;
        return;
      }
      const double incl = wave_incl_scan_dpp(tot);
      if (has) spr[bq & ring_mask] = carry + (incl - tot) + part;
      carry += readlane_d(incl, 63);
      if (__any(bad)) {
        int64_t ct = 0, cp = 0;
#pragma unroll
        for (int e = 0; e < RG_E; ++e) {
          const int64_t c = null_code(T.v[e]);  // 0 for the masked positions (0.0f)
          ct += c;
          cp += off(e) <= eb ? c : 0;
        }
        const int64_t ci = wave_incl_scan_i64(ct, lane);
        if (has) cdr[bq & ring_mask] = ccarry + (ci - ct) + cp;
        ccarry += __shfl(ci, 63, 64);
      } else if (has) {
        cdr[bq & ring_mask] = ccarry;
      }
      // outputs whose window ends by this tile (kS <= its last position)
      // leave ebatch (<= 64, a power of 2) at a time — one coalesced store
      // per 64 outputs instead of a few lanes' per tile; the ring holds every
      // prefix they need (launcher) — the rest after the unit's last tile
      const int kmax = min(k1 - 1, (tb + RG_P - 1) / S);
      if ((kmax - kn + 1 >= ebatch || kmax == k1 - 1) && !(diag & 2)) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int kend = kmax == k1 - 1 ? kmax + 1 : kn + ((kmax - kn + 1) & ~(ebatch - 1));
        for (int k = kn + lane; k < kend; k += 64) {
          const int j = k * Q;
          const double sum = spr[j & ring_mask] - spr[(j - M) & ring_mask];
          const int64_t code = cdr[j & ring_mask] - cdr[(j - M) & ring_mask];
          const float mean = (float)(sum * inv_w);
          yo[(int64_t)k * ys_t] = code ? null_mean(code, mean) : mean;
        }
        kn = kend;
      }
    };
    // edge tile at the head, interior tiles through a ring of NPF + 1 (NPF
    // tiles' loads in flight behind the one processed; the prefetch index is
    // clamped to the last interior tile, never a branch), edge tiles at the tail
    const int tb0 = pos0 & ~3;
    const int tI0 = tb0 >= pos0 ? tb0 : tb0 + RG_P;
    const int nI = pend + 1 - tI0 >= RG_P ? (pend + 1 - tI0) / RG_P : 0;
    if (tb0 < tI0) {
      Tile T;
      load_g(tb0, T);
      process(tb0, T);
    }
    if (nI > 0) {
      Tile Tr[NPF + 1];
#pragma unroll
      for (int d = 0; d < NPF; ++d) load_i(tI0 + min(d, nI - 1) * RG_P, Tr[d]);
      int i = 0;
      bool fin = false;
      while (!fin) {
#pragma unroll
        for (int uu = 0; uu <= NPF; ++uu) {
          load_i(tI0 + min(i + NPF, nI - 1) * RG_P, Tr[(uu + NPF) % (NPF + 1)]);
          process(tI0 + i * RG_P, Tr[uu]);
          if (++i == nI) {
            fin = true;
            break;
          }
        }
      }
    }
    for (int tb = tI0 + nI * RG_P; tb <= pend; tb += RG_P) {
      Tile T;
      load_g(tb, T);
      process(tb, T);
    }
  }
}


// ---------------------------------------------------------------------------
// k_block_functionals_mfma — the block functionals as a skinny GEMM on the
// fp64 matrix cores (lfd_internal.h TapGeom):
//   F[k][c][ch] = sum_p Kx[c][p] x[ch][base + k*L + row_off + p].
// A wave owns 16 channels x bpw consecutive blocks (bpw <= MF_RUN, fewer for
// narrow arrays so the grid still fills the chip).  One
// v_mfma_f64_16x16x4_f64 multiplies taps (A: 16 functionals x 4 samples; rows
// >= nc are zero) by samples (B: 4 samples x 16 channels): lane l supplies
// A[c = l&15][k = l>>4] from the LDS tap table and B[k = l>>4][ch = l&15] from
// one 16-B load of its channel per 16-sample group, so a wave-instruction
// loads 16 rows x 64 B and every float feeds exactly one MFMA.  D[c][ch]
// lands with the channel on the lane, so F stores are 16 consecutive
// channels.  The next iteration's 4 loads (64 samples) are in flight behind
// the current iteration's 16 MFMAs; the VALU only converts f32 -> f64.
// ---------------------------------------------------------------------------
typedef double d4v __attribute__((ext_vector_type(4)));
constexpr int MF_RUN = 32;  // max blocks per wave

// guarded 4-sample load (edge blocks only): FIR history is 0 before the
// channel start; the zero-tap padding after the block may run past n_t
__device__ __forceinline__ f4v mf_load_guarded(const float *__restrict__ xr, int64_t off,
                                               int64_t n_t) {
  f4v v;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t i = off + e;
    const int64_t ic = i < 0 ? 0 : (i >= n_t ? n_t - 1 : i);
    const float xv = xr[ic];
    v[e] = (i >= 0 && i < n_t) ? xv : 0.0f;
  }
  return v;
}

// finite-mask the elements of one 64-sample iteration that lie outside the
// block's own samples (row offsets [lo, hi) = [J + v, J + v + L)); o0 = this
// lane's first offset (64 it + 4 q).  Only a block's first iteration (FIR
// history) and last iteration (zero-tap padding) hold such elements.
__device__ __forceinline__ void mf_mask_outside(f4v (&cur)[4], int o0, int lo, int hi) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int o = o0 + 16 * j + e;
      if ((o < lo || o >= hi) && !__builtin_isfinite(cur[j][e])) cur[j][e] = 0.0f;
    }
}


// 16 MFMAs of one 64-sample iteration: taps kt (this lane's A column) x cur.
// Lanes of A rows c >= nc read a copy of row nc-1 instead of zeros: MFMA rows
// are independent (D[c][:] depends on A[c][:] only) and rows >= nc of D are
// never read, so no per-MFMA select is needed.
__device__ __forceinline__ void mf_iter(const double *kt, int kstride, bool colv,
                                        const f4v (&cur)[4], d4v &acc0, d4v &acc1) {
  (void)colv;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double2 b01 = *reinterpret_cast<const double2 *>(kt + j * kstride);
    const double2 b23 = *reinterpret_cast<const double2 *>(kt + j * kstride + 2);
    const double a0 = b01.x, a1 = b01.y;
    const double a2 = b23.x, a3 = b23.y;
    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, (double)cur[j].x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, (double)cur[j].y, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, (double)cur[j].z, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a3, (double)cur[j].w, acc1, 0, 0, 0);
  }
}

// lane holds D[c = q + 4r][ch]: 16 consecutive channels per (block, c)
__device__ __forceinline__ void mf_store(const d4v &acc0, const d4v &acc1, double *F, int64_t k,
                                         int nc, int q, int64_t ch, const BlockGeom &g) {
  if (ch >= g.n_ch) return;
  const d4v acc = acc0 + acc1;
  double *Fo = F + f_index(k, 0, ch, g.nb, nc);
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (q + 4 * r < nc) Fo[(q + 4 * r) * F_CSTRIDE] = acc[r];
}

// (Round 6, measured and not kept: whole 128-B lines per wave instruction —
// 8 rows x 128 B, which streams 2-4 % faster loads-only at full width and
// 10 % at an 8-GPU shard (profiles/r06_k1_shape.txt) — either moved into this
// layout by 16 DPP row exchanges per iteration (1-1.5 % slower,
// profiles/r06_k1_lines_ab.txt) or fed as is to 4x4x4_4b products whose blocks
// take the taps of their piece parity (3-7 % slower,
// profiles/r06_k1_lines4x4_ab.txt).)
// (non-temporal loads of the sample stream were measured 40 % slower on cfg3:
// 18.5 vs 13.1 ms — the 64-B row pieces of consecutive iterations no longer
// meet in L2)
__device__ __forceinline__ f4v ldx4(const float *p) { return *reinterpret_cast<const f4u *>(p); }

// MODE 0: production.  Diagnostic modes (timing experiments only, results
// invalid; LFD_MF_MODE): 1 = no MFMA (VALU sum of the loads) = the memory
// ceiling of the x stream + F stores; 3 = no MFMA and no F stores = the
// x-stream ceiling alone.
template <int PF, int MODE>
__global__ __launch_bounds__(1024) void k_block_functionals_mfma(
    const float *__restrict__ x, int64_t s_ch, int64_t n_t, BlockGeom g,
    const double *__restrict__ taps, TapGeom tg, double *__restrict__ F, int64_t n_runs,
    int bpw) {
  extern __shared__ double Ks[];
  const int tab = tg.Lp * tg.nc;  // doubles per shift table (even)
  for (int i = 2 * threadIdx.x; i < tab * tg.nvar; i += 2 * blockDim.x)
    *reinterpret_cast<double2 *>(Ks + i) = *reinterpret_cast<const double2 *>(taps + i);
  __syncthreads();
  // wave-uniform (SGPR) unit arithmetic: the whole block/producer walk is scalar
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t n_cg = (g.n_ch + 15) / 16;
  const int64_t unit = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  if (unit >= n_cg * n_runs) return;
  const int64_t cg = unit % n_cg, run = unit / n_cg;
  const int64_t k0 = run * bpw;
  const int64_t k1 = k0 + bpw < g.nb ? k0 + bpw : g.nb;
  const int col = lane & 15, q = lane >> 4;
  const int64_t ch = cg * 16 + col;
  const float *xr = x + (ch < g.n_ch ? ch : g.n_ch - 1) * s_ch;  // channel row
  const bool colv = col < tg.nc;
  const double *kl = Ks + (q * tg.nc + (colv ? col : tg.nc - 1)) * 4;
  const int nit = tg.Lp / 64;
  const int kstride = 16 * tg.nc;  // doubles per 16-sample group
  const int64_t s0 = g.base - tg.J;  // first extended sample of block 0
  const int L = g.L;
  // shift table of a block whose row starts at sample s (s >= 0 in the interior)
  auto table = [&](int64_t s) { return tg.nvar == 1 ? kl : kl + (int)(s & 3) * tab; };

  // blocks whose row may leave [0, n_t) (channel start / end) take the guarded
  // path; the rest run the pipelined loop with plain 16-B loads
  int64_t ka = s0 < 0 ? (-s0 + L - 1) / L : 0;                        // s_k >= 0
  int64_t kb = n_t - tg.Lp - s0 >= 0 ? (n_t - tg.Lp - s0) / L + 1 : 0;  // s_k + Lp <= n_t
  ka = uniform64(ka < k0 ? k0 : (ka > k1 ? k1 : ka));
  kb = uniform64(kb > k1 ? k1 : (kb < ka ? ka : kb));
  for (int64_t k = k0; k < k1; ++k) {
    if (k == ka) k = kb;  // skip the interior
    if (k >= k1) break;
    const int64_t s = s0 + k * L;
    const int v = (int)(((s % 4) + 4) % 4);
    const double *kt = tg.nvar == 1 ? kl : kl + v * tab;
    const int64_t a = s - v + 4 * q;
    d4v acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    for (int it = 0; it < nit; ++it) {
      f4v cur[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) cur[j] = mf_load_guarded(xr, a + 64 * it + 16 * j, n_t);
      if (it == 0 || it == nit - 1) mf_mask_outside(cur, 64 * it + 4 * q, tg.J + v, tg.J + v + L);
      mf_iter(kt + (4 * it) * kstride, kstride, colv, cur, acc0, acc1);
    }
    mf_store(acc0, acc1, F, k, tg.nc, q, ch, g);
  }
  if (ka >= kb) return;

  // interior: flattened (block, iteration) stream; the loads of the next PF
  // iterations are in flight behind the current iteration's MFMAs
  const float *xl = xr + 4 * q;
  auto addr = [&](int64_t ss, int ii) { return xl + (ss & ~(int64_t)3) + 64 * ii; };
  int64_t k = ka, s = s0 + ka * L;  // consumer position
  int it = 0;
  int64_t kp = ka, sp = s;          // producer position
  int itp = 0;
  // producer: loads are unconditional (the waitcnt pass then counts exactly
  // PF iterations of loads in flight); past the unit's last iteration it
  // re-loads that iteration (cache hits)
  const float *pp = addr(sp, itp);
  auto produce = [&]() {
    if (kp == kb - 1 && itp == nit - 1) return;
    if (++itp == nit) {
      itp = 0;
      ++kp;
      sp += L;
    }
    pp = addr(sp, itp);
  };
  f4v buf[PF + 1][4];
#pragma unroll
  for (int d = 0; d < PF; ++d) {
#pragma unroll
    for (int j = 0; j < 4; ++j) buf[d][j] = ldx4(pp + 16 * j);
    produce();
  }
  const double *kt = table(s);
  d4v acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
  // the ring is unrolled PF+1 times so buffer indices are static: moving
  // prefetched registers would wait for every load in flight
  bool fin = false;
  while (!fin) {
#pragma unroll
    for (int u = 0; u <= PF; ++u) {
      constexpr int NB = PF + 1;
      const int lb = (u + PF) % NB;
#pragma unroll
      for (int j = 0; j < 4; ++j) buf[lb][j] = ldx4(pp + 16 * j);
      produce();
      if (MODE == 1 || MODE == 3) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc0[j] += (double)(buf[u][j].x + buf[u][j].y + buf[u][j].z + buf[u][j].w);
      } else {
        if (it == 0 || it == nit - 1) {
          const int v = (int)(s & 3);
          mf_mask_outside(buf[u], 64 * it + 4 * q, tg.J + v, tg.J + v + L);
        }
        mf_iter(kt + (4 * it) * kstride, kstride, colv, buf[u], acc0, acc1);
      }
      if (++it == nit) {
        if (MODE == 6) {  // diagnostic: same stores into a 64 KB L2-resident window
          BlockGeom gh = g;
          gh.nb = 1;
          mf_store(acc0, acc1, F + ((k & 7) * 16 + (ch >> 4) % 32) * 16 * 9, 0, tg.nc, q, ch & 15, gh);
        } else if (MODE != 3) {
          mf_store(acc0, acc1, F, k, tg.nc, q, ch, g);
        }
        else if (acc0[0] == 1234.5) F[0] = acc0[1];
        acc0 = d4v{0.0, 0.0, 0.0, 0.0};
        acc1 = d4v{0.0, 0.0, 0.0, 0.0};
        it = 0;
        ++k;
        s += L;
        if (k >= kb) {
          fin = true;
          break;
        }
        kt = table(s);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// k_block_runs_mfma — K1 in run mode (lfd_internal.h RunConst): the same fp64
// MFMA block functionals, folded in-register into runs so that only
// y0(k) (8 B per block per channel) and the run aggregates E_f, E_r (64 B per
// run per channel) reach HBM instead of 72 B of functionals per block.
// Lane (q, col) holds component q of channel col: the run's forward prefix
// S0 (one state per lane), the per-block reverse inputs v = e_r0 + M S0 and
// pg = p0 + G0.S0 go to a wave-private LDS buffer [p][pg, v0..v3][16 ch]; at
// the run's last block a backward sweep over it gives y0 and E_r = T0(ks).
// One 1024-thread workgroup per CU (taps + constants + 16 run buffers).
// ---------------------------------------------------------------------------
// The 4 values a column's lanes hold in the 4 16-lane rows (lane 16k + c
// holds component k of column c in the MFMA output layout), gathered into
// every lane of that column: three permlane swaps per 32-bit half (VALU lane
// exchanges, no LDS round trip).  permlane32_swap(x, x) leaves row (k & 1)'s
// value in [0] and row 2 + (k & 1)'s in [1]; permlane16_swap(y, y) then
// leaves y's even row in [0] and its odd row in [1] of every lane.
__device__ __forceinline__ void row_gather4(double v, double (&o)[4]) {
  const uint32_t lo = (uint32_t)__double2loint(v), hi = (uint32_t)__double2hiint(v);
  const auto r_lo = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto r_hi = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const auto a_lo = __builtin_amdgcn_permlane16_swap(r_lo[0], r_lo[0], false, false);
  const auto a_hi = __builtin_amdgcn_permlane16_swap(r_hi[0], r_hi[0], false, false);
  const auto b_lo = __builtin_amdgcn_permlane16_swap(r_lo[1], r_lo[1], false, false);
  const auto b_hi = __builtin_amdgcn_permlane16_swap(r_hi[1], r_hi[1], false, false);
  o[0] = __hiloint2double((int)a_hi[0], (int)a_lo[0]);
  o[1] = __hiloint2double((int)a_hi[1], (int)a_lo[1]);
  o[2] = __hiloint2double((int)b_hi[0], (int)b_lo[0]);
  o[3] = __hiloint2double((int)b_hi[1], (int)b_lo[1]);
}

// Streaming run epilogue (SEPI): the run's reverse pass accumulated FORWARD,
// block by block, in registers — no LDS run buffer, no backward sweep at
// the run end.  With v_p = e_r0(p) + M S0(p) and pg_p = p0(p) + G0 S0(p):
//   E_r  = T0(ks)  = sum_p PhiR^p v_p
//   y0_p = pg_p + sum_{m > p} H0 PhiR^(m-p-1) v_m      (RunConst::B[d] = H0 PhiR^d)
// Lane (q, col) keeps S0[q], E_r[q] and the y0 of the run's blocks q and
// q + 4 (the blocks it stores), adding each later block's contribution as
// that block arrives.
constexpr int RUN_CST_S = 224;  // doubles: PhiF M PhiR G0 H0 (56) + PhiR^p (128) + B (32)
struct RunAccS {
  double S0 = 0.0, Er = 0.0, ya = 0.0, yb = 0.0;
};
__device__ __forceinline__ void run_block_stream(const double *__restrict__ cst, int q, int p, const double (&a)[3],
                                                 RunAccS &st) {
  const double *PhiF = cst, *Mm = cst + 16, *G0 = cst + 48, *PhiRp = cst + 56, *Bc = cst + 184;
  double sv[4];
  row_gather4(st.S0, sv);
  double v = a[1], pg = a[2], sn = a[0];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v = fma(Mm[q * 4 + j], sv[j], v);
    pg = fma(G0[j], sv[j], pg);
    sn = fma(PhiF[q * 4 + j], sv[j], sn);
  }
  st.S0 = sn;
  double vv[4];
  row_gather4(v, vv);
  const double *pr = PhiRp + p * 16 + q * 4;
  const int da = p - q - 1, db = p - q - 5;  // held blocks q, q + 4: offsets m - p' - 1
  const double *ca = Bc + (da > 0 ? da : 0) * 4, *cb = Bc + (db > 0 ? db : 0) * 4;
  double er = st.Er, ya = st.ya, yb = st.yb;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    er = fma(pr[j], vv[j], er);
    ya = fma(ca[j], vv[j], ya);
    yb = fma(cb[j], vv[j], yb);
  }
  st.Er = er;
  st.ya = da >= 0 ? ya : (da == -1 ? pg : st.ya);
  st.yb = db >= 0 ? yb : (db == -1 ? pg : st.yb);
}

constexpr int RUN_WB = RUN_R * 5 * 16;  // doubles per wave run buffer
constexpr int RUN_CST = 64;             // doubles of epilogue constants in LDS

// MODE 0: production.  Diagnostics (timing only, results invalid;
// LFD_RUN_MODE, diagnostic build): 1 = VALU sum instead of the MFMAs, 4 =
// MFMAs but the run epilogue reduced to one store per block.
// MINW: minimum waves per SIMD the register allocation must allow (4: 128
// VGPRs, 16 waves per CU with two 512-thread workgroups' LDS).
// LAT (lattice one-pass plans): tg.nc = 8 + n_off, MFMA rows 8 + d the
// outputs at offset d of the block; every run's first block is an output
// block (the plan cuts runs there), so only its y0 is formed, streamed: with
// v_p = e_r0(p) + M S0(p) and S0 = 0 at the run start,
//   y0_d(first) = p0_d + H0_d T1,  E_r = v_0 + PhiR T1,  T1 = sum_{p>=1} PhiR^(p-1) v_p.
// Lane (q, col) holds offsets q (row 8 + q, acc[2]) and 4 + q (acc[3]).
// (Measured and removed, records in profiles/ and CHANGELOG.md: 4x4x4
// MFMA steps, buffer-descriptor loads, the streaming epilogue on
// channel-major rows, persistent waves, band / workgroup-per-channel-group
// unit orders.)
struct LatAcc {
  double S0 = 0.0, T1 = 0.0, v0 = 0.0, ya = 0.0, yb = 0.0;
};
template <int PF, int MODE = 0, int NT = 512, int MINW = 0, bool LAT = false>
__global__ __launch_bounds__(NT, MINW > 0 ? MINW : 1) void k_block_runs_mfma(
    const float *__restrict__ x, int64_t s_ch, int64_t n_t, BlockGeom g,
    const double *__restrict__ taps, TapGeom tg, RunGeom rg, double *__restrict__ Y0,
    double *__restrict__ AG) {
  extern __shared__ double Ks[];
  const int tab = tg.Lp * tg.nc;
  const int ntab = tab * tg.nvar;
  for (int i = 2 * threadIdx.x; i < ntab; i += 2 * blockDim.x)
    *reinterpret_cast<double2 *>(Ks + i) = *reinterpret_cast<const double2 *>(taps + i);
  double *cst = Ks + ntab;  // PhiF[16] M[16] PhiR[16] G0[4] H0[4] (LAT: + PhiR^p[8][16] + H0L[8][4])
  for (int i = threadIdx.x; i < 56; i += blockDim.x) cst[i] = (&rg.rc->PhiF[0])[i];
  if (LAT) {
    for (int i = threadIdx.x; i < RUN_R * 16; i += blockDim.x) cst[56 + i] = (&rg.rc->PhiRp[0][0])[i];
    for (int i = threadIdx.x; i < RUN_R * 4; i += blockDim.x) cst[184 + i] = (&rg.rc->H0L[0][0])[i];
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int n_off = tg.nc - 2 * RUN_N;  // (LAT)
  const int64_t y0_slice = ((g.n_ch + 15) / 16) * g.nb * 16;
  (void)n_off;
  (void)y0_slice;
  double *wb = Ks + ntab + RUN_CST + wave * RUN_WB;
  (void)wb;
  const int64_t n_cg = (g.n_ch + 15) / 16;
  const int64_t unit = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  if (unit >= n_cg * rg.n_groups) return;
  // channel-group-major unit order (time-major measured 2 % slower on cfg3)
  const int64_t cg = unit % n_cg, grp = unit / n_cg;
  int r = __builtin_amdgcn_readfirstlane(rg.group_r0[grp]);
  const int r_end = __builtin_amdgcn_readfirstlane(rg.group_r0[grp + 1]);
  // the unit's run table (<= 32 runs) is held one run per lane and read with
  // v_readlane at run ends: a vector load there would wait (vmcnt(0)) for
  // every sample load in flight
  const int ru0 = r;
  const int my_len = lane < r_end - ru0 ? rg.run_len[ru0 + lane] : 0;
  const int64_t my_ks = lane < r_end - ru0 ? rg.run_ks[ru0 + lane] : 0;
  auto run_len_of = [&](int rr) { return __builtin_amdgcn_readlane(my_len, rr - ru0); };
  auto run_ks_of = [&](int rr) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)my_ks, rr - ru0);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)my_ks >> 32), rr - ru0);
    return (int64_t)(((uint64_t)hi << 32) | lo);
  };
  const int64_t k0 = run_ks_of(r);
  const int64_t k1 = run_ks_of(r_end - 1) + run_len_of(r_end - 1);
  const int col = lane & 15, q = lane >> 4;
  const int64_t ch = cg * 16 + col;  // stores land in the 16-channel padding past n_ch
  const float *xr = x + (ch < g.n_ch ? ch : g.n_ch - 1) * s_ch;
  const bool colv = col < tg.nc;
  const double *kl = Ks + (q * tg.nc + (colv ? col : tg.nc - 1)) * 4;
  const int nit = tg.Lp / 64;
  const int kstride = 16 * tg.nc;
  const int64_t s0 = g.base - tg.J;
  const int L = g.L;
  auto table = [&](int64_t s) { return tg.nvar == 1 ? kl : kl + (int)(s & 3) * tab; };
  const double *PhiF = cst, *Mm = cst + 16, *PhiR = cst + 32, *G0 = cst + 48, *H0 = cst + 52;

  int64_t rks = k0;
  int rlen = run_len_of(r);
  double S0 = 0.0;  // run prefix state, component q of channel col
  LatAcc la;        // (LAT)
  auto block_done = [&](const d4v &a, int64_t k) {
    // a[0] = e_f[q], a[1] = e_r0[q], a[2] = p0 (q = 0)
    const int p = (int)(k - rks);
    if constexpr (LAT) {
      double sv[4];
      row_gather4(la.S0, sv);
      double v = a[1], sn = a[0];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v = fma(Mm[q * 4 + j], sv[j], v);
        sn = fma(PhiF[q * 4 + j], sv[j], sn);
      }
      la.S0 = sn;
      if (p == 0) {
        la.ya = a[2];
        la.yb = a[3];
        la.v0 = v;
        la.T1 = 0.0;
      } else {
        double vv[4];
        row_gather4(v, vv);
        const double *pr = cst + 56 + (p - 1) * 16 + q * 4;
        double t1 = la.T1;
#pragma unroll
        for (int j = 0; j < 4; ++j) t1 = fma(pr[j], vv[j], t1);
        la.T1 = t1;
      }
      if (p + 1 == rlen) {
        double tv[4];
        row_gather4(la.T1, tv);
        const double *ha = cst + 184 + q * 4, *hb = cst + 184 + (4 + q) * 4;
        double ya = la.ya, yb = la.yb, er = la.v0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ya = fma(ha[j], tv[j], ya);
          yb = fma(hb[j], tv[j], yb);
          er = fma(PhiR[q * 4 + j], tv[j], er);
        }
        double *y0o = Y0 + (cg * g.nb + rks) * 16 + col;
        if (q < n_off) y0o[q * y0_slice] = ya;
        if (q + 4 < n_off) y0o[(q + 4) * y0_slice] = yb;
        double *ag = AG + ((cg * rg.n_runs + r) * 8) * 16 + col;
        ag[q * 16] = la.S0;
        ag[(4 + q) * 16] = er;
        la = LatAcc{};
        ++r;
        if (r < r_end) {
          rks = run_ks_of(r);
          rlen = run_len_of(r);
        }
      }
      return;
    }
    double sv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) sv[j] = __shfl(S0, col + 16 * j, 64);
    double v = a[1], pg = a[2], sn = a[0];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v = fma(Mm[q * 4 + j], sv[j], v);
      pg = fma(G0[j], sv[j], pg);
      sn = fma(PhiF[q * 4 + j], sv[j], sn);
    }
    S0 = sn;
    wb[(p * 5 + 1 + q) * 16 + col] = v;
    if (q == 0) wb[(p * 5) * 16 + col] = pg;
    if (p + 1 == rlen) {
      __builtin_amdgcn_wave_barrier();
      double T[4] = {0.0, 0.0, 0.0, 0.0};
      double *y0o = Y0 + (cg * g.nb + rks) * 16 + col;
      for (int pp = rlen - 1; pp >= 0; --pp) {
        double y0 = wb[(pp * 5) * 16 + col];
#pragma unroll
        for (int j = 0; j < 4; ++j) y0 = fma(H0[j], T[j], y0);
        if ((pp & 3) == q) y0o[pp * 16] = y0;
        double nt[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          double acc = wb[(pp * 5 + 1 + i) * 16 + col];
#pragma unroll
          for (int j = 0; j < 4; ++j) acc = fma(PhiR[i * 4 + j], T[j], acc);
          nt[i] = acc;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) T[i] = nt[i];
      }
      double *ag = AG + ((cg * rg.n_runs + r) * 8) * 16 + col;
      ag[q * 16] = S0;
      ag[(4 + q) * 16] = q == 0 ? T[0] : (q == 1 ? T[1] : (q == 2 ? T[2] : T[3]));
      __builtin_amdgcn_wave_barrier();
      S0 = 0.0;
      ++r;
      if (r < r_end) {
        rks = run_ks_of(r);
        rlen = run_len_of(r);
      }
    }
  };
  // one block through the guarded (edge) path
  auto guarded_block = [&](int64_t k) {
    const int64_t s = s0 + k * L;
    const int v = (int)(((s % 4) + 4) % 4);
    const double *kt = tg.nvar == 1 ? kl : kl + v * tab;
    const int64_t a = s - v + 4 * q;
    d4v acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    for (int it = 0; it < nit; ++it) {
      f4v cur[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) cur[j] = mf_load_guarded(xr, a + 64 * it + 16 * j, n_t);
      if (it == 0 || it == nit - 1) mf_mask_outside(cur, 64 * it + 4 * q, tg.J + v, tg.J + v + L);
      mf_iter(kt + (4 * it) * kstride, kstride, colv, cur, acc0, acc1);
    }
    block_done(acc0 + acc1, k);
  };

  int64_t ka = s0 < 0 ? (-s0 + L - 1) / L : 0;
  int64_t kb = n_t - tg.Lp - s0 >= 0 ? (n_t - tg.Lp - s0) / L + 1 : 0;
  ka = uniform64(ka < k0 ? k0 : (ka > k1 ? k1 : ka));
  kb = uniform64(kb > k1 ? k1 : (kb < ka ? ka : kb));
  for (int64_t k = k0; k < ka; ++k) guarded_block(k);
  if (ka < kb) {
    const float *xl = xr + 4 * q;
    auto addr = [&](int64_t ss, int ii) { return xl + (ss & ~(int64_t)3) + 64 * ii; };
    int64_t k = ka, s = s0 + ka * L;
    int it = 0;
    int64_t kp = ka, sp = s;
    int itp = 0;
    const float *pp = addr(sp, itp);
    auto produce = [&]() {
      if (kp == kb - 1 && itp == nit - 1) return;
      if (++itp == nit) {
        itp = 0;
        ++kp;
        sp += L;
      }
      pp = addr(sp, itp);
    };
    auto load_iter = [&](f4v (&b)[4]) {
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = ldx4(pp + 16 * j);
    };
    f4v buf[PF + 1][4];
#pragma unroll
    for (int d = 0; d < PF; ++d) {
      load_iter(buf[d]);
      produce();
    }
    const double *kt = table(s);
    d4v acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    bool fin = false;
    while (!fin) {
#pragma unroll
      for (int u = 0; u <= PF; ++u) {
        constexpr int NB = PF + 1;
        const int lb = (u + PF) % NB;
        load_iter(buf[lb]);
        produce();
        if (MODE == 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc0[j] += (double)(buf[u][j].x + buf[u][j].y + buf[u][j].z + buf[u][j].w);
        } else {
          // every chunk's first and last full block is a run end, and inside
          // a run the out-of-block samples belong to the run's own blocks:
          // only a run's first and last iteration need the finite mask
          if ((it == 0 && k == rks) || (it == nit - 1 && k + 1 == rks + rlen)) {
            const int v = (int)(s & 3);
            mf_mask_outside(buf[u], 64 * it + 4 * q, tg.J + v, tg.J + v + L);
          }
          mf_iter(kt + (4 * it) * kstride, kstride, colv, buf[u], acc0, acc1);
        }
        if (++it == nit) {
          const d4v a = acc0 + acc1;
          if (MODE == 4) {
            Y0[(cg * g.nb + k) * 16 + col] = a[q & 3];
          } else {
            block_done(a, k);
          }
          acc0 = d4v{0.0, 0.0, 0.0, 0.0};
          acc1 = d4v{0.0, 0.0, 0.0, 0.0};
          it = 0;
          ++k;
          s += L;
          if (k >= kb) {
            fin = true;
            break;
          }
          kt = table(s);
        }
      }
    }
  }
  for (int64_t k = kb; k < k1; ++k) guarded_block(k);
}

// ---------------------------------------------------------------------------
// k_block_runs_mfma_tm — run-mode K1 for (time, channel) storage (the real
// files' layout, low_pass_dascore.ipynb cell 14 data[:, ch]: s_ch = 1, rows
// of s_t floats).  A wave owns 32 channels = one 128-B line of every sample
// row, i.e. two MFMA column tiles.  Lane (q, col) loads row +4q of its
// channels (X2: the channel pair 2 col, 2 col + 1 with one 8-B load, tile 0
// = even channels, tile 1 = odd, so every load instruction reads 4 whole
// 128-B lines; else col and 16 + col with two dword loads), i.e. the B
// operand layout of v_mfma_f64_16x16x4_f64 with the channel-major kernel's
// sample order: the same tap table (row shift 0) and the same run algebra
// apply, once per tile.  (Measured and removed, records in profiles/ and
// CHANGELOG.md: permlane-swapped row loads, one tile per wave, 4x4x4 steps,
// 768-thread groups, prefetch depth 3, 128-thread groups.)
// ---------------------------------------------------------------------------

struct TmIter {
  float p[4][4], q[4][4];  // [16-sample group j][step e]
};

// Interior loads: the row pointer is wave-uniform (SGPR base) and the lane's
// part a 32-bit element offset, so a load needs no per-lane 64-bit address
// arithmetic (global_load ... saddr).
template <bool X2>
__device__ __forceinline__ void tm_load_u(const float *__restrict__ x, int64_t c0, int64_t s_t, int64_t row0,
                                          uint32_t offp, uint32_t offq, TmIter &b) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t ro = uniform64(c0 + (row0 + 16 * j + e) * s_t);  // element offset of the row
      const char *rp = reinterpret_cast<const char *>(x + ro);
      if (X2) {
        const float2 v = *reinterpret_cast<const float2 *>(rp + offp);
        b.p[j][e] = v.x;
        b.q[j][e] = v.y;
      } else {
        b.p[j][e] = *reinterpret_cast<const float *>(rp + offp);
        b.q[j][e] = *reinterpret_cast<const float *>(rp + offq);
      }
    }
}

// the edge blocks' loads: rows outside [0, n_t) read 0
__device__ __forceinline__ void tm_load_guarded(const float *__restrict__ xc, const float *__restrict__ xq,
                                                int64_t s_t, int64_t n_t, int64_t row0, TmIter &b) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t rp = row0 + 16 * j + e;
      const int64_t cp = rp < 0 ? 0 : (rp >= n_t ? n_t - 1 : rp);
      const float vp = xc[cp * s_t], vq = xq[cp * s_t];
      b.p[j][e] = (rp >= 0 && rp < n_t) ? vp : 0.0f;
      b.q[j][e] = (rp >= 0 && rp < n_t) ? vq : 0.0f;
    }
}

// 2 x 16 MFMAs of one 64-sample iteration (offset o0 = 64 it); out-of-block
// samples (row offsets outside [lo, hi)) finite-masked when `mask`
__device__ __forceinline__ void tm_iter(const double *kt, int kstride, const TmIter &b, int o0, int q, bool mask,
                                        int lo, int hi, d4v &acc0, d4v &acc1) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double2 b01 = *reinterpret_cast<const double2 *>(kt + j * kstride);
    const double2 b23 = *reinterpret_cast<const double2 *>(kt + j * kstride + 2);
    const double a[4] = {b01.x, b01.y, b23.x, b23.y};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v0 = b.p[j][e], v1 = b.q[j][e];
      if (mask) {
        const int o = o0 + 16 * j + 4 * q + e;
        if (o < lo || o >= hi) {
          v0 = finite_or_zero(v0);
          v1 = finite_or_zero(v1);
        }
      }
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[e], (double)v0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[e], (double)v1, acc1, 0, 0, 0);
    }
  }
}

// BUF (with X2): interior loads as buffer loads — one descriptor per
// iteration at the wave-uniform row base, the 16 row offsets (16j + e) s_t
// in SGPRs (soffset), the lane's part in voffset — instead of 16 64-bit
// wave-uniform row pointers per iteration
__device__ __forceinline__ void tm_load_buf(__amdgpu_buffer_rsrc_t rs, uint32_t offp, const int (&soff)[16],
                                            TmIter &b) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, offp, soff[4 * j + e], 0);
      const float2 f = __builtin_bit_cast(float2, v);
      b.p[j][e] = f.x;
      b.q[j][e] = f.y;
    }
}

// SEPI: streaming run epilogue (run_block_stream): the LDS holds only the
// taps and RUN_CST_S constants; no backward sweep at run ends, during which
// a wave issued no loads.  MINW: waves per SIMD the registers are capped for
// (production: 256-thread groups, 2 per SIMD: 8 waves per CU, the occupancy
// at which this access shape streams fastest, profiles/archive_r01_r03.md (r03_ubench_tm.txt)).
// MODE 0: production.  Diagnostics (timing only, results invalid;
// LFD_TM_MODE): 3 = loads only (a VALU sum of the samples, no MFMA, no run
// epilogue, no stores) = the floor of this access shape; 4 = loads + MFMAs,
// the run epilogue reduced to nothing.
template <int TM_PF, int NT, bool X2, bool BUF, bool SEPI, int MINW, int MODE = 0>
__global__ __launch_bounds__(NT, MINW) void k_block_runs_mfma_tm(
    const float *__restrict__ x, int64_t s_t, int64_t n_t, BlockGeom g, const double *__restrict__ taps,
    TapGeom tg, RunGeom rg, double *__restrict__ Y0, double *__restrict__ AG) {
  static_assert(!BUF || X2, "buffer loads read channel pairs");
  extern __shared__ double Ks[];
  const int tab = tg.Lp * tg.nc;  // one table: row shift 0
  for (int i = 2 * threadIdx.x; i < tab; i += 2 * blockDim.x)
    *reinterpret_cast<double2 *>(Ks + i) = *reinterpret_cast<const double2 *>(taps + i);
  double *cst = Ks + tab;  // PhiF[16] M[16] PhiR[16] G0[4] H0[4] (SEPI: + PhiR^p[8][16] + B[8][4])
  for (int i = threadIdx.x; i < 56; i += blockDim.x) cst[i] = (&rg.rc->PhiF[0])[i];
  if (SEPI) {
    for (int i = threadIdx.x; i < RUN_R * 16; i += blockDim.x) cst[56 + i] = (&rg.rc->PhiRp[0][0])[i];
    for (int i = threadIdx.x; i < RUN_R * 4; i += blockDim.x) cst[184 + i] = (&rg.rc->B[0][0])[i];
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  double *wbase = Ks + tab + RUN_CST + wave * 2 * RUN_WB;  // tile t's buffer: wbase + t * RUN_WB
  (void)wbase;
  const int64_t n_c32 = (g.n_ch + 31) / 32;
  const int64_t unit = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  if (unit >= n_c32 * rg.n_groups) return;
  const int64_t c32 = unit % n_c32, grp = unit / n_c32;
  int r = __builtin_amdgcn_readfirstlane(rg.group_r0[grp]);
  const int r_end = __builtin_amdgcn_readfirstlane(rg.group_r0[grp + 1]);
  const int ru0 = r;
  const int my_len = lane < r_end - ru0 ? rg.run_len[ru0 + lane] : 0;
  const int64_t my_ks = lane < r_end - ru0 ? rg.run_ks[ru0 + lane] : 0;
  auto run_len_of = [&](int rr) { return __builtin_amdgcn_readlane(my_len, rr - ru0); };
  auto run_ks_of = [&](int rr) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)my_ks, rr - ru0);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)my_ks >> 32), rr - ru0);
    return (int64_t)(((uint64_t)hi << 32) | lo);
  };
  const int64_t k0 = run_ks_of(r);
  const int64_t k1 = run_ks_of(r_end - 1) + run_len_of(r_end - 1);
  const int col = lane & 15, q = lane >> 4;
  const bool tile1 = c32 * 32 + 16 < g.n_ch;  // tile 1 holds a real channel (else its stores would
                                              // leave the 16-channel padding of Y0 / AG)
  // this lane's load channel and row offset (X2: channel pairs 2 col,
  // 2 col + 1; n_ch is even, a pair past n_ch reads the last pair; else
  // channels past n_ch, in a ragged last group, read channel n_ch - 1)
  const int lc = X2 ? 2 * col : col;
  const int64_t lch = X2 ? min(c32 * 32 + lc, g.n_ch - 2) : min(c32 * 32 + lc, g.n_ch - 1);
  const float *xc = x + lch;
  const int rsel = 4 * q;
  // Q loads: tile 1's channel (16 + col), clamped like P so no load leaves the array
  const int64_t lchq = X2 ? lch + 1 : min(c32 * 32 + 16 + col, g.n_ch - 1);
  const float *xq = x + lchq;
  const int64_t c0 = uniform64(c32 * 32);  // interior loads: uniform row base + lane offset
  const uint32_t offp = (uint32_t)(4 * (lch - c32 * 32 + rsel * s_t)),  // bytes
      offq = (uint32_t)(4 * (lchq - c32 * 32 + rsel * s_t));

  const bool colv = col < tg.nc;
  const double *kl = Ks + (q * tg.nc + (colv ? col : tg.nc - 1)) * 4;
  const int nit = tg.Lp / 64;
  const int kstride = 16 * tg.nc;
  const int64_t s0 = g.base - tg.J;
  const int L = g.L;
  const int lo = tg.J, hi = tg.J + L;  // the block's own samples in its row
  const double *PhiF = cst, *Mm = cst + 16, *PhiR = cst + 32, *G0 = cst + 48, *H0 = cst + 52;

  int64_t rks = k0;
  int rlen = run_len_of(r);
  double S0[2] = {0.0, 0.0};  // run prefix state, component q of channel col, per tile
  auto block_done = [&](const d4v &a, int t, int64_t k) {
    // a[0] = e_f[q], a[1] = e_r0[q], a[2] = p0 (q = 0)
    const int p = (int)(k - rks);
    double sv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) sv[j] = __shfl(S0[t], col + 16 * j, 64);
    double v = a[1], pg = a[2], sn = a[0];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v = fma(Mm[q * 4 + j], sv[j], v);
      pg = fma(G0[j], sv[j], pg);
      sn = fma(PhiF[q * 4 + j], sv[j], sn);
    }
    S0[t] = sn;
    double *wb = wbase + t * RUN_WB;
    wb[(p * 5 + 1 + q) * 16 + col] = v;
    if (q == 0) wb[(p * 5) * 16 + col] = pg;
  };
  auto run_done = [&]() {
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (!X2 && t == 1 && !tile1) break;
      const double *wb = wbase + t * RUN_WB;
      // tile t, lane col: channel 16 (2 c32 + t) + col, or (X2) 32 c32 + 2 col + t
      const int64_t chn = X2 ? c32 * 32 + 2 * col + t : (2 * c32 + t) * 16 + col;
      const int64_t cg = chn >> 4;
      const int cc = (int)(chn & 15);
      const bool st_ok = !X2 || cg * 16 < g.n_ch;  // (X2) inside the 16-channel padding
      double T[4] = {0.0, 0.0, 0.0, 0.0};
      double *y0o = Y0 + (cg * g.nb + rks) * 16 + cc;
      for (int pp = rlen - 1; pp >= 0; --pp) {
        double y0 = wb[(pp * 5) * 16 + col];
#pragma unroll
        for (int j = 0; j < 4; ++j) y0 = fma(H0[j], T[j], y0);
        if ((pp & 3) == q && st_ok) y0o[pp * 16] = y0;
        double nt[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          double acc = wb[(pp * 5 + 1 + i) * 16 + col];
#pragma unroll
          for (int j = 0; j < 4; ++j) acc = fma(PhiR[i * 4 + j], T[j], acc);
          nt[i] = acc;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) T[i] = nt[i];
      }
      if (st_ok) {
        double *ag = AG + ((cg * rg.n_runs + r) * 8) * 16 + cc;
        ag[q * 16] = S0[t];
        ag[(4 + q) * 16] = q == 0 ? T[0] : (q == 1 ? T[1] : (q == 2 ? T[2] : T[3]));
      }
    }
    __builtin_amdgcn_wave_barrier();
    S0[0] = S0[1] = 0.0;
    ++r;
    if (r < r_end) {
      rks = run_ks_of(r);
      rlen = run_len_of(r);
    }
  };
  RunAccS ra[2];
  // SEPI run end: tile t's y0 of blocks q and q + 4, and the aggregates
  auto run_end_stream = [&]() {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (!X2 && t == 1 && !tile1) break;
      const int64_t chn = X2 ? c32 * 32 + 2 * col + t : (2 * c32 + t) * 16 + col;
      const int64_t cg = chn >> 4;
      const int cc = (int)(chn & 15);
      if (X2 && cg * 16 >= g.n_ch) continue;
      double *y0o = Y0 + (cg * g.nb + rks) * 16 + cc;
      if (q < rlen) y0o[q * 16] = ra[t].ya;
      if (q + 4 < rlen) y0o[(q + 4) * 16] = ra[t].yb;
      double *ag = AG + ((cg * rg.n_runs + r) * 8) * 16 + cc;
      ag[q * 16] = ra[t].S0;
      ag[(4 + q) * 16] = ra[t].Er;
      ra[t] = RunAccS{};
    }
    ++r;
    if (r < r_end) {
      rks = run_ks_of(r);
      rlen = run_len_of(r);
    }
  };
  auto finish_block = [&](const d4v &acc0, const d4v &acc1, int64_t k) {
    if constexpr (SEPI) {
      const int p = (int)(k - rks);
      const double a0[3] = {acc0[0], acc0[1], acc0[2]};
      const double a1[3] = {acc1[0], acc1[1], acc1[2]};
      run_block_stream(cst, q, p, a0, ra[0]);
      run_block_stream(cst, q, p, a1, ra[1]);
      if (p + 1 == rlen) run_end_stream();
      return;
    }
    block_done(acc0, 0, k);
    block_done(acc1, 1, k);
    if (k - rks + 1 == rlen) run_done();
  };
  auto guarded_block = [&](int64_t k) {
    const int64_t s = s0 + k * L;
    d4v acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    for (int it = 0; it < nit; ++it) {
      TmIter b;
      tm_load_guarded(xc, xq, s_t, n_t, s + 64 * it + rsel, b);
      tm_iter(kl + (4 * it) * kstride, kstride, b, 64 * it, q, it == 0 || it == nit - 1, lo, hi, acc0, acc1);
    }
    if (MODE == 0) finish_block(acc0, acc1, k);  // (diagnostics: no LDS run buffers)
  };

  int64_t ka = s0 < 0 ? (-s0 + L - 1) / L : 0;
  int64_t kb = n_t - tg.Lp - s0 >= 0 ? (n_t - tg.Lp - s0) / L + 1 : 0;
  ka = uniform64(ka < k0 ? k0 : (ka > k1 ? k1 : ka));
  kb = uniform64(kb > k1 ? k1 : (kb < ka ? ka : kb));
  for (int64_t k = k0; k < ka; ++k) guarded_block(k);
  if (ka < kb) {
    // interior: flattened (block, iteration) stream, TM_PF iterations of
    // loads in flight (ring unrolled so buffer indices are static)
    int64_t k = ka, s = s0 + ka * L;
    int it = 0;
    int64_t kp = ka, sp = s;
    int itp = 0;
    auto produce = [&]() {
      if (kp == kb - 1 && itp == nit - 1) return;  // past the end: re-load the last one
      if (++itp == nit) {
        itp = 0;
        ++kp;
        sp += L;
      }
    };
    TmIter buf[TM_PF + 1];
    int soff[16];
    const int nrec = (int)(64 * s_t * 4 + 256);
#pragma unroll
    for (int k = 0; k < 16; ++k) soff[k] = (int)((16 * (k >> 2) + (k & 3)) * s_t * 4);
    auto load_it = [&](TmIter &b) {
      if constexpr (BUF) {
        const float *rowp = x + uniform64(c0 + (sp + 64 * itp) * s_t);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(rowp), (short)0, nrec, 0x00020000);
        tm_load_buf(rs, offp, soff, b);
      } else {
        tm_load_u<X2>(x, c0, s_t, uniform64(sp + 64 * itp), offp, offq, b);
      }
    };
#pragma unroll
    for (int d = 0; d < TM_PF; ++d) {
      load_it(buf[d]);
      produce();
    }
    d4v acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    bool fin = false;
    while (!fin) {
#pragma unroll
      for (int u = 0; u <= TM_PF; ++u) {
        constexpr int NB = TM_PF + 1;
        const int lb = (u + TM_PF) % NB;
        load_it(buf[lb]);
        produce();
        // a run's first and last iteration need the finite mask (chunk
        // boundaries are run boundaries)
        const bool mask = (it == 0 && k == rks) || (it == nit - 1 && k + 1 == rks + rlen);
        if (MODE == 3) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc0[e] += (double)(buf[u].p[j][e] + buf[u].q[j][e]);
        } else {
          tm_iter(kl + (4 * it) * kstride, kstride, buf[u], 64 * it, q, mask, lo, hi, acc0, acc1);
        }
        if (++it == nit) {
          if (MODE == 0) {
            finish_block(acc0, acc1, k);
            acc0 = d4v{0.0, 0.0, 0.0, 0.0};
            acc1 = d4v{0.0, 0.0, 0.0, 0.0};
          } else if (acc0[0] + acc1[1] == 1234.5) {  // keep the loads and MFMAs alive
            Y0[lane] = acc0[1];
          }
          it = 0;
          ++k;
          s += L;
          if (k >= kb) {
            fin = true;
            break;
          }
        }
      }
    }
  }
  for (int64_t k = kb; k < k1; ++k) guarded_block(k);
}

inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

template <int NS, bool FIR32>
hipError_t block_functionals_ns(const float *x, int64_t s_ch, int64_t s_t, const BlockGeom &g,
                                const BlockConst &kc, double *F, hipStream_t st) {
  const bool lds = (s_t == 1) && (g.L % 4 == 0) && (g.base % 4 == 0) && (s_ch % 4 == 0) &&
                   ((reinterpret_cast<uintptr_t>(x) & 15) == 0) && !knob_flag("LFD_K1_NOLDS");
  if (lds) {
    const int64_t tiles = ((g.n_ch + 15) / 16) * ((g.nb + 15) / 16);
    k_block_functionals_lds<NS, FIR32><<<dim3((unsigned)tiles), 256, 0, st>>>(
        x, s_ch, g, kc, F, knob_flag("LFD_K1_CHAN_FAST") ? 1 : 0);
  } else {
    const int64_t tiles = ((g.n_ch + 63) / 64) * ((g.nb + 3) / 4);
    k_block_functionals_gen<NS, FIR32><<<dim3((unsigned)tiles), 256, 0, st>>>(x, s_ch, s_t, g,
                                                                             kc, F);
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_block_runs_mfma_tm(const float *x, int64_t s_t, int64_t n_t, const BlockGeom &g,
                                     const double *taps, const TapGeom &tg, const RunGeom &rg, double *Y0,
                                     double *AG, hipStream_t st) {
  if (tg.nc != 2 * RUN_N + 1 || tg.Lp % 64 != 0 || tg.nvar != 1 || tg.v0 != 0 || rg.n_groups < 1)
    return hipErrorInvalidValue;
  const size_t tab = sizeof(double) * ((size_t)tg.Lp * tg.nc + RUN_CST);
  auto go = [&](auto kern, size_t lds, int nt) -> hipError_t {
    if (lds > (size_t)TAP_LDS_MAX) return hipErrorInvalidValue;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, TAP_LDS_MAX);
    if (e != hipSuccess) return e;
    const int64_t units = ((g.n_ch + 31) / 32) * rg.n_groups;  // two 16-channel tiles per wave
    const int w = nt / 64;
    kern<<<(unsigned)((units + w - 1) / w), nt, lds, st>>>(x, s_t, n_t, g, taps, tg, rg, Y0, AG);
    return hipGetLastError();
  };
  // channel-pair loads need 8-B aligned pairs (even n_ch and row stride)
  const bool x2 = g.n_ch % 2 == 0 && s_t % 2 == 0 && (reinterpret_cast<uintptr_t>(x) & 7) == 0 &&
                  !option(LFD_OPT_TM_NO_PAIRS);
  if (x2 && s_t < (int64_t)1 << 22) {
    // buffer loads at prefetch depth 1 (14.01 vs 14.18 ms) with the streaming
    // run epilogue, taps + constants only in LDS (13.85 vs 14.35 ms) on cfg3
    // stored time-major (profiles/archive_r01_r03.md (r03_ab_tm_sepi.txt)); 256-thread groups (4
    // per CU, registers for 2 waves per SIMD as before): 13.06 vs 13.50 ms
    // median against 512-thread groups, bit-identical; 128-thread groups 15.03
    // (profiles/r04q_ab_tm_w.txt)
    const size_t lds_s = sizeof(double) * ((size_t)tg.Lp * tg.nc + RUN_CST_S);
#ifdef LFD_DIAG
    // timing-only modes (results invalid): LFD_TM_MODE=3 loads only, =4 no run epilogue
    if (const char *v = knob("LFD_TM_MODE")) {
      if (std::atoi(v) == 3) return go(&k_block_runs_mfma_tm<1, 256, true, true, true, 2, 3>, lds_s, 256);
      if (std::atoi(v) == 4) return go(&k_block_runs_mfma_tm<1, 256, true, true, true, 2, 4>, lds_s, 256);
    }
#endif
    return go(&k_block_runs_mfma_tm<1, 256, true, true, true, 2>, lds_s, 256);
  }
  const size_t lds = tab + sizeof(double) * 8 * 2 * RUN_WB;  // + 8 waves x 2 tiles of run buffers
  if (x2) return go(&k_block_runs_mfma_tm<2, 512, true, false, false, 1>, lds, 512);
  return go(&k_block_runs_mfma_tm<2, 512, false, false, false, 1>, lds, 512);
}

hipError_t launch_block_functionals(int n_sec, bool fir32, const float *x, int64_t s_ch,
                                    int64_t s_t, const BlockGeom &g, const BlockConst &kc,
                                    double *F, hipStream_t st) {
#define LFD_BF(NS)                                                        \
  return fir32 ? block_functionals_ns<NS, true>(x, s_ch, s_t, g, kc, F, st) \
               : block_functionals_ns<NS, false>(x, s_ch, s_t, g, kc, F, st)
  switch (n_sec) {
    case 1: LFD_BF(1);
    case 2: LFD_BF(2);
    case 3: LFD_BF(3);
    case 4: LFD_BF(4);
  }
#undef LFD_BF
  return hipErrorInvalidValue;
}

hipError_t launch_block_functionals_mfma(const float *x, int64_t s_ch, int64_t n_t,
                                         const BlockGeom &g, const double *taps,
                                         const TapGeom &tg, double *F, hipStream_t st) {
  if (tg.nc < 1 || tg.nc > 16 || tg.Lp % 64 != 0 || g.nb < 1 || !(tg.nvar == 1 || tg.nvar == 4) ||
      (tg.nvar == 1 && g.L % 4 != 0))
    return hipErrorInvalidValue;
  const size_t lds = sizeof(double) * (size_t)tg.Lp * tg.nc * tg.nvar;
  if (lds > (size_t)TAP_LDS_MAX) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    for (const void *fn : {reinterpret_cast<const void *>(&k_block_functionals_mfma<2, 0>),
#ifdef LFD_DIAG
                           reinterpret_cast<const void *>(&k_block_functionals_mfma<2, 1>),
                           reinterpret_cast<const void *>(&k_block_functionals_mfma<2, 3>),
                           reinterpret_cast<const void *>(&k_block_functionals_mfma<2, 6>),
#endif
                           }) {
      hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         TAP_LDS_MAX);
      if (e != hipSuccess) return e;
    }
    attr = true;
  }
  // 16 waves per CU whatever the table size: 4 x 256, 2 x 512 or 1 x 1024 threads
  // share one LDS tap table each
  int threads = lds <= 40 * 1024 ? 256 : (lds <= 80 * 1024 ? 512 : 1024);
  if (const char *v = knob("LFD_MF_THREADS")) threads = std::max(threads, std::atoi(v));
  threads = std::min(threads, 1024);
  int pf = 2, mode = 0;
  if (const char *v = knob("LFD_MF_PF")) pf = std::atoi(v);
  if (const char *v = knob("LFD_MF_MODE")) mode = std::atoi(v);  // diagnostics (results invalid)
  // blocks per wave: narrow arrays (the real-time edge runs: 2,000
  // channels, 44 blocks of 2,000 samples) get fewer so that >= ~4,096 waves
  // (16 per CU) cover the chip; within that, the largest count whose units
  // fill their last round of wave slots to >= 95 % (every wave streams at
  // about the same rate, so a last round of 13 % of the slots costs nearly a
  // full round: the full-rate functionals of 2,000 x 600,000 ran 4,625 units
  // of 32 blocks = 1.13 rounds; 12 blocks make 2.99 rounds)
  const int64_t n_cg = (g.n_ch + 15) / 16;
  const int slots = 16 * cu_count();
  const int bmax = (int)std::max<int64_t>(1, std::min<int64_t>(MF_RUN, n_cg * g.nb / slots));
  int bpw = bmax;
  {
    double best = -1.0;
    for (int b = bmax; b >= 1; --b) {
      const double rounds = (double)(n_cg * ((g.nb + b - 1) / b)) / slots;
      const double eff = rounds / std::ceil(rounds);
      if (eff >= 0.95) {
        bpw = b;
        break;
      }
      if (eff > best + 1e-9) {
        best = eff;
        bpw = b;
      }
    }
  }
  if (const char *v = knob("LFD_MF_BPW")) bpw = std::max(1, std::min(MF_RUN, std::atoi(v)));
  const int64_t n_runs = (g.nb + bpw - 1) / bpw;
  const int64_t units = n_cg * n_runs;
  const unsigned grid = nblk(units, threads / 64);
#define LFD_MF(PF_, MODE_)                                                                      \
  k_block_functionals_mfma<PF_, MODE_><<<grid, threads, lds, st>>>(x, s_ch, n_t, g, taps, tg, F, \
                                                                   n_runs, bpw)
#ifdef LFD_DIAG
  // timing-only modes (results invalid, LFD_MF_MODE): 1 loads only, 3 no
  // stores, 6 stores into an L2-resident window
  (void)pf;
  if (mode == 1)
    LFD_MF(2, 1);
  else if (mode == 3)
    LFD_MF(2, 3);
  else if (mode == 6)
    LFD_MF(2, 6);
  else
    LFD_MF(2, 0);
#else
  (void)pf;
  (void)mode;
  LFD_MF(2, 0);
#endif
#undef LFD_MF
  return hipGetLastError();
}

template <int PF, int MODE, int NT, int MINW = 0, bool LAT = false>
hipError_t run_k1(const float *x, int64_t s_ch, int64_t n_t, const BlockGeom &g, const double *taps,
                  const TapGeom &tg, const RunGeom &rg, double *Y0, double *AG, int64_t units, hipStream_t st) {
  constexpr int W = NT / 64;  // waves per workgroup, each with its own run buffer
  // (MODE 4 diagnostic and LAT: no run buffers)
  const size_t lds = LAT ? sizeof(double) * ((size_t)tg.Lp * tg.nc * tg.nvar + RUN_CST_S)
                         : sizeof(double) * ((size_t)tg.Lp * tg.nc * tg.nvar + RUN_CST + (MODE == 4 ? 0 : W) * RUN_WB);
  if (lds > (size_t)TAP_LDS_MAX) return hipErrorInvalidValue;
  auto kern = &k_block_runs_mfma<PF, MODE, NT, MINW, LAT>;
  static std::once_flag attr_once;
  hipError_t ea = hipSuccess;
  std::call_once(attr_once, [&] {
    ea = hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                             TAP_LDS_MAX);
  });
  if (ea != hipSuccess) return ea;
  kern<<<nblk(units, W), NT, lds, st>>>(x, s_ch, n_t, g, taps, tg, rg, Y0, AG);
  return hipGetLastError();
}

hipError_t launch_block_runs_mfma(const float *x, int64_t s_ch, int64_t n_t, const BlockGeom &g,
                                  const double *taps, const TapGeom &tg, const RunGeom &rg,
                                  double *Y0, double *AG, hipStream_t st) {
  if (tg.nc != 2 * RUN_N + 1 || tg.Lp % 64 != 0 || rg.n_groups < 1) return hipErrorInvalidValue;
  const int64_t units = ((g.n_ch + 15) / 16) * rg.n_groups;
  // 512-thread workgroups (2 per CU: 16 waves), prefetch depth 1, registers
  // capped for 4 waves per SIMD: 12.77 ms vs 13.09-13.12 for depth 2 at the
  // compiler's 144 VGPRs on cfg3 (in-process A/B, profiles/archive_r01_r03.md (r02_ab_k1_minw.txt))
#ifdef LFD_DIAG
  // timing-only modes (results invalid): LFD_RUN_MODE=1 loads only, =4 no run epilogue
  if (const char *v = knob("LFD_RUN_MODE")) {
    const int mode = std::atoi(v);
    if (mode == 1) return run_k1<1, 1, 512, 4>(x, s_ch, n_t, g, taps, tg, rg, Y0, AG, units, st);
    if (mode == 4) return run_k1<1, 4, 512, 4>(x, s_ch, n_t, g, taps, tg, rg, Y0, AG, units, st);
  }
#endif
  return run_k1<1, 0, 512, 4>(x, s_ch, n_t, g, taps, tg, rg, Y0, AG, units, st);
}

hipError_t launch_block_runs_mfma_lat(const float *x, int64_t s_ch, int64_t n_t, const BlockGeom &g,
                                      const double *taps, const TapGeom &tg, const RunGeom &rg, double *Y0,
                                      double *AG, hipStream_t st) {
  if (tg.nc <= 2 * RUN_N || tg.nc > 2 * RUN_N + LAT_MAX_OFF || tg.Lp % 64 != 0 || rg.n_groups < 1)
    return hipErrorInvalidValue;
  const int64_t units = ((g.n_ch + 15) / 16) * rg.n_groups;
  return run_k1<1, 0, 512, 4, true>(x, s_ch, n_t, g, taps, tg, rg, Y0, AG, units, st);
}

// ---------------------------------------------------------------------------
// k_run_outputs — the outputs of every run, after k_chunk_scan<2, true, true>
// has carried the states: one wave = 64 channels x one run slot j (runs of
// all chunks, SR / TR layout), y(ks + p) = y0(ks + p) + A[len][p] S_in +
// B[len-1-p] T_in (+ the chunk's p0 correction at block kb).  Outputs leave
// through LDS as 8 rows x 8 consecutive samples per store instruction.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_run_outputs(BlockGeom g, const ChunkGeom *__restrict__ cgs, RunGeom rg,
                                                     const int *__restrict__ slot_chunk,
                                                     const double *__restrict__ Y0, const double *__restrict__ SR,
                                                     const double *__restrict__ TR, const double *__restrict__ CR,
                                                     double *__restrict__ y, int64_t ys_ch, int64_t ys_t) {
  constexpr int N = RUN_N;
  // only the output constants A[len][p], B[d] (2.5 KB; the whole RunConst
  // is 12 KB, and a 1,250-channel shard launches ~2,200 of these groups)
  __shared__ double sA[RUN_R + 1][RUN_R][4], sB[RUN_R][4];
  __shared__ double outs[4][64][RUN_R + 1];
  {
    const double *srcA = &rg.rc->A[0][0][0], *srcB = &rg.rc->B[0][0];
    for (int i = threadIdx.x; i < (RUN_R + 1) * RUN_R * 4; i += blockDim.x) (&sA[0][0][0])[i] = srcA[i];
    for (int i = threadIdx.x; i < RUN_R * 4; i += blockDim.x) (&sB[0][0])[i] = srcB[i];
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int64_t n_c64 = (g.n_ch + 63) / 64;
  const int64_t w = uniform64((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6));
  if (w >= n_c64 * rg.n_sr) return;
  const int64_t c64 = w % n_c64, j = w / n_c64;
  const int64_t ch = c64 * 64 + lane;
  const bool valid = ch < g.n_ch;
  const int c = __builtin_amdgcn_readfirstlane(slot_chunk[j]);
  const ChunkGeom &G = cgs[c];
  const int64_t r = G.r0 + (j - G.sr_off);
  const int64_t ks = rg.run_ks[r];
  const int len = rg.run_len[r];
  const int kst = (int)G.kstep;
  auto is_out = [&](int64_t k) {
    return k >= G.kout0 && k < G.kout1 && (kst == 1 || (int)(k - G.kout0) % kst == 0);
  };
  auto out_j = [&](int64_t k) -> int64_t {
    return G.jout0 + (kst == 1 ? k - G.kout0 : (int64_t)((int)(k - G.kout0) / kst));
  };
  const int64_t chc = valid ? ch : g.n_ch - 1;
  double sin[N], tin[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    sin[i] = SR[sf_index(j, i, chc, rg.n_sr, N)];
    tin[i] = TR[sf_index(j, i, chc, rg.n_sr, N)];
  }
  const double *y0b = Y0 + ((chc >> 4) * g.nb) * 16 + (chc & 15);
  const double cr = CR[c * (n_c64 * 64) + chc];
  double ov[RUN_R];
#pragma unroll
  for (int pp = 0; pp < RUN_R; ++pp) {
    const int64_t k = ks + pp;
    ov[pp] = 0.0;
    if (pp >= len || !is_out(k)) continue;
    double acc = y0b[k * 16] + (k == G.kb ? cr : 0.0);
    const double *A = sA[len][pp];
    const double *B = sB[len - 1 - pp];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      acc = fma(A[i], sin[i], acc);
      acc = fma(B[i], tin[i], acc);
    }
    ov[pp] = acc;
  }
  if (c64 * 64 + 63 < g.n_ch) {
    double(*wl)[RUN_R + 1] = outs[(threadIdx.x >> 6) & 3];
#pragma unroll
    for (int pp = 0; pp < RUN_R; ++pp) wl[lane][pp] = ov[pp];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int e = lane & 7;
    const int64_t k = ks + e;
    const bool ok = e < len && is_out(k);
    double *yb = y + (c64 * 64) * ys_ch + (ok ? out_j(k) : 0) * ys_t;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int row = m * 8 + (lane >> 3);
      const double v = wl[row][e];
      if (ok) yb[row * ys_ch] = v;
    }
  } else if (valid) {
#pragma unroll
    for (int pp = 0; pp < RUN_R; ++pp) {
      const int64_t k = ks + pp;
      if (pp < len && is_out(k)) y[ch * ys_ch + out_j(k) * ys_t] = ov[pp];
    }
  }
}

// ---------------------------------------------------------------------------
// k_fold_runs — run mode for the K1 kernels that emit per-block functionals
// F (the recurrence kernels: strided / time-major / unaligned rows; the MFMA
// kernel when taps + run buffers exceed LDS, L = 2000).  Applies the same
// run epilogue as k_block_runs_mfma (forward prefix S0 over the run's blocks,
// reverse inputs v = e_r0 + M S0 and pg = p0 + G0.S0, backward sweep from a
// zero state) to F and writes Y0 and the run aggregates, so the scan walks
// runs (9x fewer steps) instead of blocks.  One lane = one channel (64
// consecutive channels per wave: 4 x 128-B pieces per F load), one wave = one
// run; the whole run (<= RUN_R blocks) stays in registers.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fold_runs(const double *__restrict__ F, BlockGeom g,
                                                   RunGeom rg, double *__restrict__ Y0,
                                                   double *__restrict__ AG) {
  constexpr int N = RUN_N;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t n_c64 = (g.n_ch + 63) / 64;
  const int64_t unit = (int64_t)blockIdx.x * 4 + wave;  // run-major: r = unit / n_c64
  if (unit >= n_c64 * rg.n_runs) return;
  const int64_t r = unit / n_c64, c64 = unit % n_c64;
  const int64_t ch = c64 * 64 + lane;
  if (ch >= g.n_ch) return;
  const RunConst &rc = *rg.rc;
  double PhiF[16], Mm[16], PhiR[16], G0[4], H0[4];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    PhiF[i] = rc.PhiF[i];
    Mm[i] = rc.M[i];
    PhiR[i] = rc.PhiR[i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    G0[i] = rc.G0[i];
    H0[i] = rc.H0[i];
  }
  const int64_t ks = rg.run_ks[r];
  const int len = rg.run_len[r];
  double S0[N] = {0.0, 0.0, 0.0, 0.0};
  double v[RUN_R][N], pg[RUN_R];
#pragma unroll
  for (int p = 0; p < RUN_R; ++p) {
    if (p < len) {
      const double *Fo = F + f_index(ks + p, 0, ch, g.nb, 2 * N + 1);
      double ef[N], er[N];
#pragma unroll
      for (int i = 0; i < N; ++i) {
        ef[i] = Fo[i * F_CSTRIDE];
        er[i] = Fo[(N + i) * F_CSTRIDE];
      }
      double pgp = Fo[2 * N * F_CSTRIDE];
      double sn[N];
#pragma unroll
      for (int i = 0; i < N; ++i) {
        double vi = er[i], si = ef[i];
#pragma unroll
        for (int j = 0; j < N; ++j) {
          vi = fma(Mm[i * 4 + j], S0[j], vi);
          si = fma(PhiF[i * 4 + j], S0[j], si);
        }
        v[p][i] = vi;
        sn[i] = si;
      }
#pragma unroll
      for (int j = 0; j < N; ++j) pgp = fma(G0[j], S0[j], pgp);
      pg[p] = pgp;
#pragma unroll
      for (int i = 0; i < N; ++i) S0[i] = sn[i];
    }
  }
  double T[N] = {0.0, 0.0, 0.0, 0.0};
  double *y0o = Y0 + ((ch >> 4) * g.nb + ks) * 16 + (ch & 15);
#pragma unroll
  for (int p = RUN_R - 1; p >= 0; --p) {
    if (p < len) {
      double y0 = pg[p];
#pragma unroll
      for (int j = 0; j < N; ++j) y0 = fma(H0[j], T[j], y0);
      y0o[p * 16] = y0;
      double nt[N];
#pragma unroll
      for (int i = 0; i < N; ++i) {
        double acc = v[p][i];
#pragma unroll
        for (int j = 0; j < N; ++j) acc = fma(PhiR[i * 4 + j], T[j], acc);
        nt[i] = acc;
      }
#pragma unroll
      for (int i = 0; i < N; ++i) T[i] = nt[i];
    }
  }
  double *ag = AG + (((ch >> 4) * rg.n_runs + r) * 8) * 16 + (ch & 15);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    ag[i * 16] = S0[i];
    ag[(4 + i) * 16] = T[i];
  }
}

// ---------------------------------------------------------------------------
// k_seg_fwd / k_seg_bwd — the run chains of the deferred scan cut into
// segments (SegGeom): a workgroup = one chunk x 64 channels, wave w = segment
// w, lane = channel.  Forward: each segment's aggregate from a zero state,
// the entering state S_w = P_{w-1} (... (P_0 S_head + A_0) ...) + A_{w-1}
// over the earlier segments (LDS), then the segment again from S_w writing
// S_in of every run (SR); the chunk's last segment leaves the state after the
// last run for the tail (SC).  Backward the same with T from the right:
// T(ks) = PhiR^len T + E_r + C[len] S_in (+ the FIR-history correction at
// run r0), writing the T entering every run (TR).  Between the two, the
// head and the tail run in k_chunk_scan<..., SEGM = 1 / 2>.  Each thread's
// chain shrinks from a chunk's runs to a segment's (lattice plans: ~1,350 ->
// ~85 runs).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_seg_fwd(BlockGeom g, const ChunkGeom *__restrict__ cgs, RunGeom rg,
                                                  const SegGeom *__restrict__ sgs, int seg_max,
                                                  const double *__restrict__ AG, double *__restrict__ SR,
                                                  double *__restrict__ SC) {
  constexpr int N = RUN_N;
  __shared__ double sPF[RUN_R + 1][16];
  __shared__ double agg[SEG_MAX][64][N];
  for (int i = threadIdx.x; i < (RUN_R + 1) * 16; i += blockDim.x) (&sPF[0][0])[i] = (&rg.rc->PhiFp[0][0])[i];
  __syncthreads();
  const int64_t n_c64 = (g.n_ch + 63) / 64, ch64 = n_c64 * 64;
  const int64_t c = blockIdx.x / n_c64, c64 = blockIdx.x % n_c64;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t ch = c64 * 64 + lane;
  const bool valid = ch < g.n_ch;
  const int64_t chc = valid ? ch : g.n_ch - 1;
  const ChunkGeom &G = cgs[c];
  const SegGeom &sg = sgs[c * seg_max + wv];
  const int64_t ra = sg.ra, rb = sg.rb;
  const double *agb = AG + (((chc >> 4) * rg.n_runs) * 8) * 16 + (chc & 15);
  double cf[N];
#pragma unroll
  for (int i = 0; i < N; ++i) cf[i] = ra == G.r0 ? SC[(c * SC_N + SC_CORR + i) * ch64 + chc] : 0.0;
  auto step = [&](int64_t r, double (&S)[N]) {
    const int len = rg.run_len[r];
    const double *P = sPF[len];
    double ns[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      double acc = agb[(r * 8 + i) * 16] + (r == G.r0 ? cf[i] : 0.0);
#pragma unroll
      for (int j = 0; j < N; ++j) acc = fma(P[i * 4 + j], S[j], acc);
      ns[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) S[i] = ns[i];
  };
  double a[N] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t r = ra; r < rb; ++r) step(r, a);
#pragma unroll
  for (int i = 0; i < N; ++i) agg[wv][lane][i] = a[i];
  __syncthreads();
  if (ra >= rb) return;
  double S[N];
#pragma unroll
  for (int i = 0; i < N; ++i) S[i] = SC[(c * SC_N + SC_HS + i) * ch64 + chc];
  for (int k = 0; k < wv; ++k) {
    const SegGeom &sk = sgs[c * seg_max + k];
    if (sk.ra >= sk.rb) continue;
    double ns[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      double acc = agg[k][lane][i];
#pragma unroll
      for (int j = 0; j < N; ++j) acc = fma(sk.P[i * 4 + j], S[j], acc);
      ns[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) S[i] = ns[i];
  }
  for (int64_t r = ra; r < rb; ++r) {
    if (valid) {
      double *sr = SR + sf_index(G.sr_off + (r - G.r0), 0, ch, rg.n_sr, N);
#pragma unroll
      for (int i = 0; i < N; ++i) sr[i * SF_ISTRIDE] = S[i];
    }
    step(r, S);
  }
  if (sg.last && valid)
#pragma unroll
    for (int i = 0; i < N; ++i) SC[(c * SC_N + SC_SE + i) * ch64 + ch] = S[i];
}

__global__ __launch_bounds__(1024) void k_seg_bwd(BlockGeom g, const ChunkGeom *__restrict__ cgs, RunGeom rg,
                                                  const SegGeom *__restrict__ sgs, int seg_max,
                                                  const double *__restrict__ AG, const double *__restrict__ SR,
                                                  double *__restrict__ TR, const double *__restrict__ SC) {
  constexpr int N = RUN_N;
  __shared__ double sPR[RUN_R + 1][16], sC[RUN_R + 1][16];
  __shared__ double agg[SEG_MAX][64][N];
  for (int i = threadIdx.x; i < (RUN_R + 1) * 16; i += blockDim.x) {
    (&sPR[0][0])[i] = (&rg.rc->PhiRp[0][0])[i];
    (&sC[0][0])[i] = (&rg.rc->C[0][0])[i];
  }
  __syncthreads();
  const int64_t n_c64 = (g.n_ch + 63) / 64, ch64 = n_c64 * 64;
  const int64_t c = blockIdx.x / n_c64, c64 = blockIdx.x % n_c64;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t ch = c64 * 64 + lane;
  const bool valid = ch < g.n_ch;
  const int64_t chc = valid ? ch : g.n_ch - 1;
  const ChunkGeom &G = cgs[c];
  const SegGeom &sg = sgs[c * seg_max + wv];
  const int64_t ra = sg.ra, rb = sg.rb;
  const double *agb = AG + (((chc >> 4) * rg.n_runs) * 8) * 16 + (chc & 15);
  double cr[N];
#pragma unroll
  for (int i = 0; i < N; ++i) cr[i] = ra == G.r0 ? SC[(c * SC_N + SC_CORR + N + i) * ch64 + chc] : 0.0;
  auto step = [&](int64_t r, double (&T)[N]) {
    const int len = rg.run_len[r];
    const double *PR = sPR[len], *CC = sC[len];
    const double *sr = SR + sf_index(G.sr_off + (r - G.r0), 0, chc, rg.n_sr, N);
    double sin[N], nt[N];
#pragma unroll
    for (int i = 0; i < N; ++i) sin[i] = sr[i * SF_ISTRIDE];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      double acc = agb[(r * 8 + 4 + i) * 16] + (r == G.r0 ? cr[i] : 0.0);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        acc = fma(PR[i * 4 + j], T[j], acc);
        acc = fma(CC[i * 4 + j], sin[j], acc);
      }
      nt[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) T[i] = nt[i];
  };
  double b[N] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t r = rb - 1; r >= ra; --r) step(r, b);
#pragma unroll
  for (int i = 0; i < N; ++i) agg[wv][lane][i] = b[i];
  __syncthreads();
  if (ra >= rb) return;
  double T[N];
#pragma unroll
  for (int i = 0; i < N; ++i) T[i] = SC[(c * SC_N + SC_TE + i) * ch64 + chc];
  for (int k = seg_max - 1; k > wv; --k) {
    const SegGeom &sk = sgs[c * seg_max + k];
    if (sk.ra >= sk.rb) continue;
    double nt[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      double acc = agg[k][lane][i];
#pragma unroll
      for (int j = 0; j < N; ++j) acc = fma(sk.Q[i * 4 + j], T[j], acc);
      nt[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) T[i] = nt[i];
  }
  for (int64_t r = rb - 1; r >= ra; --r) {
    if (valid) {
      double *tr = TR + sf_index(G.sr_off + (r - G.r0), 0, ch, rg.n_sr, N);
#pragma unroll
      for (int i = 0; i < N; ++i) tr[i * SF_ISTRIDE] = T[i];
    }
    step(r, T);
  }
}


// ---------------------------------------------------------------------------
// k_scan_fused — the run-mode chunk scan in ONE launch, latency-lean.  A
// 256-thread workgroup = one chunk x 16 channels (one K1 channel group);
// lane (col = l & 15, s = l >> 4) owns channel col and segment s of the
// chunk's runs (FU_SEG = 16 segments of <= FU_SEGR runs: SegGeom table).  A
// lane holds its segment's run inputs in registers, so every chain below is
// FMAs on registers / LDS and the whole scan costs a handful of memory round
// trips instead of one per run step:
//   1. every lane loads its runs' E_f (one round trip); RunConst and the
//      segments' transitions P / Q go to LDS; segment 0's lanes run the left
//      edge (scan_head: S_head, the corrections);
//   2. forward aggregate of the segment from a zero state (segment 0: with
//      the forward correction at r0), to LDS;
//   3. S entering the segment = the earlier segments folded into S_head
//      (P_k S + a_k); the segment again from it: S_in of every run (kept, and
//      stored to SR); the chunk's last segment's lanes then run the right edge
//      (scan_tail: T_end, the tail output);
//   4. E_r loaded; backward aggregate from a zero T, to LDS;
//   5. T entering the segment from the right (Q_k T + b_k folded into T_end);
//      the segment backward: T_in of every run to TR;
//   6. all 256 lanes form the chunk's outputs in parallel, one (run, channel)
//      per lane and step: y(ks + p) = y0(ks + p) + A[len][p] S_in +
//      B[len-1-p] T_in (+ the p0 correction at block kb).
// Same algebra as k_chunk_scan<2, true, true> + k_run_outputs (segment 0 and
// the last segment bit-identical; the others differ by the combine's
// summation order, like k_seg_fwd / k_seg_bwd).  Chunks of more than
// FU_SEG x FU_SEGR runs take the multi-launch scans.
// ---------------------------------------------------------------------------
constexpr int FU_SEG = 16;  // segments per chunk (lfd_internal.h FU_SEG_HOST)
constexpr int FU_SEGR = 5;  // runs per segment held in registers
static_assert(FU_SEG == FU_SEG_HOST && FU_SEGR == FU_SEGR_HOST, "fused scan geometry");
#ifdef LFD_DIAG
// k_scan_fused timing-only variants (LFD_FU_DIAG, results invalid): bit 1 no
// y stores in the T walk, 2 no y0 loads
__constant__ int g_fu_diag = 0;
// k_scan_fused phase stamps (LFD_FU_TIMES): [wg < 8192][wave < 4][8]
__device__ uint64_t g_fu_times[8192 * 4 * 8];
#endif
// (registers for 3 workgroups per CU — one round of the 1,250-channel
// shard's 553 workgroups — spill 34 dwords: scan 0.073 -> 0.080 ms,
// profiles/r05_scan_tailmap.txt)
__global__ __launch_bounds__(256, 2) void k_scan_fused(
    const float *__restrict__ x, int64_t s_ch, int64_t s_t, BlockGeom g, int padlen, const ScanConst sc,
    const ChunkGeom *__restrict__ cgs, int64_t n_chunks, RunGeom rg, const SegGeom *__restrict__ sgs,
    const double *__restrict__ Y0, const double *__restrict__ AG, double *__restrict__ SR,
    double *__restrict__ TR, double *__restrict__ TP, double *__restrict__ y, int64_t ys_ch, int64_t ys_t) {
  constexpr int N = RUN_N, NF = 2 * N + 1, SR_ = FU_SEGR;
#ifdef LFD_DIAG
  // phase stamps of every wave, 100 MHz s_memrealtime
  uint64_t *fu_t = g_fu_times + ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8;
  int fu_i = 0;
#define FU_STAMP()                                                          \
  do {                                                                      \
    if (blockIdx.x < 8192) {                                                \
      const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                 \
      if ((threadIdx.x & 63) == 0 && fu_i < 8) fu_t[fu_i] = t_;             \
    }                                                                       \
    ++fu_i;                                                                 \
  } while (0)
#else
#define FU_STAMP() \
  do {             \
  } while (0)
#endif
  FU_STAMP();
  __shared__ RunConst rcs;
  __shared__ double Ps[FU_SEG][16], Qs[FU_SEG][16];
  __shared__ double aggf[FU_SEG][N][16], aggb[FU_SEG][N][16], hS[N][16], tT[N][16], corr[NF][16], tY[16];
  __shared__ double otile[4][64][RUN_R + 1];  // output staging per wave
  __shared__ int64_t omk[4][64];             // its run's first block
  __shared__ int oml[4][64];                 // its run's length (0: nothing to store)
  const int64_t n_cg = (g.n_ch + 15) / 16;
  const int64_t c = blockIdx.x / n_cg, cg = blockIdx.x % n_cg;
  const int col = threadIdx.x & 15, sg = threadIdx.x >> 4;
  const int64_t ch = cg * 16 + col;
  const bool valid = ch < g.n_ch;
  const int64_t chc = valid ? ch : g.n_ch - 1;
  const ChunkGeom G = cgs[c];
  const SegGeom *sgc = sgs + c * FU_SEG;
  const int64_t ra = sgc[sg].ra, rb = sgc[sg].rb;
  const int nrun = (int)(rb - ra);  // 0 .. FU_SEGR
  // the lanes that run the right edge: the chunk's last active segment
  // (segment 0 when the chunk has no full blocks)
  int tail_seg = 0;
  for (int k = FU_SEG - 1; k > 0; --k)
    if (sgc[k].ra < sgc[k].rb) {
      tail_seg = k;
      break;
    }
  // (lanes past n_ch mirror channel n_ch - 1 bit for bit — its aggregates,
  // samples and edges — so their tail scratch writes, which share that
  // channel's TP slots, carry the same values; K1 folds that leave the
  // padding channels' Y0 / AG unwritten (k_fold_runs) are read nowhere)
  const double *agb = AG + (((chc >> 4) * rg.n_runs) * 8) * 16 + (chc & 15);
  (void)SR;
  (void)TR;
  // ---- 1. run inputs (E_f) into registers; constants into LDS; the edges'
  // sample rows touched (their lines and translations warm when the left /
  // right edge walks run)
  const float *xc = x + chc * s_ch;
  float touch = 0.f;  // (consumed by an empty asm at the end: the load stays in flight)
  if (sg == 0 || sg == tail_seg) {
    const int64_t t0 = sg == 0 ? G.s0 : max(G.s0, G.s1 - padlen - 1);
#pragma unroll
    for (int i = 0; i < 2; ++i) touch += xc[min(t0 + 16 * i, G.s1) * s_t];
  }
  int len[SR_];
  double ef[SR_][N];
#pragma unroll
  for (int u = 0; u < SR_; ++u) {
    const int64_t r = u < nrun ? ra + u : G.r0;  // (a clamped, unused load past the segment)
    len[u] = u < nrun ? rg.run_len[r] : 0;
#pragma unroll
    for (int i = 0; i < N; ++i) ef[u][i] = agb[(r * 8 + i) * 16];
  }
  {
    // (every load issued before the LDS writes: one round trip)
    constexpr int NRC = (int)(sizeof(RunConst) / sizeof(double)), NRI = (NRC + 255) / 256;
    double v[NRI];
#pragma unroll
    for (int j = 0; j < NRI; ++j) {
      const int i = (int)threadIdx.x + 256 * j;
      v[j] = i < NRC ? (&rg.rc->PhiFp[0][0])[i] : 0.0;
    }
    const double pv = sgc[threadIdx.x >> 4].P[threadIdx.x & 15], qv = sgc[threadIdx.x >> 4].Q[threadIdx.x & 15];
#pragma unroll
    for (int j = 0; j < NRI; ++j) {
      const int i = (int)threadIdx.x + 256 * j;
      if (i < NRC) (&rcs.PhiFp[0][0])[i] = v[j];
    }
    (&Ps[0][0])[threadIdx.x] = pv;
    (&Qs[0][0])[threadIdx.x] = qv;
  }
  __syncthreads();
  FU_STAMP();
  const SeqR<2> R(sc.r);
  double S[N] = {0.0, 0.0, 0.0, 0.0};
  if (sg == 0) {
    double cr[NF];
    scan_head<2, true>(xc, s_t, G, g.L, padlen, R, sc, &rcs, AG, rg, chc, S, cr);
#pragma unroll
    for (int i = 0; i < N; ++i) hS[i][col] = S[i];
#pragma unroll
    for (int i = 0; i < NF; ++i) corr[i][col] = cr[i];
  }
  // right edge, state-free part: the edge is affine in the S entering it
  // (SegGeom::TM / tm, host-simulated), so its lanes walk it from S = 0 now
  // — beside the left edge, while the forward chain is not known yet — and
  // add TM S after the forward walk (step 3)
  const bool tmap = sgc[tail_seg].tmap != 0;
  if (tmap && sg == tail_seg) {
    double Sz[N] = {0.0, 0.0, 0.0, 0.0}, Tz[N], yz = 0.0;
    scan_tail<2>(xc, s_t, G, padlen, R, sc, Sz, TP + c * g.n_ch + chc, n_chunks * g.n_ch, y, ch, ys_ch, ys_t, Tz,
                 false, &yz);
#pragma unroll
    for (int i = 0; i < N; ++i) tT[i][col] = Tz[i];
    tY[col] = yz;
  }
  // (segment 0's lanes wrote corr themselves: a wave reads its own LDS writes
  // in order; the other segments never reach run r0)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  auto fstep = [&](double (&St)[N], const double (&e)[N], int ln, int64_t r) {
    const double *P = rcs.PhiFp[ln];
    double ns[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      double acc = e[i] + (r == G.r0 ? corr[i][col] : 0.0);
#pragma unroll
      for (int j = 0; j < N; ++j) acc = fma(P[i * 4 + j], St[j], acc);
      ns[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) St[i] = ns[i];
  };
  auto bstep = [&](double (&Tt)[N], const double (&sin)[N], const double (&er)[N], int ln, int64_t r) {
    const double *PR = rcs.PhiRp[ln], *CC = rcs.C[ln];
    double nr[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      double acc = er[i] + (r == G.r0 ? corr[N + i][col] : 0.0);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        acc = fma(PR[i * 4 + j], Tt[j], acc);
        acc = fma(CC[i * 4 + j], sin[j], acc);
      }
      nr[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) Tt[i] = nr[i];
  };
  // ---- 2. forward aggregates
  {
    double a[N] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int u = 0; u < SR_; ++u)
      if (u < nrun) fstep(a, ef[u], len[u], ra + u);
#pragma unroll
    for (int i = 0; i < N; ++i) aggf[sg][i][col] = a[i];
  }
  __syncthreads();
  FU_STAMP();
  // ---- 3. true forward states; right edge
  double sin[SR_][N];
#pragma unroll
  for (int i = 0; i < N; ++i) S[i] = hS[i][col];
  for (int k = 0; k < sg; ++k) {
    if (sgc[k].ra >= sgc[k].rb) continue;
    double ns[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      double acc = aggf[k][i][col];
#pragma unroll
      for (int j = 0; j < N; ++j) acc = fma(Ps[k][i * 4 + j], S[j], acc);
      ns[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) S[i] = ns[i];
  }
#pragma unroll
  for (int u = 0; u < SR_; ++u) {
#pragma unroll
    for (int i = 0; i < N; ++i) sin[u][i] = S[i];
    if (u < nrun) fstep(S, ef[u], len[u], ra + u);
  }
  // the segment's y0: the last run's in flight behind the right edge, the
  // backward aggregates and the reverse combine; each earlier run's loads one
  // run ahead in the T walk (holding all of them took 80 VGPRs: 2 workgroups
  // per CU instead of 3)
  const double *y0b = Y0 + ((chc >> 4) * g.nb) * 16 + (chc & 15);
  int64_t ksv[SR_];
#pragma unroll
  for (int u = 0; u < SR_; ++u) ksv[u] = u < nrun ? rg.run_ks[ra + u] : 0;
  auto y0run = [&](int u, double (&yr)[RUN_R]) {
#pragma unroll
    for (int pp = 0; pp < RUN_R; ++pp)
      yr[pp] = (u >= nrun || pp >= len[u] || (LFD_DG(g_fu_diag) & 2)) ? 0.0 : y0b[(ksv[u] + pp) * 16];
  };
  double ycur[RUN_R];
  y0run(SR_ - 1, ycur);
  if (sg == tail_seg) {
    double T[N];
    if (tmap) {
      const double *TM = sgc[tail_seg].TM, *tm = sgc[tail_seg].tm;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        double acc = tT[i][col];
#pragma unroll
        for (int j = 0; j < N; ++j) acc = fma(TM[i * 4 + j], S[j], acc);
        T[i] = acc;
      }
      if (G.tail_out_j >= 0 && valid) {
        double yv = tY[col];
#pragma unroll
        for (int j = 0; j < N; ++j) yv = fma(tm[j], S[j], yv);
        y[ch * ys_ch + G.tail_out_j * ys_t] = yv;
      }
    } else {
      scan_tail<2>(xc, s_t, G, padlen, R, sc, S, TP + c * g.n_ch + chc, n_chunks * g.n_ch, y, ch, ys_ch, ys_t, T,
                   valid);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) tT[i][col] = T[i];
  }
  // E_r of the segment's runs (after the right edge: fewer live registers there)
  // (step 4 holds them all; the T walk re-reads each run's, one run ahead,
  // from the cache, so they are not live through step 5)
  auto errun = [&](int u, double (&e)[N]) {
    const int64_t r = u < nrun ? ra + u : G.r0;
#pragma unroll
    for (int i = 0; i < N; ++i) e[i] = agb[(r * 8 + 4 + i) * 16];
  };
  double er[SR_][N];
#pragma unroll
  for (int u = 0; u < SR_; ++u) errun(u, er[u]);
  FU_STAMP();
  // ---- 4. backward aggregates
  {
    double b[N] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int u = SR_ - 1; u >= 0; --u)
      if (u < nrun) bstep(b, sin[u], er[u], len[u], ra + u);
#pragma unroll
    for (int i = 0; i < N; ++i) aggb[sg][i][col] = b[i];
  }
  __syncthreads();
  FU_STAMP();
  // ---- 5. true reverse states; the outputs of every run as its T_in is known
  const int kst = (int)G.kstep;
  auto is_out = [&](int64_t k) {
    return k >= G.kout0 && k < G.kout1 && (kst == 1 || (int)(k - G.kout0) % kst == 0);
  };
  auto out_j = [&](int64_t k) -> int64_t {
    return G.jout0 + (kst == 1 ? k - G.kout0 : (int64_t)((int)(k - G.kout0) / kst));
  };
  const double crk = corr[2 * N][col];
  double T[N];
#pragma unroll
  for (int i = 0; i < N; ++i) T[i] = tT[i][col];
  for (int k = FU_SEG - 1; k > sg; --k) {
    if (sgc[k].ra >= sgc[k].rb) continue;
    double nt[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      double acc = aggb[k][i][col];
#pragma unroll
      for (int j = 0; j < N; ++j) acc = fma(Qs[k][i * 4 + j], T[j], acc);
      nt[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) T[i] = nt[i];
  }
  FU_STAMP();
  // outputs leave through a per-wave LDS tile: lane g's 8 outputs of run u
  // (its channel, its segment's run) go out as 8 lanes x 4 consecutive bytes,
  // so a store instruction writes 8 row pieces of 32 B (one L2 request each)
  // instead of 64 scattered 4-B lanes
  const int wv = threadIdx.x >> 6, ln64 = threadIdx.x & 63;
  double(*tile)[RUN_R + 1] = otile[wv];
  double ecur[N];
#pragma unroll
  for (int i = 0; i < N; ++i) ecur[i] = er[SR_ - 1][i];
#pragma unroll
  for (int u = SR_ - 1; u >= 0; --u) {
    const bool live = u < nrun;
    const int ln = live ? len[u] : 0;
    const int64_t ks = ksv[u];
    double ynext[RUN_R], enext[N];
    if (u > 0) {
      y0run(u - 1, ynext);
      errun(u - 1, enext);
    }
#pragma unroll
    for (int pp = 0; pp < RUN_R; ++pp) {
      const int64_t k = ks + pp;
      double o = 0.0;
      if (pp < ln && is_out(k)) {
        double acc = ycur[pp] + (k == G.kb ? crk : 0.0);
        const double *A = rcs.A[ln][pp];
        const double *B = rcs.B[ln - 1 - pp];
#pragma unroll
        for (int j = 0; j < N; ++j) {
          acc = fma(A[j], sin[u][j], acc);
          acc = fma(B[j], T[j], acc);
        }
        o = acc;
      }
      tile[ln64][pp] = o;
    }
    omk[wv][ln64] = ks;
    oml[wv][ln64] = valid ? ln : 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int e = ln64 & 7;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int gl = m * 8 + (ln64 >> 3);  // source lane: channel cg*16 + (gl & 15)
      const int64_t kg = omk[wv][gl] + e;
      const bool ok = e < oml[wv][gl] && is_out(kg) && !(LFD_DG(g_fu_diag) & 1);
      if (ok) y[(cg * 16 + (gl & 15)) * ys_ch + out_j(kg) * ys_t] = tile[gl][e];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (live) bstep(T, sin[u], ecur, ln, ra + u);
    if (u > 0) {
#pragma unroll
      for (int pp = 0; pp < RUN_R; ++pp) ycur[pp] = ynext[pp];
#pragma unroll
      for (int i = 0; i < N; ++i) ecur[i] = enext[i];
    }
  }
  FU_STAMP();
#undef FU_STAMP
  asm volatile("" ::"v"(touch));
}

hipError_t launch_scan_fused(const float *x, int64_t s_ch, int64_t s_t, const BlockGeom &g, int padlen,
                             const ScanConst &sc, const ChunkGeom *cg, int64_t n_chunks, const RunGeom &rg,
                             const SegGeom *seg_fu, const double *Y0, const double *AG, double *SR, double *TR,
                             double *TP, double *y, int64_t ys_ch, int64_t ys_t, hipStream_t st) {
  const unsigned nwg = (unsigned)(n_chunks * ((g.n_ch + 15) / 16));
#ifdef LFD_DIAG
  {
    static int fu_diag = -1;
    const char *v = knob("LFD_FU_DIAG");
    const int want = v ? std::atoi(v) : 0;
    if (want != fu_diag) {
      hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_fu_diag), &want, sizeof(int));
      if (e != hipSuccess) return e;
      fu_diag = want;
    }
  }
#endif
  k_scan_fused<<<nwg, 256, 0, st>>>(x, s_ch, s_t, g, padlen, sc, cg, n_chunks, rg, seg_fu, Y0, AG, SR, TR, TP, y,
                                    ys_ch, ys_t);
#ifdef LFD_DIAG
  if (knob_flag("LFD_FU_TIMES")) {
    // phase durations (us) averaged over workgroups: per wave, stamps 0
    // start, 1 constants + E_f loaded, 2 forward aggregates (+ left edge),
    // 3 forward walk (+ right edge, E_r issued), 4 backward aggregates, 5 T
    // walk + outputs, 6 (unused)
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    const unsigned nw = std::min(nwg, 8192u);
    std::vector<uint64_t> t((size_t)nw * 4 * 8);
    e = hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_fu_times), t.size() * sizeof(uint64_t));
    if (e != hipSuccess) return e;
    uint64_t t0 = ~0ull, t1 = 0;
    for (unsigned b = 0; b < nw; ++b)
      for (int w = 0; w < 4; ++w) {
        t0 = std::min(t0, t[((size_t)b * 4 + w) * 8]);
        t1 = std::max(t1, t[((size_t)b * 4 + w) * 8 + 6]);
      }
    for (int w = 0; w < 4; ++w) {
      double d[6] = {0};
      for (unsigned b = 0; b < nw; ++b)
        for (int i = 0; i < 6; ++i)
          d[i] += 0.01 * (double)(t[((size_t)b * 4 + w) * 8 + i + 1] - t[((size_t)b * 4 + w) * 8 + i]);
      fprintf(stderr, "k_scan_fused wave %d us: load %.2f fagg+head %.2f fwalk+tail %.2f bagg %.2f combine %.2f "
              "twalk+out %.2f\n", w, d[0] / nw, d[1] / nw, d[2] / nw, d[3] / nw, d[4] / nw, d[5] / nw);
    }
    fprintf(stderr, "k_scan_fused first start -> last end %.2f us over %u workgroups\n", 0.01 * (double)(t1 - t0), nw);
  }
#endif
  return hipGetLastError();
}

// head -> segmented forward -> tail -> segmented backward (CR and the
// deferred outputs as in the unsegmented deferred scan)
static hipError_t launch_seg_scan(const float *x, int64_t s_ch, int64_t s_t, const BlockGeom &g, int padlen,
                                  const ScanConst &sc, const RunGeom &rg, const ChunkGeom *cg, int64_t n_chunks,
                                  const double *Y0, const double *AG, double *SR, double *TP, int64_t tp_len,
                                  double *y, int64_t ys_ch, int64_t ys_t, hipStream_t st, double *TR, double *CR,
                                  const SegGeom *seg, int seg_max, double *SC) {
  const int dthr = n_chunks * g.n_ch < 40000 ? 64 : 256;
  const unsigned nb = nblk(n_chunks * g.n_ch, dthr);
  k_chunk_scan<2, true, true, SCAN_DF, SCAN_DB, 1><<<nb, dthr, 0, st>>>(x, s_ch, s_t, g, padlen, sc, cg, n_chunks, AG,
                                                                       SR, TP, tp_len, y, ys_ch, ys_t, rg, Y0, TR, CR,
                                                                       SC);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const unsigned nwg = (unsigned)(n_chunks * ((g.n_ch + 63) / 64));
  k_seg_fwd<<<nwg, 64 * seg_max, 0, st>>>(g, cg, rg, seg, seg_max, AG, SR, SC);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  k_chunk_scan<2, true, true, SCAN_DF, SCAN_DB, 2><<<nb, dthr, 0, st>>>(x, s_ch, s_t, g, padlen, sc, cg, n_chunks, AG,
                                                                       SR, TP, tp_len, y, ys_ch, ys_t, rg, Y0, TR, CR,
                                                                       SC);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  k_seg_bwd<<<nwg, 64 * seg_max, 0, st>>>(g, cg, rg, seg, seg_max, AG, SR, TR, SC);
  return hipGetLastError();
}

hipError_t launch_fold_runs(const double *F, const BlockGeom &g, const RunGeom &rg, double *Y0,
                            double *AG, hipStream_t st) {
  if (g.nF != 2 * RUN_N + 1 || rg.n_runs < 1) return hipErrorInvalidValue;
  const int64_t units = ((g.n_ch + 63) / 64) * rg.n_runs;
  k_fold_runs<<<nblk(units, 4), 256, 0, st>>>(F, g, rg, Y0, AG);
  return hipGetLastError();
}

hipError_t launch_chunk_scan_runs(const float *x, int64_t s_ch, int64_t s_t, const BlockGeom &g,
                                  int padlen, const ScanConst &sc, const RunGeom &rg,
                                  const ChunkGeom *cg, int64_t n_chunks, const double *Y0,
                                  const double *AG, double *SR, double *TP, int64_t tp_len,
                                  double *y, int64_t ys_ch, int64_t ys_t, hipStream_t st, double *TR,
                                  double *CR, const int *slot_chunk, const SegGeom *seg, int seg_max, double *SC,
                                  const SegGeom *seg_fu, int nw_fu, int *scan_used) {
  int scan_dummy = 0;
  if (!scan_used) scan_used = &scan_dummy;
  // deferred outputs (k_run_outputs) when the scan has few (chunk, channel)
  // threads and is latency-bound: 1,250 ch x 7 chunks (an 8-GPU shard of
  // cfg3) 0.247 -> 0.152 ms, 2,500 ch 0.263 -> 0.191, 5,000 ch equal, 10,000
  // ch 0.339 -> 0.431 (the TR round trip); and when the chunks hold long
  // run chains (dt = 10 s at 1 kHz: ~300 runs per chunk, 0.79 -> 0.67 ms);
  // option LFD_OPT_SCAN_DEFER = 1 / 2 forces in-chain / deferred outputs
  bool defer = n_chunks * g.n_ch < 40000 || rg.n_sr >= 128 * n_chunks;
  // (option 1 / 2 force in-chain / deferred outputs; 3 / 4 fall back to the
  // default choice when their segment tables do not fit the plan)
  if (const int64_t o = option(LFD_OPT_SCAN_DEFER); o == 1 || o == 2) defer = o == 2;
#ifdef LFD_DIAG
  static int diag = -1, threads_ab = 256;
  if (diag < 0) {
    const char *v = knob("LFD_SCAN_DIAG");
    diag = v ? std::atoi(v) : 0;
    if (diag) (void)hipMemcpyToSymbol(HIP_SYMBOL(g_scan_diag), &diag, sizeof(int));
    // workgroup size A/B knob (64, 128 or 256 threads; the kernel's LDS
    // staging is per wave and its launch bound is 256)
    if (const char *t = knob("LFD_SCAN_THREADS")) {
      const int w = std::atoi(t);
      if (w == 64 || w == 128 || w == 256) threads_ab = w;
    }
  }
#endif
  // the fused one-launch segmented scan (option scan_defer = 4; by default
  // when its (chunk, 16-channel) workgroups number <= 6 per CU: latency-bound
  // narrow shards — 1,250 channels x 7 chunks (an 8-GPU share of cfg3):
  // 0.109 -> 0.087 ms (profiles/r05_scan_fused.txt); 2,500 channels (a 4-GPU
  // share) 0.1445 -> 0.1315 ms after the round-6 ring changes; 5,000 equal
  // (profiles/r06_scan_variants.txt)
  const int64_t o_scan = option(LFD_OPT_SCAN_DEFER);
  const bool fused_fits = n_chunks * ((g.n_ch + 15) / 16) <= 6 * (int64_t)cu_count();
  if (seg_fu && nw_fu == FU_SEG && TR && (o_scan == 4 || (o_scan == 0 && fused_fits))) {
    *scan_used = LFD_SCAN_FUSED;
    return launch_scan_fused(x, s_ch, s_t, g, padlen, sc, cg, n_chunks, rg, seg_fu, Y0, AG, SR, TR, TP, y, ys_ch,
                             ys_t, st);
  }
  // segmented chains (option scan_defer = 3, or automatically for long chains
  // on few threads: >= 128 runs per chunk and < 40,000 (chunk, channel)
  // threads — the 3 kHz lattice line's state scan 0.42 -> 0.31 ms; with
  // 40,000 threads (dt = 10 s at 10,000 channels) the unsegmented deferred
  // scan is faster, 0.60 vs 0.72 ms)
  const int64_t o_defer = option(LFD_OPT_SCAN_DEFER);
  const bool segm = seg && SC && seg_max >= 1 && TR && CR && slot_chunk &&
                    (o_defer == 3 || ((o_defer == 0 || o_defer == 4) && n_chunks * g.n_ch < 40000 &&
                                      rg.n_sr >= 128 * n_chunks));
  if (segm) {
    *scan_used = LFD_SCAN_SEGMENTED;
    hipError_t e = launch_seg_scan(x, s_ch, s_t, g, padlen, sc, rg, cg, n_chunks, Y0, AG, SR, TP, tp_len, y, ys_ch,
                                   ys_t, st, TR, CR, seg, seg_max, SC);
    if (e != hipSuccess) return e;
    const int64_t waves = ((g.n_ch + 63) / 64) * rg.n_sr;
    k_run_outputs<<<nblk(waves, 4), 256, 0, st>>>(g, cg, rg, slot_chunk, Y0, SR, TR, CR, y, ys_ch, ys_t);
    return hipGetLastError();
  }
  if (TR && CR && slot_chunk && defer) {
    *scan_used = LFD_SCAN_DEFERRED;
    // narrow shards: 64-thread workgroups (one wave per CU instead of four
    // sharing one): 1,250 channels 0.150 -> 0.126 ms, bit-identical
    // (profiles/archive_r01_r03.md (r03_ab_scan_narrow.txt); A/B knob LFD_SCAN_DEFER_THREADS)
    int dthr = n_chunks * g.n_ch < 40000 ? 64 : 256;
    if (const char *tv = knob("LFD_SCAN_DEFER_THREADS")) dthr = std::atoi(tv) == 64 ? 64 : (std::atoi(tv) == 128 ? 128 : 256);
    const unsigned nb = nblk(n_chunks * g.n_ch, dthr);
    // 16 / 8 runs in flight instead of 4 / 2: dt = 10 s at 1 kHz 0.401 ->
    // 0.352 ms (profiles/archive_r01_r03.md (r03_ab_scan_deep.txt)); the 1,250- / 2,500-channel
    // shards' scan kernel 90.6 -> 74.4 / 99.6 -> 78.3 us by rocprofv3 kernel
    // trace (profiles/r04l_scan_deep.txt); bit-identical (A/B knob
    // LFD_SCAN_DEEP=0/1)
    bool deep = true;
    if (const char *dv = knob("LFD_SCAN_DEEP")) deep = std::atoi(dv) != 0;
    if (deep)
      k_chunk_scan<2, true, true, 16, 8><<<nb, dthr, 0, st>>>(x, s_ch, s_t, g, padlen, sc, cg, n_chunks, AG, SR, TP,
                                                              tp_len, y, ys_ch, ys_t, rg, Y0, TR, CR);
    else
      k_chunk_scan<2, true, true><<<nb, dthr, 0, st>>>(x, s_ch, s_t, g, padlen, sc, cg, n_chunks, AG, SR, TP, tp_len,
                                                       y, ys_ch, ys_t, rg, Y0, TR, CR);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int64_t waves = ((g.n_ch + 63) / 64) * rg.n_sr;
    k_run_outputs<<<nblk(waves, 4), 256, 0, st>>>(g, cg, rg, slot_chunk, Y0, SR, TR, CR, y, ys_ch, ys_t);
    return hipGetLastError();
  }
  int threads = 256;
#ifdef LFD_DIAG
  threads = threads_ab;
#endif
  const unsigned nb = nblk(n_chunks * g.n_ch, threads);
  *scan_used = LFD_SCAN_IN_CHAIN;
  // (ring depth: 3 slots = 2 runs in flight; 2 / 4 / 6 measured equal or
  // slower on cfg3, r06)
  k_chunk_scan<2, true, false, 4, 3><<<nb, threads, 0, st>>>(x, s_ch, s_t, g, padlen, sc, cg, n_chunks, AG, SR, TP,
                                                             tp_len, y, ys_ch, ys_t, rg, Y0);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// k_lat_outputs — the one-pass lattice plan's outputs, every offset in one
// launch: one wave = 64 channels x one run slot; the run's entering states
// (S_in, T_in) are loaded once and its first block (every output block starts
// a run) gives y = y0_d + A_d[len][0] S_in + B_d[len-1] T_in for each offset
// d whose points include that block, into a slot-major scratch
// tmp[(d n_g + j) n_ch + ch] (64 consecutive channels per store).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_lat_outputs(BlockGeom g, const ChunkGeom *__restrict__ cg_off, int64_t n_chunks,
                                                     int n_off, RunGeom rg, const int *__restrict__ slot_chunk,
                                                     const RunConst *__restrict__ rc_off, const double *__restrict__ Y0,
                                                     const double *__restrict__ SR, const double *__restrict__ TR,
                                                     double *__restrict__ tmp, int64_t n_g) {
  constexpr int N = RUN_N;
  __shared__ double sA[LAT_MAX_OFF][RUN_R + 1][4], sB[LAT_MAX_OFF][RUN_R + 1][4];
  for (int i = threadIdx.x; i < n_off * (RUN_R + 1) * 4; i += blockDim.x) {
    const int d = i / ((RUN_R + 1) * 4), rem = i - d * (RUN_R + 1) * 4, len = rem >> 2, e = rem & 3;
    sA[d][len][e] = rc_off[d].A[len][0][e];
    sB[d][len][e] = len >= 1 ? rc_off[d].B[len - 1][e] : 0.0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t n_c64 = (g.n_ch + 63) / 64;
  const int64_t w = uniform64((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6));
  if (w >= n_c64 * rg.n_sr) return;
  const int64_t c64 = w % n_c64, j = w / n_c64;
  const int64_t ch = c64 * 64 + lane;
  const bool valid = ch < g.n_ch;
  const int64_t chc = valid ? ch : g.n_ch - 1;
  const int c = __builtin_amdgcn_readfirstlane(slot_chunk[j]);
  const ChunkGeom &G0 = cg_off[c];
  const int64_t r = G0.r0 + (j - G0.sr_off);
  const int64_t ks = rg.run_ks[r];
  const int len = rg.run_len[r];
  double sin[N], tin[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    sin[i] = SR[sf_index(j, i, chc, rg.n_sr, N)];
    tin[i] = TR[sf_index(j, i, chc, rg.n_sr, N)];
  }
  const int64_t slice = ((g.n_ch + 15) / 16) * g.nb * 16;
  const double *y0b = Y0 + ((chc >> 4) * g.nb + ks) * 16 + (chc & 15);
  for (int d = 0; d < n_off; ++d) {
    const ChunkGeom &G = cg_off[(int64_t)d * n_chunks + c];
    const int64_t kst = G.kstep;
    if (ks < G.kout0 || ks >= G.kout1 || (ks - G.kout0) % kst != 0) continue;
    const int64_t jo = G.jout0 + (ks - G.kout0) / kst;
    double acc = y0b[d * slice];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      acc = fma(sA[d][len][i], sin[i], acc);
      acc = fma(sB[d][len][i], tin[i], acc);
    }
    if (valid) tmp[((int64_t)d * n_g + jo) * g.n_ch + ch] = acc;
  }
}

// ---------------------------------------------------------------------------
// k_blend_grid_sm — the interp1d blend from the slot-major scratch: a
// workgroup = 64 blend points x 64 channels; reads of tmp rows (64 channels)
// and writes of y rows (64 points) both coalesced through an LDS tile.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_blend_grid_sm(const double *__restrict__ tmp, int64_t n_ch,
                                                       const int64_t *__restrict__ bj, const int64_t *__restrict__ bi,
                                                       const double *__restrict__ bw, int64_t nb, double *__restrict__ y,
                                                       int64_t ys_ch, int64_t ys_t, GridGen gen) {
  __shared__ double tile[64][65];
  const int64_t i0 = (int64_t)blockIdx.x * 64, c0 = (int64_t)blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int ii = ty; ii < 64; ii += 4) {
    const int64_t i = i0 + ii, ch = c0 + tx;
    double v = 0.0;
    if (i < nb && ch < n_ch) {
      const int64_t ia = bi[2 * i], ib = bi[2 * i + 1];
      double a = tmp[ia * n_ch + ch];
      if (ib >= 0) {
        double wv;
        if (gen.dts > 0) {
          const int64_t rel = gen.rel0 + bj[i] * gen.step;
          int64_t lo = rel / gen.dts;
          if (rel % gen.dts != 0 && rel < 0) --lo;
          wv = (double)(rel - lo * gen.dts) / (double)gen.dts;
        } else {
          wv = bw[i];
        }
        a = fma(wv, tmp[ib * n_ch + ch] - a, a);
      }
      v = a;
    }
    tile[ii][tx] = v;
  }
  __syncthreads();
  const int64_t i = i0 + tx;
  if (i >= nb) return;
  const int64_t jj = bj[i];
  for (int cc = ty; cc < 64; cc += 4) {
    const int64_t ch = c0 + cc;
    if (ch < n_ch) y[ch * ys_ch + jj * ys_t] = tile[tx][cc];
  }
}

hipError_t launch_blend_grid_sm(const double *tmp, int64_t n_ch, const int64_t *bj, const int64_t *bi,
                                const double *bw, int64_t nb, double *y, int64_t ys_ch, int64_t ys_t, hipStream_t st,
                                const GridGen &gen) {
  if (nb <= 0 || n_ch <= 0) return hipSuccess;
  if ((n_ch + 63) / 64 > 65535) return hipErrorInvalidValue;
  dim3 grid((unsigned)((nb + 63) / 64), (unsigned)((n_ch + 63) / 64));
  k_blend_grid_sm<<<grid, 256, 0, st>>>(tmp, n_ch, bj, bi, bw, nb, y, ys_ch, ys_t, gen);
  return hipGetLastError();
}

hipError_t launch_lattice_scan(const float *x, int64_t s_ch, int64_t s_t, const BlockGeom &g, int padlen,
                               const ScanConst &sc, const RunGeom &rg, const ChunkGeom *cg, int64_t n_chunks,
                               const double *Y0, const double *AG, double *SR, double *TP, int64_t tp_len,
                               double *TR, double *CR, const int *slot_chunk, int n_off, const RunConst *rc_off,
                               const ChunkGeom *cg_off, double *y, int64_t ys_ch, int64_t y_off, hipStream_t st,
                               const SegGeom *seg, int seg_max, double *SC, int *scan_used) {
  if (n_off < 1 || n_off > LAT_MAX_OFF || !TR || !CR || !slot_chunk) return hipErrorInvalidValue;
  const int dthr = n_chunks * g.n_ch < 40000 ? 64 : 256;
  const unsigned nb = nblk(n_chunks * g.n_ch, dthr);
  const int64_t o_defer = option(LFD_OPT_SCAN_DEFER);
  if (seg && SC && seg_max >= 1 &&
      (o_defer == 3 || (o_defer != 1 && o_defer != 2 && n_chunks * g.n_ch < 40000 && rg.n_sr >= 128 * n_chunks))) {
    if (scan_used) *scan_used = LFD_SCAN_SEGMENTED;
    const hipError_t e = launch_seg_scan(x, s_ch, s_t, g, padlen, sc, rg, cg, n_chunks, Y0, AG, SR, TP, tp_len, y,
                                         ys_ch, 1, st, TR, CR, seg, seg_max, SC);
    if (e != hipSuccess) return e;
  } else if ((scan_used ? (*scan_used = LFD_SCAN_DEFERRED) : 0), rg.n_sr >= 128 * n_chunks)
    k_chunk_scan<2, true, true, 16, 8><<<nb, dthr, 0, st>>>(x, s_ch, s_t, g, padlen, sc, cg, n_chunks, AG, SR, TP,
                                                            tp_len, y, ys_ch, 1, rg, Y0, TR, CR);
  else
    k_chunk_scan<2, true, true><<<nb, dthr, 0, st>>>(x, s_ch, s_t, g, padlen, sc, cg, n_chunks, AG, SR, TP, tp_len,
                                                     y, ys_ch, 1, rg, Y0, TR, CR);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t waves = ((g.n_ch + 63) / 64) * rg.n_sr;
  (void)ys_ch;
  k_lat_outputs<<<nblk(waves, 4), 256, 0, st>>>(g, cg_off, n_chunks, n_off, rg, slot_chunk, rc_off, Y0, SR, TR, y,
                                                y_off);
  return hipGetLastError();
}

hipError_t launch_chunk_scan(int n_sec, bool fir32, const float *x, int64_t s_ch, int64_t s_t,
                             const BlockGeom &g, int padlen, const ScanConst &sc,
                             const ChunkGeom *cg, int64_t n_chunks, const double *F, double *SF,
                             double *TP, int64_t tp_len, double *y, int64_t ys_ch, int64_t ys_t,
                             hipStream_t st) {
  (void)fir32;
  const unsigned nb = nblk(n_chunks * g.n_ch, 256);
#define LFD_SCAN(NS)                                                                         \
  k_chunk_scan<NS, false><<<nb, 256, 0, st>>>(x, s_ch, s_t, g, padlen, sc, cg, n_chunks, F, SF, \
                                               TP, tp_len, y, ys_ch, ys_t, RunGeom{}, nullptr)
  switch (n_sec) {
    case 1: LFD_SCAN(1); break;
    case 2: LFD_SCAN(2); break;
    case 3: LFD_SCAN(3); break;
    case 4: LFD_SCAN(4); break;
    default: return hipErrorInvalidValue;
  }
#undef LFD_SCAN
  return hipGetLastError();
}

hipError_t launch_fullrate_blocks(int n_sec, bool out, const float *x, int64_t s_ch, int64_t s_t,
                                  int64_t n_ch, int64_t nb, const FRConst *fc, const double *SF,
                                  const double *ST, double *F, double *y, int64_t ys_ch, int64_t ys_t,
                                  hipStream_t st, bool mb, int64_t n_mb) {
  const int64_t n_wg = n_ch * nb;
  if (n_wg < 1 || n_wg > INT32_MAX) return hipErrorInvalidValue;
#ifdef LFD_DIAG
  static int stage_old = -1;
  if (stage_old < 0) {
    stage_old = knob_flag("LFD_FR_STAGE_OLD") ? 1 : 0;
    if (stage_old) (void)hipMemcpyToSymbol(HIP_SYMBOL(g_fr_stage_old), &stage_old, sizeof(int));
    const int stagger = knob("LFD_FR_STAGGER") ? std::atoi(knob("LFD_FR_STAGGER")) : 0;
    if (stagger) (void)hipMemcpyToSymbol(HIP_SYMBOL(g_fr_stagger), &stagger, sizeof(int));
  }
#endif
#define LFD_FR(NS, OUT) \
  k_fullrate_wave<NS, OUT><<<(unsigned)n_wg, 64, 0, st>>>(x, s_ch, s_t, n_ch, nb, fc, SF, ST, F, y, ys_ch, ys_t)
#ifdef LFD_DIAG
  // (LFD_FR_ORDER: the workgroup order A/B, 0 / 1 / 2 below)
  static const int fr_ord = knob("LFD_FR_ORDER") ? std::atoi(knob("LFD_FR_ORDER")) : 2;
#else
  constexpr int fr_ord = 2;
#endif
#define LFD_FR2(NS)   \
  if (out && mb)      \
    k_fullrate_out_mb<NS><<<(unsigned)n_wg, 64, 0, st>>>(x, s_ch, n_ch, nb, n_mb, fc, SF, ST, y, ys_ch, ys_t, fr_ord); \
  else if (out)       \
    LFD_FR(NS, true); \
  else                \
    LFD_FR(NS, false)
  switch (n_sec) {
    case 1: LFD_FR2(1); break;
    case 2: LFD_FR2(2); break;
    case 3: LFD_FR2(3); break;
    case 4: LFD_FR2(4); break;
    default: return hipErrorInvalidValue;
  }
#undef LFD_FR2
#undef LFD_FR
#ifdef LFD_DIAG
  if (out && mb && knob_flag("LFD_FR_TIMES")) {
    // phase durations (us, mean over the first waves): 0-1 tile load, 1-2
    // KAZ products + transposes, 2-3 row scans, 3-4 Q / Kr products, 4-5 stage
    // + stores; and the first start -> last end of those waves
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    const size_t nw = (size_t)std::min<int64_t>(n_wg, 16384);
    std::vector<uint64_t> t(nw * 8);
    e = hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_fr_times), t.size() * sizeof(uint64_t));
    if (e != hipSuccess) return e;
    double d[5] = {0, 0, 0, 0, 0};
    uint64_t t0 = ~0ull, t1 = 0;
    for (size_t b = 0; b < nw; ++b) {
      for (int i = 0; i < 5; ++i) d[i] += 0.01 * (double)(t[b * 8 + i + 1] - t[b * 8 + i]);
      t0 = std::min(t0, t[b * 8]);
      t1 = std::max(t1, t[b * 8 + 5]);
    }
    fprintf(stderr, "k_fullrate_out_mb us/wave: load %.2f kaz %.2f scans %.2f qkr %.2f store %.2f; %zu waves span %.1f us\n",
            d[0] / nw, d[1] / nw, d[2] / nw, d[3] / nw, d[4] / nw, nw, 0.01 * (double)(t1 - t0));
  }
#endif
  return hipGetLastError();
}

hipError_t launch_fullrate_scan(int n_sec, const float *x, int64_t s_ch, int64_t s_t, int64_t n_ch,
                                int64_t n_t, int64_t nb, int padlen, const FRConst *fc, const double *F,
                                double *SF, double *ST, double *TP, double *y, int64_t ys_ch, int64_t ys_t,
                                hipStream_t st) {
  const unsigned g = nblk(n_ch, 64);
#define LFD_FRS(NS) \
  k_fullrate_scan<NS><<<g, 64, 0, st>>>(x, s_ch, s_t, n_ch, n_t, nb, padlen, fc, F, SF, ST, TP, y, ys_ch, ys_t)
  switch (n_sec) {
    case 1: LFD_FRS(1); break;
    case 2: LFD_FRS(2); break;
    case 3: LFD_FRS(3); break;
    case 4: LFD_FRS(4); break;
    default: return hipErrorInvalidValue;
  }
#undef LFD_FRS
  return hipGetLastError();
}

// dynamic LDS cap of k_fullrate_scan_seg (agg + edge windows; 160 KB per CU
// minus the static matrices and slots)
constexpr size_t FR_SEG_LDS_MAX = 148 * 1024;
hipError_t launch_fullrate_scan_seg(int n_sec, const float *x, int64_t s_ch, int64_t s_t, int64_t n_ch, int64_t n_t,
                                    int64_t M, int padlen, const FRConst *fc, const double *F2, double *SFm,
                                    double *STm, double *TP, double *y, int64_t ys_ch, int64_t ys_t,
                                    const FRSeg &sg, hipStream_t st) {
  if ((sg.cw != 16 && sg.cw != 8) || sg.G < 1 || sg.G * sg.cw > 512 || sg.Gu < 1 || sg.Gu > sg.G || sg.seglen < 1 ||
      M < 1)
    return hipErrorInvalidValue;
  const unsigned g = nblk(n_ch, sg.cw);
  size_t lds = sizeof(double) * (size_t)sg.G * sg.cw * 2 * n_sec;
  // edge windows in LDS when they fit (SciPy's padlen < n_t): the last xl
  // samples cover the tail and the samples the right pad reflects
  const int64_t nt_tail = n_t - M * FR_LB;
  int64_t xl = std::max<int64_t>(nt_tail, (int64_t)padlen + 1);
  const size_t wb = (size_t)sg.cw * (sizeof(double) * (size_t)(nt_tail + padlen) + sizeof(float) * (size_t)xl +
                                     sizeof(float) * (size_t)(padlen + 1));
  if (xl > n_t || lds + wb > FR_SEG_LDS_MAX || knob_flag("LFD_FR_TAIL_GLOBAL")) {
    xl = 0;  // (diag A/B knob: the global-memory edge walks)
  } else {
    lds += wb;
  }
  static bool attr = false;  // (dynamic LDS above 64 KB with the static part)
  if (!attr) {
    for (const void *fn : {reinterpret_cast<const void *>(&k_fullrate_scan_seg<1>),
                           reinterpret_cast<const void *>(&k_fullrate_scan_seg<2>),
                           reinterpret_cast<const void *>(&k_fullrate_scan_seg<3>),
                           reinterpret_cast<const void *>(&k_fullrate_scan_seg<4>),
                           reinterpret_cast<const void *>(&k_fullrate_scan_seg<1, 8>),
                           reinterpret_cast<const void *>(&k_fullrate_scan_seg<2, 8>),
                           reinterpret_cast<const void *>(&k_fullrate_scan_seg<3, 8>),
                           reinterpret_cast<const void *>(&k_fullrate_scan_seg<4, 8>)}) {
      const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)FR_SEG_LDS_MAX);
      if (e != hipSuccess) return e;
    }
    attr = true;
  }
#define LFD_FRSS(NS)                                                                                               \
  if (sg.cw == 8)                                                                                                  \
    k_fullrate_scan_seg<NS, 8><<<g, sg.cw * sg.G, lds, st>>>(x, s_ch, s_t, n_ch, n_t, M, padlen, fc, F2, SFm, STm, \
                                                            TP, y, ys_ch, ys_t, sg, (int)xl);                      \
  else                                                                                                             \
    k_fullrate_scan_seg<NS><<<g, sg.cw * sg.G, lds, st>>>(x, s_ch, s_t, n_ch, n_t, M, padlen, fc, F2, SFm, STm, TP,  \
                                                         y, ys_ch, ys_t, sg, (int)xl)
  switch (n_sec) {
    case 1: LFD_FRSS(1); break;
    case 2: LFD_FRSS(2); break;
    case 3: LFD_FRSS(3); break;
    case 4: LFD_FRSS(4); break;
    default: return hipErrorInvalidValue;
  }
#undef LFD_FRSS
#ifdef LFD_DIAG
  if (knob_flag("LFD_FRS_TIMES")) {
    // phase durations (us, mean over the first workgroups): 0-1 LDS windows,
    // 1-2 forward aggregates + left edge, 2-3 forward states + tail, 3-4
    // reverse aggregates, 4-5 entering T + reverse states
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    const size_t nw = (size_t)std::min<int64_t>(g, 256);
    std::vector<uint64_t> t(nw * 8);
    e = hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_frs_times), t.size() * sizeof(uint64_t));
    if (e != hipSuccess) return e;
    double d[5] = {0, 0, 0, 0, 0};
    for (size_t b = 0; b < nw; ++b)
      for (int i = 0; i < 5; ++i) d[i] += 0.01 * (double)(t[b * 8 + i + 1] - t[b * 8 + i]);
    fprintf(stderr, "k_fullrate_scan_seg us/group: windows %.2f fagg %.2f fstates+tail %.2f ragg %.2f rstates %.2f (%zu groups)\n",
            d[0] / nw, d[1] / nw, d[2] / nw, d[3] / nw, d[4] / nw, nw);
  }
#endif
  return hipGetLastError();
}

hipError_t launch_sosfiltfilt(int n_sec, const float *x, int64_t n_ch,
                              int64_t n_t, int64_t s_ch, int64_t s_t,
                              const SosCoef &c, const ZiVec &zi, int padlen,
                              double *ws, double *y, int64_t ys_ch,
                              int64_t ys_t, hipStream_t st) {
  const unsigned nb = nblk(n_ch, 256);
#define LFD_FULL(NS)                                                      \
  k_sosfiltfilt_full<NS><<<nb, 256, 0, st>>>(x, n_ch, n_t, s_ch, s_t, c, zi, \
                                             padlen, ws, y, ys_ch, ys_t)
  switch (n_sec) {
    case 1: LFD_FULL(1); break;
    case 2: LFD_FULL(2); break;
    case 3: LFD_FULL(3); break;
    case 4: LFD_FULL(4); break;
    default: return hipErrorInvalidValue;
  }
#undef LFD_FULL
  return hipGetLastError();
}

hipError_t launch_interp_linear(const double *x, int64_t n_ch, int64_t n_t,
                                int64_t s_ch, int64_t s_t, const int64_t *lo,
                                const double *w, int64_t n_out, double *y,
                                int64_t ys_ch, int64_t ys_t, hipStream_t st) {
  k_interp_linear<<<nblk(n_ch * n_out, 256), 256, 0, st>>>(
      x, n_ch, n_t, s_ch, s_t, lo, w, n_out, y, ys_ch, ys_t);
  return hipGetLastError();
}

hipError_t launch_rolling_mean(const float *x, int64_t n_ch, int64_t n_t,
                               int64_t s_ch, int64_t s_t, int64_t W, int64_t S,
                               float *y, int64_t ys_ch, int64_t ys_t,
                               hipStream_t st) {
  const int64_t n_out = (n_t + S - 1) / S;
  // workgroups of the grid-stride launches: the running-sum scan (S < W / 2)
  // keeps 8,192 (4.54 vs 4.66 ms uncapped on cfg2 at S = 1); the segment-sum
  // and direct-window kernels take up to 65,536 groups (cfg2, S = 250: one
  // unit per wave, 2.61 -> 2.45 ms; S = W: 2.16 -> 2.13 ms at 16,384 groups;
  // profiles/r04aa_ab_roll_cap.txt)
  int64_t cap = 256 * 32, cap_unit = 65536;
  if (const char *v = knob("LFD_ROLL_CAP")) cap = cap_unit = std::atoll(v) > 0 ? std::atoll(v) : INT32_MAX;  // (diag A/B; 0 = none)
  // step < window: the running-sum scan reads each sample twice (x[t] and,
  // from cache, x[t - W]) and scans every position; summing each window
  // directly reads it W/S times from L2/L1 (W/S = 4: 5.25 ms vs 3.81 ms on
  // cfg2), so the scan takes every W > 2S (A/B knob LFD_ROLL_DIRECT_MAX)
  int64_t direct_max = 2;
  if (const char *v = knob("LFD_ROLL_DIRECT_MAX")) direct_max = std::atoll(v);
  // segment prefix sums (k_rolling_seg) when g = gcd(W, S) >= 16 and the
  // prefix ring fits: no per-position running sum (A/B knob LFD_ROLL_SEGSUM=0)
  {
    int64_t ga = W, gb = S;
    while (gb) {
      const int64_t t = ga % gb;
      ga = gb;
      gb = t;
    }
    const int64_t g = ga;
    // prefix ring: the boundaries of up to ebatch + (one tile's outputs)
    // pending outputs' windows plus one tile's new boundaries (k_rolling_seg
    // emits its outputs ebatch at a time: 64, fewer when the ring would not
    // fit 1,024 entries).  Measured r05t on cfg2, W = 1000, S = 250: the
    // per-tile output pass cost 2.45 vs 2.15 ms without it
    // (profiles/r05_roll_seg_diag.txt)
    auto ring_for = [&](int64_t eb) {
      int64_t r = 16;
      while (r < W / g + (eb + RG_P / S + 1) * (S / g) + RG_P / g + 3) r *= 2;
      return r;
    };
    int ebatch = 64;
    while (ebatch > 1 && ring_for(ebatch) > 1024) ebatch /= 2;
    const int64_t ring = ring_for(ebatch);
    // (rows of any stride: 4-B aligned 16-B pieces, f4u)
    bool seg = s_t == 1 && S > 1 && S < W && g >= 16 && ring <= 1024 && n_t < ((int64_t)1 << 29) &&
               (reinterpret_cast<uintptr_t>(x) & 3) == 0;
    if (const char *v = knob("LFD_ROLL_SEGSUM")) seg = seg && std::atoi(v) != 0;
    if (seg) {
      // units: each channel cut into the fewest equal pieces that give >= 3
      // rounds of the resident waves (16 per CU) — a unit's first loads wait
      // a full memory latency, so long units stream better: cfg2 at S = 250
      // 32,768-position units (23 rounds) 2.36 ms, 65,536 2.29, 200,000 (3
      // per channel) 2.25 (profiles/r05_roll_seg_diag.txt) — and >= 4W
      // positions each (the halo re-read)
      const int64_t resident = 16 * (int64_t)cu_count();
      const int64_t pieces = std::max<int64_t>(1, (3 * resident + n_ch - 1) / n_ch);
      int64_t seg_out = std::max<int64_t>((n_out + pieces - 1) / pieces, (4 * W + S - 1) / S);
      if (const char *v = knob("LFD_ROLL_SEG")) seg_out = std::max<int64_t>(4 * W, std::atoll(v)) / S;
      seg_out = std::max<int64_t>(1, seg_out);
      const int64_t units = n_ch * ((n_out + seg_out - 1) / seg_out);
      int64_t blocks = (units + 3) / 4;
      if (blocks > cap_unit) blocks = cap_unit;
      const size_t lds = sizeof(double) * 2 * (size_t)ring * 4 + sizeof(float) * RG_P * 4;
      static bool attr = false;
      if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_rolling_seg<2>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
        if (e != hipSuccess) return e;
        attr = true;
      }
      int sdiag = 0;
      if (const char *v = knob("LFD_ROLL_SEG_DIAG")) sdiag = std::atoi(v);
      k_rolling_seg<2><<<(unsigned)blocks, 256, lds, st>>>(x, n_ch, (int)n_t, s_ch, (int)W, (int)S, (int)g, y, ys_ch,
                                                           ys_t, (int)seg_out, (int)ring - 1, ebatch, sdiag);
      return hipGetLastError();
    }
  }
  if (s_t == 1 && W <= direct_max * S) {
    // windows overlap little or not at all: each is summed directly by one wave
    const int64_t waves = n_ch * n_out;
    int64_t blocks = (waves + 3) / 4;
    if (blocks > cap_unit) blocks = cap_unit;
    const bool vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    k_rolling_tc<<<(unsigned)blocks, 256, 0, st>>>(x, n_ch, n_t, s_ch, W, S, y,
                                                   ys_ch, ys_t, vec);
  } else if (s_t == 1 && n_t < (int64_t)INT32_MAX - 1024 && W < ((int64_t)1 << 21)) {
    // overlapping windows: running sum over segments of >= max(32768, 4W)
    // positions (halo W per segment), fewer when that leaves the chip idle
    int64_t seg_pos = std::max<int64_t>(32768, 4 * W);
    if (const char *v = knob("LFD_ROLL_SEG")) seg_pos = std::max<int64_t>(4 * W, std::atoll(v));
    while (seg_pos > std::max<int64_t>(4096, 4 * W) && n_ch * ((n_t + seg_pos - 1) / seg_pos) < 16384)
      seg_pos /= 2;
    const int64_t seg_out = std::max<int64_t>(1, seg_pos / S);
    const int64_t units = n_ch * ((n_out + seg_out - 1) / seg_out);
    int64_t blocks = (units + 3) / 4;
    if (blocks > cap) blocks = cap;
    const bool vec = (reinterpret_cast<uintptr_t>(x) & 3) == 0;  // (any row stride: f4u loads)
    const bool vec_out = vec && ys_t == 1 && ys_ch % 4 == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0;
    // lanes load their 8 positions directly, outputs leave through LDS as
    // coalesced float4 stores (cfg2 at S = 1: 4.77 ms vs 5.93 with the loads
    // staged through LDS too; deeper prefetch and 4 waves per SIMD measured
    // slower: profiles/archive_r01_r03.md (r02_ab_roll_)*.txt, r05_roll_scan_ab.txt)
    // the per-step wave scan on DPP lane moves (A/B knob LFD_ROLL_DPP=0: shuffles)
    bool dpp = true;
    if (const char *v = knob("LFD_ROLL_DPP")) dpp = std::atoi(v) != 0;
    // LDS ring for x[t - W] (vector rows, W + 512 <= 4096): A/B knob LFD_ROLL_RING
    int ring = 0;
    while (ring < W + RS_P) ring = ring ? 2 * ring : 1024;
    bool use_ring = vec && ring <= 4096 && n_t < ((int64_t)1 << 29);
    if (const char *v = knob("LFD_ROLL_RING")) use_ring = use_ring && std::atoi(v) != 0;
    if (use_ring) {
      static bool attr = false;
      if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_rolling_scan_tc<true, 2, 1, 3, true>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 4 * 4096 * 4);
        if (e != hipSuccess) return e;
        attr = true;
      }
      k_rolling_scan_tc<true, 2, 1, 3, true><<<(unsigned)blocks, 256, sizeof(float) * 4 * ring, st>>>(
          x, n_ch, (int)n_t, s_ch, (int)W, (int)S, y, ys_ch, ys_t, (int)seg_out, vec_out, ring - 1, dpp);
      return hipGetLastError();
    }
#define LFD_ROLL(V, ST, PF_)                                                                                    \
  k_rolling_scan_tc<V, ST, PF_><<<(unsigned)blocks, 256, 0, st>>>(x, n_ch, (int)n_t, s_ch, (int)W, (int)S, y, ys_ch, \
                                                             ys_t, (int)seg_out, V && vec_out, 0, dpp)
    if (!vec)
      LFD_ROLL(false, 0, 1);
    else
      LFD_ROLL(true, 2, 1);
#undef LFD_ROLL
  } else {
    const int64_t seg_out = S >= W ? 64 : std::max<int64_t>(1, std::max<int64_t>(4096, 4 * W) / S);
    const int64_t units = n_ch * ((n_out + seg_out - 1) / seg_out);
    int64_t blocks = (units + 255) / 256;
    if (blocks > cap) blocks = cap;
    k_rolling_cols<<<(unsigned)blocks, 256, 0, st>>>(x, n_ch, n_t, s_ch, s_t, W, S, y, ys_ch, ys_t,
                                                    seg_out);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// k_fir_decimate — FIR decimation by q (Patch.decimate(filter_type='fir'):
// scipy.signal.decimate(x, q, ftype='fir', zero_phase=True) =
// resample_poly(x, 1, q, window=firwin(20q+1, 1/q, 'hamming')),
// scipy/signal/_signaltools.py decimate / resample_poly):
//   y[k] = sum_{i < n_taps} h[i] x[k q + delay - i],  x = 0 outside [0, n_t)
// in polyphase form: i = u q + v,  y[k] = sum_v sum_u h[u q + v] X_v[k - u]
// with X_v[n] = x[n q + delay - v].  One workgroup = one channel x `to`
// consecutive outputs; the input span is staged through LDS as the q
// polyphase rows X_v (coalesced global reads, zero outside the record), so
// the lanes' reads along a row are 2 words apart at any q (two-way bank
// sharing, not q-dependent).  A thread owns two consecutive outputs: walking u,
// each X_v value it loads feeds both (2 fp64 FMAs per LDS read); the taps
// are wave-uniform (scalar loads).  Every input sample is read from HBM
// once per tile (+ the (U - 1) q halo).
// ---------------------------------------------------------------------------
constexpr int FD_THREADS = 256;
constexpr int FD_LDS = 64 * 1024;
__global__ __launch_bounds__(FD_THREADS) void k_fir_decimate(const float *__restrict__ x, int64_t n_t, int64_t s_ch,
                                                             int64_t s_t, const double *__restrict__ h,
                                                             int n_taps, int q, int64_t delay, int64_t n_out,
                                                             int tiles, int to, int U, int rowlen,
                                                             double *__restrict__ y, int64_t ys_ch,
                                                             int64_t ys_t) {
  extern __shared__ float fd_x[];  // [v][rowlen]: X_v[k0 - U + 1 + n]
  const int64_t ch = blockIdx.x / tiles;
  const int64_t k0 = (int64_t)(blockIdx.x % tiles) * to;
  const int nrow = to + U;  // X_v values a tile reads (+1: the odd thread's second output)
  const int64_t g0 = (k0 - U + 1) * q + delay - (q - 1);  // sample of m = 0
  const float *xr = x + ch * s_ch;
  // (span <= 16384: n = m / q by a float reciprocal, corrected to exact)
  const int span = nrow * q;
  const float rq = 1.0f / (float)q;
  // 8 loads per thread in flight before their LDS writes (a tile is up to
  // 16 K samples: enough bytes in flight per CU to stream)
  constexpr int FU = 8;
  for (int m0 = threadIdx.x; m0 < span; m0 += FU * blockDim.x) {
    float xv8[FU];
#pragma unroll
    for (int e = 0; e < FU; ++e) {
      const int m = m0 + e * blockDim.x;
      const int64_t t = g0 + m;
      xv8[e] = (m < span && t >= 0 && t < n_t) ? xr[t * s_t] : 0.0f;
    }
#pragma unroll
    for (int e = 0; e < FU; ++e) {
      const int m = m0 + e * blockDim.x;
      if (m >= span) break;
      int n = (int)((float)m * rq);
      n -= n * q > m ? 1 : 0;
      n += (n + 1) * q <= m ? 1 : 0;
      const int v = q - 1 - (m - n * q);
      fd_x[v * rowlen + n] = xv8[e];
    }
  }
  __syncthreads();
  for (int base = 2 * threadIdx.x; base < to; base += 2 * blockDim.x) {  // outputs k0 + base, + 1
  double a0 = 0.0, a1 = 0.0;
  for (int v = 0; v < q; ++v) {
    const float *xv = fd_x + v * rowlen + base;
    // output r uses X_v[base + r + U - 1 - u]: walking s = U - 1 - u upward,
    // x_s feeds output 0 and x_{s+1} output 1
    double xs = (double)xv[0];
#pragma unroll 4
    for (int s2 = 0; s2 < U; ++s2) {
      const int u = U - 1 - s2;
      const double xn = (double)xv[s2 + 1];
      if (u * q + v < n_taps) {
        const double hv = h[u * q + v];
        a0 = fma(hv, xs, a0);
        a1 = fma(hv, xn, a1);
      }
      xs = xn;
    }
  }
  const int64_t k = k0 + base;
  if (k < n_out) y[ch * ys_ch + k * ys_t] = a0;
  if (base + 1 < to && k + 1 < n_out) y[ch * ys_ch + (k + 1) * ys_t] = a1;
  }
}

// ---------------------------------------------------------------------------
// k_fir_decimate_mfma — the same FIR decimation on the fp64 matrix cores
// (v_mfma_f64_4x4x4_4b: 4 x 4 x 4 per block, 4 blocks per instruction).
// Polyphase: y[o] = sum_v sum_u h_v[u] X_v[o - u], h_v[u] = h[u q + v].  For
// 4 consecutive outputs o = 4G + i and 4 consecutive polyphase indices
// n = 4(G - d) + k the taps form a 4 x 4 Toeplitz piece A_{v,d}[i][k] =
// h_v[4d + i - k] that depends on (v, d) only, so
//   Y[G] = sum_v sum_{d < D_v} A_{v,d} X_v[4(G - d) .. 4(G - d) + 3]
// with D_v = ceil((U_v - 1)/4) + 1 (U_v = taps of phase v).  MFMA lane
// layout (tools/check_mfma4x4.hip): A[i][k] at lane 16k + 4b + i, B[k][j] at
// 16k + 4b + j, D[i][j] at 16i + 4b + j.  Blocks b = 4 consecutive output
// groups, j = 4 channels: one MFMA = 16 outputs x 4 channels x 4 indices;
// a wave owns 64 consecutive outputs (4 accumulators) of 4 channels.
// A workgroup (4 waves) stages its 4 channels' span of input in LDS by
// LDS-DMA (global_load_lds_dwordx4, wave w = channel w, 1 KB per
// instruction, no VGPRs, no ds_write): the raw sample image, from which a B
// read takes polyphase row v, index n as sample n q + q - 1 - v (a stride-q
// ds_read_b32; the channels' image bases are offset so one B read — 4 rows x
// 16 consecutive indices — hits distinct banks, fdd_bank_offsets).  Tiles
// whose span leaves the record, or rows that are not 16-B aligned, stage
// through registers into the same image (zeros outside the record).  The A
// pieces sit in LDS ([v][d][16 lanes]).  Each B value (one ds_read_b32 +
// cvt) feeds every (tile, d) pair with the same index offset.  Slots of the Toeplitz pieces outside a row's taps
// multiply neighbouring samples by 0, so a non-finite sample there would
// poison a finite output: every non-finite result is recomputed by the
// direct sum (SciPy's value: NaN / +-inf exactly where 0 * NaN, inf * h
// arise), which also keeps SciPy's NaN footprint of the zero pre-pad taps.
// ---------------------------------------------------------------------------
// Compile-time geometry per decimation factor Q: DM = 6 Toeplitz steps cover
// taps u <= 20 of every phase and u = 21 for rows i >= 1; the one tap
// h[21 Q] (phase 0, u = 21: decimate's firwin(20Q+1) behind its Q pre-pad
// zeros has n_taps = 21Q + 1) of row-0 outputs is added in the epilogue.
constexpr int FDM_DM = 6;
constexpr int FDM_NO = 256;                          // outputs per tile: 4 waves x 64
constexpr int FDM_NN = FDM_NO + 4 * (FDM_DM - 1) + 1;  // polyphase indices per tile (+1: the u = 21 tap)
// Staging (round 6): the LDS-DMA image replaced register staging into the
// polyphase rows (16-B global loads, then per-element ds_write at computed
// row / index): 1.540 -> 1.497 ms at q = 10, 1.745 -> 1.676 at q = 5 on
// 2,000 x 600,000, bit-identical (profiles/r06_fir_dma_ab.txt).  Single
// buffer: fill, barrier, products, barrier; 3 workgroups per CU (53 KB of
// LDS each) overlap one group's fill with the others' products (a
// double-buffered image at 1 workgroup per CU measured slower,
// profiles/archive_r01_r03.md (r03_ab_fir.txt)).  A scheduling barrier
// closes every phase: without it the compiler hoisted the next phase's
// f32 -> f64 conversions — and so the wait for that phase's LDS reads —
// into this phase's first MFMAs (1.648 -> 1.565 ms, profiles/r05_fir_sched.txt).
// cj: the channel images' bank offsets (launcher).
template <int Q>
constexpr int fdd_nrd() { return (FDM_NN * Q + 3 + 255) / 256; }
template <int Q>
constexpr int fdd_raw() { return 256 * fdd_nrd<Q>() + 32; }
template <int Q>
constexpr size_t fdd_lds_bytes() {
  return sizeof(double) * Q * FDM_DM * 16 + sizeof(float) * 4 * fdd_raw<Q>();
}
template <int Q>
__global__ __launch_bounds__(256, 3) void k_fir_decimate_mfma(const float *__restrict__ x, int64_t n_ch, int64_t n_t,
                                                          int64_t s_ch, const double *__restrict__ h, int n_taps,
                                                          int64_t delay, int64_t n_out, int64_t tiles_o, int strip,
                                                          double *__restrict__ y, int64_t ys_ch, int64_t ys_t,
                                                          int4 cj, int dma_ok) {
  constexpr int DM = FDM_DM, NO = FDM_NO, NRD = fdd_nrd<Q>(), RAW = fdd_raw<Q>();
  extern __shared__ double fdm_lds[];
  double *At = fdm_lds;                                          // [v][d][16]
  float *Xr = reinterpret_cast<float *>(fdm_lds + Q * DM * 16);  // [j][RAW] raw sample images
  const int64_t n_strips = (tiles_o + strip - 1) / strip;
  int64_t bid = blockIdx.x;
  const int64_t nb = (int64_t)gridDim.x;
  if ((nb & 7) == 0) bid = (bid & 7) * (nb >> 3) + (bid >> 3);
  const int64_t cg = bid / n_strips;
  const int64_t t_begin = (bid % n_strips) * strip;
  const int64_t t_end = t_begin + strip < tiles_o ? t_begin + strip : tiles_o;
  auto cof = [&](int j) { return j == 0 ? cj.x : (j == 1 ? cj.y : (j == 2 ? cj.z : cj.w)); };
  for (int e = threadIdx.x; e < Q * DM * 16; e += blockDim.x) {
    const int l16 = e & 15, vd = e >> 4;
    const int v = vd / DM, d = vd - v * DM;
    const int kk = l16 >> 2, ii = l16 & 3;
    const int u = 4 * d + ii - kk;
    const int64_t ti = (int64_t)u * Q + v;
    At[e] = (u >= 0 && ti < n_taps) ? h[ti] : 0.0;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t ch_ld = cg * 4 + w;
  const bool live = ch_ld < n_ch;
  const float *xr_ld = x + (live ? ch_ld : 0) * s_ch;
  float *img_ld = Xr + w * RAW + cof(w);
  // the tile's image: samples s0a .. s0a + 256 NRD of channel w (s0a = s0
  // rounded down to 16 B; the reads add sh = s0 - s0a)
  auto fill = [&](int64_t Ot) {
    const int64_t s0 = (Ot - 4 * (DM - 1) - 1) * Q + delay - (Q - 1);
    const int64_t s0a = s0 & ~(int64_t)3;
    if (!live) return;
    if (dma_ok && s0a >= 0 && s0a + 256 * NRD <= n_t) {
      const float *g = xr_ld + s0a + 4 * lane;
#pragma unroll
      for (int r = 0; r < NRD; ++r)
        __builtin_amdgcn_global_load_lds(g + 256 * r, img_ld + 256 * r, 16, 0, 0);
    } else {
#pragma unroll
      for (int r = 0; r < NRD; ++r)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t t = s0a + 256 * r + 4 * lane + e;
          const int64_t tc = t < 0 ? 0 : (t >= n_t ? n_t - 1 : t);
          const float v = xr_ld[tc];
          img_ld[256 * r + 4 * lane + e] = (t >= 0 && t < n_t) ? v : 0.0f;
        }
    }
  };
  const int jl = lane & 3;
  const int lane_n = 4 * ((lane >> 2) & 3) + (lane >> 4);
  const int lane_a = 4 * (lane >> 4) + (lane & 3);
  const int64_t ch = cg * 4 + jl;
  const int io = lane >> 4, bo = (lane >> 2) & 3;
  const float *xbase = Xr + jl * RAW + cof(jl);
  const double h21 = (io == 0 && 21 * Q < n_taps) ? h[21 * Q] : 0.0;
  for (int64_t tt = t_begin; tt < t_end; ++tt) {
    const int64_t O = tt * NO;
    fill(O);
    __syncthreads();  // the image has landed (the barrier waits for the DMA)
    const int sh = (int)(((O - 4 * (DM - 1) - 1) * Q + delay - (Q - 1)) & 3);
    // row v, index n of the polyphase rows = image sample n Q + Q - 1 - v
    const float *xb = xbase + sh + (64 * w + lane_n + 1) * Q + Q - 1;
    const float *x21 = xbase + sh + (64 * w + 4 * bo) * Q + Q - 1;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    {
      constexpr int NB = DM + 12;
      double an[DM];
      float bn[NB];
#pragma unroll
      for (int d = 0; d < DM; ++d) an[d] = At[d * 16 + lane_a];
#pragma unroll
      for (int si = 0; si < NB; ++si) bn[si] = xb[4 * si * Q];
#pragma unroll
      for (int v = 0; v < Q; ++v) {
        double ac[DM], bd[NB];
#pragma unroll
        for (int d = 0; d < DM; ++d) ac[d] = an[d];
#pragma unroll
        for (int si = 0; si < NB; ++si) bd[si] = (double)bn[si];
        if (v + 1 < Q) {
#pragma unroll
          for (int d = 0; d < DM; ++d) an[d] = At[((v + 1) * DM + d) * 16 + lane_a];
#pragma unroll
          for (int si = 0; si < NB; ++si) bn[si] = xb[4 * si * Q - (v + 1)];
        }
#pragma unroll
        for (int d = DM - 1; d >= 0; --d) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
            acc[t] = __builtin_amdgcn_mfma_f64_4x4x4f64(ac[d], bd[4 * t + DM - 1 - d], acc[t], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int64_t o = O + 64 * w + 16 * t + 4 * bo + io;
      if (ch >= n_ch || o >= n_out) continue;
      double val = fma(h21, (double)x21[16 * t * Q], acc[t]);
      if (!isfinite(val)) {
        const float *xr = x + ch * s_ch;
        double a2 = 0.0;
        for (int i = 0; i < n_taps; ++i) {
          const int64_t ts = o * Q + delay - i;
          if (ts >= 0 && ts < n_t) a2 = fma(h[i], (double)xr[ts], a2);
        }
        val = a2;
      }
      y[ch * ys_ch + o * ys_t] = val;
    }
    __syncthreads();  // the image's reads are done before the next fill
  }
}

// the raw images' bank offsets: the fewest conflicts of one B read (lanes
// 0-31: 4 channel rows x indices 4a + b, stride q floats; ds_read_b32 banks
// (a / 4) mod 32), brute force per q
static int4 fdd_bank_offsets(int q, int raw) {
  int best = 1 << 30;
  int4 bo{0, 0, 0, 0};
  for (int c1 = 0; c1 < 32; ++c1)
    for (int c2 = 0; c2 < 32; ++c2)
      for (int c3 = 0; c3 < 32; ++c3) {
        const int c[4] = {0, c1, c2, c3};
        int cnt[32] = {0};
        for (int l = 0; l < 32; ++l) {
          const int j = l & 3, n = 4 * ((l >> 2) & 3) + (l >> 4);
          ++cnt[(((j * raw + c[j] + n * q) % 32) + 32) % 32];
        }
        int worst = 0;
        for (int b = 0; b < 32; ++b) worst = std::max(worst, cnt[b]);
        if (worst < best) {
          best = worst;
          bo = int4{0, c1, c2, c3};
          if (best == 1) return bo;
        }
      }
  return bo;
}

hipError_t launch_fir_decimate(const float *x, int64_t n_ch, int64_t n_t, int64_t s_ch, int64_t s_t,
                               const double *h, int n_taps, int64_t q, int64_t delay, double *y, int64_t ys_ch,
                               int64_t ys_t, hipStream_t st, int *kernel_used) {
  const int64_t n_out = (n_t + q - 1) / q;
  if (n_taps < 1 || q < 1 || q > (1 << 20) || n_out < 1) return hipErrorInvalidValue;
  const int U = (int)((n_taps + q - 1) / q);  // taps per polyphase branch
  // matrix-core path (time-contiguous rows, q in {4, 5, 6, 8, 10}, phase 0
  // at most 22 taps, the others 21: n_taps <= 21 q + 1)
  if (s_t == 1 && n_taps <= 21 * q + 1 && !option(LFD_OPT_FIR_VALU)) {
    const int64_t tiles_o = (n_out + FDM_NO - 1) / FDM_NO;
    int strip = 8;
    if (const char *sv = knob("LFD_FIR_STRIP")) strip = std::max(1, std::atoi(sv));
    if (strip > tiles_o) strip = (int)tiles_o;
    const int64_t grid = (n_ch + 3) / 4 * ((tiles_o + strip - 1) / strip);
    bool launched = false;
    hipError_t e = hipSuccess;
    // LDS-DMA needs 16-B aligned rows (else every tile stages through registers)
    const int dma_ok = (reinterpret_cast<uintptr_t>(x) & 15) == 0 && s_ch % 4 == 0;
#define LFD_FDM(QV)                                                                                      \
  case QV: {                                                                                             \
    static bool attr = false;                                                                            \
    static int4 cj{};                                                                                    \
    if (!attr) {                                                                                         \
      e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_fir_decimate_mfma<QV>),                  \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)fdd_lds_bytes<QV>());     \
      if (e != hipSuccess) return e;                                                                     \
      cj = fdd_bank_offsets(QV, fdd_raw<QV>());                                                          \
      attr = true;                                                                                       \
    }                                                                                                    \
    k_fir_decimate_mfma<QV><<<(unsigned)grid, 256, fdd_lds_bytes<QV>(), st>>>(                           \
        x, n_ch, n_t, s_ch, h, n_taps, delay, n_out, tiles_o, strip, y, ys_ch, ys_t, cj, dma_ok);        \
    launched = true;                                                                                     \
    break;                                                                                               \
  }
    if (grid <= (int64_t)INT32_MAX) {
      switch (q) {
        LFD_FDM(4)
        LFD_FDM(5)
        LFD_FDM(6)
        LFD_FDM(8)
        LFD_FDM(10)
        default: break;
      }
    }
#undef LFD_FDM
    if (launched) {
      if (kernel_used) *kernel_used = 1;
      return hipGetLastError();
    }
  }
  // outputs per tile: q rows of (to + U) staged floats (odd row length) in LDS
  const int64_t cap = std::min<int64_t>(16 * 1024 / q, FD_LDS / 4 / q) - U - 2;  // span <= 16 K samples
  if (cap < 1) return hipErrorInvalidValue;
  const int to = (int)std::min<int64_t>({(int64_t)2 * FD_THREADS, cap, n_out});
  const int rowlen = (to + U) | 1;
  const int64_t tiles = (n_out + to - 1) / to;
  if (n_ch * tiles > (int64_t)INT32_MAX) return hipErrorInvalidValue;
  const size_t lds_v = sizeof(float) * (size_t)q * rowlen;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_fir_decimate),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, FD_LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  k_fir_decimate<<<(unsigned)(n_ch * tiles), FD_THREADS, lds_v, st>>>(x, n_t, s_ch, s_t, h, n_taps, (int)q, delay,
                                                                     n_out, (int)tiles, to, U, rowlen, y, ys_ch,
                                                                     ys_t);
  if (kernel_used) *kernel_used = 0;
  return hipGetLastError();
}

// Lattice-plan blend (lfd_capi.cpp plan_create_composite): linear interp1d
// between the two lattice phases' outputs y[lo] and y[lo + 1] of every grid
// point; one thread per (channel, point), points fastest.
// gen.dts > 0: the weights come from the grid's own integer time arithmetic
// instead of bw: point j sits rel = gen.rel0 + j gen.step ns after sample 0,
// w = (rel - floor(rel / dts) dts) / dts — the host's formula (lfd_stream.cpp
// run_chunks), so a stream's lattice plan serves every push whose grid has
// the same lattice structure, whatever its fractions.
__global__ __launch_bounds__(256) void k_blend_grid(const double *__restrict__ tmp, int64_t T, int64_t n_ch,
                                                    const int64_t *__restrict__ bj, const int64_t *__restrict__ bi,
                                                    const double *__restrict__ bw, int64_t nb, double *__restrict__ y,
                                                    int64_t ys_ch, int64_t ys_t, GridGen gen) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= nb * n_ch) return;
  const int64_t ch = idx / nb, i = idx - ch * nb;
  const double *row = tmp + ch * T;
  const int64_t ia = bi[2 * i], ib = bi[2 * i + 1];
  double v = row[ia];
  if (ib >= 0) {
    double wv;
    if (gen.dts > 0) {
      const int64_t rel = gen.rel0 + bj[i] * gen.step;
      int64_t lo = rel / gen.dts;
      if (rel % gen.dts != 0 && rel < 0) --lo;
      wv = (double)(rel - lo * gen.dts) / (double)gen.dts;
    } else {
      wv = bw[i];
    }
    v = fma(wv, row[ib] - v, v);
  }
  y[ch * ys_ch + bj[i] * ys_t] = v;
}

hipError_t launch_blend_grid(const double *tmp, int64_t T, int64_t n_ch, const int64_t *bj, const int64_t *bi,
                             const double *bw, int64_t nb, double *y, int64_t ys_ch, int64_t ys_t, hipStream_t st,
                             const GridGen &gen) {
  if (nb <= 0 || n_ch <= 0) return hipSuccess;
  k_blend_grid<<<nblk(nb * n_ch, 256), 256, 0, st>>>(tmp, T, n_ch, bj, bi, bw, nb, y, ys_ch, ys_t, gen);
  return hipGetLastError();
}

// Time-major -> channel-major transpose for the stream arena
// (host (time, distance) rows, as real DAS files store them,
// low_pass_dascore.ipynb:222 data[:, ch]).  64x64 tiles through LDS (one
// padding column against bank conflicts); both sides coalesced.
__global__ __launch_bounds__(256) void k_transpose_tc(const float *__restrict__ src, int64_t n_rows,
                                                      int64_t n_cols, int64_t sp,
                                                      float *__restrict__ dst, int64_t dp) {
  __shared__ float tile[64][65];
  const int64_t c0 = (int64_t)blockIdx.x * 64, r0 = (int64_t)blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    if (r < n_rows && c < n_cols) tile[i][tx] = src[r * sp + c];
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, r = r0 + tx;
    if (r < n_rows && c < n_cols) dst[c * dp + r] = tile[tx][i];
  }
}

hipError_t launch_transpose(const float *src, int64_t n_rows, int64_t n_cols, int64_t sp, float *dst,
                            int64_t dp, hipStream_t st) {
  const int64_t slab = (int64_t)65535 * 64;  // grid.y limit
  for (int64_t r = 0; r < n_rows; r += slab) {
    const int64_t nr = n_rows - r < slab ? n_rows - r : slab;
    dim3 grid((unsigned)((n_cols + 63) / 64), (unsigned)((nr + 63) / 64));
    k_transpose_tc<<<grid, 256, 0, st>>>(src + r * sp, nr, n_cols, sp, dst + r, dp);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// ---------------------------------------------------------------------------
// Notebook post-processing of the decimated output (low_pass_dascore.ipynb
// cells 14-22): demean over a channel range + strain-rate scale, and
// scipy.ndimage.median_filter (mode 'reflect', origin 0, rank = n // 2).
// ---------------------------------------------------------------------------

// One wave per time row: mean over channels [c0, c1) (float64 sum, lane
// strided then a wave reduction), then y = (x - mean) * scale over the row.
__global__ __launch_bounds__(256) void k_demean_scale(const double *__restrict__ x, int64_t n_rows,
                                                      int64_t n_cols, int64_t s_r, int64_t s_c, int64_t c0,
                                                      int64_t c1, double scale, double *__restrict__ y,
                                                      int64_t ys_r, int64_t ys_c) {
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const double *xr = x + row * s_r;
  double acc = 0.0;
  for (int64_t c = c0 + lane; c < c1; c += 64) acc += xr[c * s_c];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  const double mean = acc / (double)(c1 - c0);
  double *yr = y + row * ys_r;
  for (int64_t c = lane; c < n_cols; c += 64) yr[c * ys_c] = (xr[c * s_c] - mean) * scale;
}

__device__ __forceinline__ int64_t reflect_idx(int64_t i, int64_t n) {
  // scipy.ndimage 'reflect' (half-sample symmetric, period 2n): d c b a | a b c d | d c b a
  if (n == 1) return 0;
  const int64_t p = 2 * n;
  i %= p;
  if (i < 0) i += p;
  return i < n ? i : p - 1 - i;
}

constexpr int MED_T = 16;  // output tile edge

// 16x16 outputs per workgroup; the (16+k0-1) x (16+k1-1) input tile (reflect
// padded) is staged in LDS; each output selects the rank-th smallest of its
// k0*k1 window by counting (exact: the result is one of the inputs).
__global__ __launch_bounds__(256) void k_median2d(const double *__restrict__ x, int64_t n0, int64_t n1,
                                                  int64_t s0, int64_t s1, int k0, int k1,
                                                  double *__restrict__ y, int64_t ys0, int64_t ys1) {
  extern __shared__ double tile[];
  const int T1 = MED_T + k1 - 1, T0 = MED_T + k0 - 1;
  const int64_t b0 = (int64_t)blockIdx.y * MED_T - k0 / 2, b1 = (int64_t)blockIdx.x * MED_T - k1 / 2;
  for (int idx = threadIdx.x; idx < T0 * T1; idx += blockDim.x) {
    const int r = idx / T1, c = idx % T1;
    tile[idx] = x[reflect_idx(b0 + r, n0) * s0 + reflect_idx(b1 + c, n1) * s1];
  }
  __syncthreads();
  const int tx = threadIdx.x % MED_T, ty = threadIdx.x / MED_T;
  const int64_t i = (int64_t)blockIdx.y * MED_T + ty, j = (int64_t)blockIdx.x * MED_T + tx;
  if (i >= n0 || j >= n1) return;
  const int n = k0 * k1, rank = n / 2;
  const double *w = tile + ty * T1 + tx;
  double res = w[0];
  for (int a = 0; a < n; ++a) {
    const double v = w[(a / k1) * T1 + a % k1];
    int lt = 0, eq = 0;
    for (int b = 0; b < n; ++b) {
      const double u = w[(b / k1) * T1 + b % k1];
      lt += u < v;
      eq += u == v;
    }
    if (lt <= rank && rank < lt + eq) {
      res = v;
      break;
    }
  }
  y[i * ys0 + j * ys1] = res;
}

hipError_t launch_demean_scale(const double *x, int64_t n_rows, int64_t n_cols, int64_t s_r, int64_t s_c,
                               int64_t c0, int64_t c1, double scale, double *y, int64_t ys_r, int64_t ys_c,
                               hipStream_t st) {
  if (n_rows <= 0) return hipSuccess;
  k_demean_scale<<<nblk(n_rows, 4), 256, 0, st>>>(x, n_rows, n_cols, s_r, s_c, c0, c1, scale, y, ys_r, ys_c);
  return hipGetLastError();
}

hipError_t launch_median2d(const double *x, int64_t n0, int64_t n1, int64_t s0, int64_t s1, int k0, int k1,
                           double *y, int64_t ys0, int64_t ys1, hipStream_t st) {
  if (n0 <= 0 || n1 <= 0) return hipSuccess;
  const size_t lds = sizeof(double) * (size_t)(MED_T + k0 - 1) * (size_t)(MED_T + k1 - 1);
  if (lds > 64 * 1024 || (n0 + MED_T - 1) / MED_T > 65535) return hipErrorInvalidValue;
  dim3 grid((unsigned)((n1 + MED_T - 1) / MED_T), (unsigned)((n0 + MED_T - 1) / MED_T));
  k_median2d<<<grid, 256, lds, st>>>(x, n0, n1, s0, s1, k0, k1, y, ys0, ys1);
  return hipGetLastError();
}

}  // namespace lfd
