// Internal interface between the C-ABI/plan code (lfd_capi.cpp) and the
// gfx950 kernels (lfd_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace lfd {

constexpr int MAX_SEC = 4;            // up to 8th-order cascades
constexpr int MAX_N = 2 * MAX_SEC;    // state dimension (TDF-II, 2 per section)

// Transposed-direct-form-II cascade, a0 normalised to 1 (SciPy's sos rows,
// scipy/signal/_signaltools.py:4706 `_sosfilt`).
struct SosCoef {
  double b0[MAX_SEC], b1[MAX_SEC], b2[MAX_SEC], a1[MAX_SEC], a2[MAX_SEC];
};

// Constants of the block-functional kernel (k_block_functionals).  One
// "block" is L consecutive samples of one channel; the kernel runs the
// forward recurrence from zero state and, in the same sweep, the reverse
// recurrence's zero-state exit state via the inverse-time accumulator
//     u <- A^{-1} u + B y_f[m]          (u_L = sum_m A^{-(L-1-m)} B y_f[m])
// so the block is read once and nothing per-sample is stored.
struct BlockConst {
  SosCoef f;
  double ia2[MAX_SEC], ra[MAX_SEC];        // A_i^{-1} = [[0, -ia2], [1, -ra]]
  double beta0[MAX_SEC], beta1[MAX_SEC];   // section input vectors
  double Bv[MAX_N];                        // cascade input vector B
  double T[MAX_N * MAX_N];                 // A^{L-1}: u -> reverse exit state
  double cp[MAX_N];                        // C A^{L-2}
  double d0;                               // D - C A^{-1} B
};

// Constants of the per-chunk scan kernel (k_chunk_scan).
struct ScanConst {
  SosCoef f;
  double zi[MAX_N];                        // sosfilt_zi(sos) (flattened)
  double Phi[MAX_N * MAX_N];               // A^L
  double M[MAX_N * MAX_N];                 // reverse exit-state response to s_f
  double G0[MAX_N];                        // output(offset 0) response to s_f
  double H0[MAX_N];                        // output(offset 0) response to r(b)
};

struct ZiVec {
  double v[MAX_N];
};

// Per-chunk geometry used by the scan kernel (device copy of the plan).
struct ChunkGeom {
  int64_t s0, s1;        // inclusive sample range
  int64_t kb, ke;        // full blocks [kb, ke) inside the chunk
  int64_t head_end;      // first sample of block kb  (== s0 when no head)
  int64_t tail_begin;    // first sample after block ke-1
  int64_t kout0, kout1;  // blocks whose offset-0 sample is an output
  int64_t jout0;         // grid index of block kout0's output
  int64_t sf_off;        // offset (in blocks) of this chunk in the s_f scratch
  int64_t head_out_pos, head_out_j;  // output inside the head (j < 0: none)
  int64_t tail_out_pos, tail_out_j;  // output inside the tail (j < 0: none)
};

struct BlockGeom {
  int64_t n_ch, nb, base;  // blocks k in [0, nb) start at sample base + k*L
  int L;
  int nF;                  // functionals per block (2n+1)
};

// Launchers (lfd_kernels.hip).  All return hipError_t of the launch.
hipError_t launch_block_functionals(int n_sec, const float *x, int64_t s_ch,
                                    int64_t s_t, const BlockGeom &g,
                                    const BlockConst &kc, double *F,
                                    hipStream_t st);
hipError_t launch_chunk_scan(int n_sec, const float *x, int64_t s_ch,
                             int64_t s_t, const BlockGeom &g, int padlen,
                             const ScanConst &sc, const ChunkGeom *cg_dev,
                             int64_t n_chunks, const double *F, double *SF,
                             double *TP, int64_t tp_len, float *y,
                             int64_t ys_ch, int64_t ys_t, hipStream_t st);
hipError_t launch_sosfiltfilt(int n_sec, const float *x, int64_t n_ch,
                              int64_t n_t, int64_t s_ch, int64_t s_t,
                              const SosCoef &c, const ZiVec &zi,
                              int padlen, double *ws, double *y, int64_t ys_ch,
                              int64_t ys_t, hipStream_t st);
hipError_t launch_interp_linear(const double *x, int64_t n_ch, int64_t n_t,
                                int64_t s_ch, int64_t s_t, const int64_t *lo,
                                const double *w, int64_t n_out, float *y,
                                int64_t ys_ch, int64_t ys_t, hipStream_t st);
hipError_t launch_rolling_mean(const float *x, int64_t n_ch, int64_t n_t,
                               int64_t s_ch, int64_t s_t, int64_t W, int64_t S,
                               float *y, int64_t ys_ch, int64_t ys_t,
                               hipStream_t st);

}  // namespace lfd
