// Internal interface between the C-ABI/plan code (lfd_capi.cpp) and the
// gfx950 kernels (lfd_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <string>

struct lfd_lowpass_plan;  // include/lfdas.h

namespace lfd {

// Sets the calling thread's lfd_last_error() message; returns `code`.
int fail(int code, const std::string &m);
// lfd_set_timing() state (HIP-event timing of executes / pushes).
bool timing_enabled();

// lfd_set_option() value of LFD_OPT_* `id` (0 = the library's choice).  In
// the diagnostic build an unset option also reads its A/B environment name
// (LFD_NO_RUNS, LFD_K1_REC, ...), so the round-1..3 recipes under tools/ run
// unchanged against liblfdas_diag.so.
int64_t option(int id);

// Tuning / diagnostic A/B knobs.  The production liblfdas.so never reads the
// environment: knob() is nullptr there and every launcher takes its measured
// default.  Only the diagnostic build (-DLFD_DIAG -> liblfdas_diag.so,
// loaded by tools/ through LFDAS_LIB) reads them, and only there are the
// "timing only, results invalid" kernel modes and the measured-and-rejected
// variants compiled at all.
#ifdef LFD_DIAG
inline const char *knob(const char *name) { return std::getenv(name); }
#else
inline const char *knob(const char *) { return nullptr; }
#endif
inline bool knob_flag(const char *name) {
  const char *v = knob(name);
  return v && v[0] && v[0] != '0';
}

constexpr int MAX_SEC = 4;            // up to 8th-order cascades
constexpr int MAX_N = 2 * MAX_SEC;    // state dimension (TDF-II, 2 per section)

// Transposed-direct-form-II cascade, a0 normalised to 1 (SciPy's sos rows,
// scipy/signal/_signaltools.py:4706 `_sosfilt`) — used by the full-rate path.
struct SosCoef {
  double b0[MAX_SEC], b1[MAX_SEC], b2[MAX_SEC], a1[MAX_SEC], a2[MAX_SEC];
};

constexpr int MAX_J = 2 * MAX_SEC;    // FIR taps - 1 of the factored numerator

// Realization "R" of the same cascade used by the decimating path:
//   w[n]   = x[n] + sum_{j=1..J} c[j] x[n-j]           (numerator / N0, FIR)
//   v_s[n] = v_{s-1}[n] - a1_s v_s[n-1] - a2_s v_s[n-2] (all-pole sections)
//   y_f[n] = G v_last[n],  G = N0 = prod_s b0_s          (forward output)
// and the reverse pass in the mirrored form on q (backward in time) with the
// FIR applied on its output: y[m] = G sum_j c[j] q_last[m+j].
// Forward state S = (v_s[n-1], v_s[n-2]) per section; reverse state
// T(m) = (q_s[m], q_s[m+1]) per section (state after processing sample m).
// Same filter as SciPy's TDF-II in exact arithmetic; the loop-carried chain
// is one FMA per section and the FIR runs in float32 for non-negative taps.
struct RCoef {
  double na1[MAX_SEC], na2[MAX_SEC];   // -a1, -a2
  double nia2[MAX_SEC], nra[MAX_SEC];  // -1/a2, -a1/a2 (inverse accumulator)
  double dcg[MAX_SEC];                 // 1/(1+a1+a2): steady-state gains
  double c64[MAX_J + 1];               // FIR taps (c[0] = 1)
  float c32[MAX_J + 1];
  double G, csum;                      // N0, sum_j c[j]
};

// Constants of the block-functional kernel (k_block_functionals*).  One
// block = L consecutive samples of one channel; the kernel runs the forward
// recurrence from zero all-pole state (true FIR history) and, in the same
// sweep, the reverse pass's zero-state exit state through the inverse-time
// accumulator  u <- A_r^{-1} u + B_r v_last[m]  (unscaled; G folded below).
// The "output functional" p of a block is the zero-phase output at the
// block's grid point lo + w: (1 - w) y[offset 0] + w y[offset 1] (linear
// interp1d between the two samples, scipy/interpolate/_interpolate.py:457-484;
// w = 0 on sample-aligned grids).  Every constant below that names p0 / G0 /
// H0 is that blend.
struct BlockConst {
  RCoef r;
  double T[MAX_N * MAX_N];   // G A_r^{L-1}: u -> e_r0
  double cp[MAX_N];          // p0 = cp.u + dp.y0[0..J]  (output functional)
  double dp[MAX_J + 1];
};

// Constants of the per-chunk scan kernel (k_chunk_scan).
struct ScanConst {
  RCoef r;
  double PhiF[MAX_N * MAX_N];  // forward all-pole state over one block
  double PhiR[MAX_N * MAX_N];  // reverse state over one block
  double M[MAX_N * MAX_N];     // reverse exit state response to S_f
  double G0[MAX_N];            // output(offset 0) response to S_f
  double H0[MAX_N];            // output(offset 0) response to T entering
  double Kc[(2 * MAX_N + 1) * MAX_J];  // functionals' response to w[0..J-1]
  double ow;                   // weight of the offset-1 sample in an output (grid w)
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
  int64_t kout0, kout1;  // output blocks: kout0, kout0 + kstep, ... < kout1
  int64_t jout0;         // grid index of block kout0's output
  int64_t sf_off;        // offset (in blocks) of this chunk in the s_f scratch
  int64_t tail_out_pos, tail_out_j;  // output inside the tail (j < 0: none)
  int64_t r0, r1;        // run-mode: runs [r0, r1) tile blocks [kb, ke) (run r0 = [kb])
  int64_t sr_off;        // run-mode: offset (in runs) of this chunk in the S_in scratch
  int64_t kstep;         // blocks per output-grid interval (sub-blocks: L = R / kstep)
  // run mode, head skip: the head [s0, head_end) is block kb-1 (a one-block
  // run, r0 - 1) minus its first samples; the scan enters block kb from
  // PhiF S + E_f(kb-1) + the head taps on (pad - raw) samples instead of
  // walking the head (off-sample grids: head = L - 1 samples)
  int64_t hskip;
};

struct BlockGeom {
  int64_t n_ch, nb, base;  // blocks k in [0, nb) start at sample base + k*L
  int L;
  int nF;                  // functionals per block (2n+1)
  int64_t n_sf;            // forward-state slots (sum over chunks of their blocks)
};

// Workspace layouts, channel-group major so that each wave's writes form one
// contiguous stream (a wave owns one channel group and walks blocks in order):
//   F  (block functionals): [ch / 16][block][comp][ch % 16]
//   SF (forward states)   : [ch / 64][chunk-block][state][ch % 64]
__host__ __device__ inline int64_t f_index(int64_t k, int c, int64_t ch, int64_t nb, int nF) {
  return (((ch >> 4) * nb + k) * nF + c) * 16 + (ch & 15);
}
__host__ __device__ inline int64_t sf_index(int64_t j, int i, int64_t ch, int64_t n_sf, int n) {
  return (((ch >> 6) * n_sf + j) * n + i) * 64 + (ch & 63);
}
constexpr int F_CSTRIDE = 16;   // element stride between comps of one (block, channel)
constexpr int SF_ISTRIDE = 64;  // element stride between states of one (block, channel)

// Block taps of the MFMA block-functional kernel.  The functionals are linear
// in the block's extended samples: F_c(k) = sum_p Kx[c][p] x[base + k*L - J + p]
// (lfd_capi.cpp block_taps).  Block k's row is read from the row's sample
// floor4(base + k*L - J) (16-B pieces, 4-B aligned on odd strides), i.e. shifted by v = (base + k*L - J) mod 4;
// the device table holds the taps for each shift that occurs (nvar = 1 when
// L % 4 == 0, else 4), zero-padded to Lp samples:
//   taps[v][((t*4 + q)*nc + c)*4 + e] = Kx[c][16t + 4q + e - v]
// (t: 16-sample group, q: MFMA k-lane group, e: MFMA step within the group).
struct TapGeom {
  int Lp;       // padded row length (multiple of 64 samples)
  int J;        // FIR history samples
  int nc;       // functionals per block (<= 16: one MFMA row tile)
  int nvar;     // 1: single shift v0 for every block; 4: table index = shift
  int v0;
};
constexpr int TAP_LDS_MAX = 160 * 1024;  // taps must fit one workgroup's LDS

// Run mode (4th-order cascades, n = 4): K1 folds consecutive blocks into runs
// of <= RUN_R blocks that never straddle a chunk start, chunk start + 1 or
// chunk end, and writes per block only the zero-boundary output y0(k) and per
// run the aggregates E_f = S0(run end), E_r = T0(run start) (zero states at
// both run ends).  With S_in entering the run and T_in entering from its right:
//   y(ks + p)  = y0(ks + p) + A[len][p] . S_in + B[len-1-p] . T_in
//   S_out      = PhiF^len S_in + E_f
//   T(ks)      = PhiR^len T_in + E_r + C[len] S_in
// Layouts (channel-group major): Y0 [ch/16][block][ch%16], AG [ch/16][run][8][ch%16].
constexpr int RUN_R = 8;
constexpr int RUN_N = 4;  // state dimension of run mode
struct RunConst {
  double PhiFp[RUN_R + 1][16];      // PhiF^j
  double PhiRp[RUN_R + 1][16];      // PhiR^j
  double C[RUN_R + 1][16];          // sum_{m<len} PhiR^m M PhiF^m
  double A[RUN_R + 1][RUN_R][4];    // G0 PhiF^p + H0 sum_{m=p+1}^{len-1} PhiR^{m-p-1} M PhiF^m
  double B[RUN_R][4];               // H0 PhiR^d
  // K1 epilogue: PhiF, M, PhiR (row-major 4x4), G0, H0
  double PhiF[16], M[16], PhiR[16], G0[4], H0[4];
  // scan head skip: e_f taps of a block row's first HSKIP_MAX samples
  // (Kx[c][p], c < 4: lfd_capi.cpp block_taps)
  double KfH[4][32];
  // lattice one-pass plans (lfd_capi.cpp plan_create_uniform n_off > 0): H0
  // of the outputs at offsets d = 0 .. LAT_MAX_OFF - 1 of a block
  double H0L[8][4];
};
constexpr int LAT_MAX_OFF = 8;  // output offsets of a lattice one-pass K1 (MFMA rows 8 .. 15)
// Segmented run chains (long chains: lattice plans, dt = 10 s): a chunk's runs
// [r0, r1) cut into <= SEG_MAX segments [ra, rb) of >= SEG_MIN_RUNS runs; P /
// Q = PhiF / PhiR to the segment's block count (the forward / reverse
// transition across it: powers of one matrix, so the run order does not
// matter); last = the chunk's last segment.  Inactive slots: ra == rb.
constexpr int SEG_MAX = 16, SEG_MIN_RUNS = 8;
// the fused one-launch scan (k_scan_fused): FU_SEG_HOST segments per chunk of
// <= FU_SEGR_HOST runs (chunks of more runs take the multi-launch scans)
constexpr int FU_SEG_HOST = 16, FU_SEGR_HOST = 5;
constexpr int SC_N_HOST = 24;  // doubles per (chunk, channel) of the segmented scan's scratch (k_chunk_scan SC_N)
struct SegGeom {
  int64_t ra, rb, last;
  double P[16], Q[16];
  // fused scan (k_scan_fused) only: the chunk's right edge is affine in the
  // forward state S entering it, T_end = T_end(S = 0) + TM S and the tail
  // output = its S = 0 value + tm . S (host-simulated, every entry of the
  // chunk; tmap = 0: walk the edge after the forward states instead)
  int64_t tmap;
  double TM[16], tm[4];
};
constexpr int HSKIP_MAX = 32;
struct RunGeom {
  int64_t n_runs, n_groups, n_sr;
  const int64_t *run_ks;    // first block of run r
  const int *run_len;       // blocks in run r (<= RUN_R)
  const int *group_r0;      // K1 unit g = runs [group_r0[g], group_r0[g+1])
  const RunConst *rc;
};

// Full-rate zero-phase filter (lfd_sosfiltfilt_f32), in SciPy's own
// coordinates: the TDF-II state z of every section (SosCoef; dimension
// N = 2 n_sec).  Big blocks of FR_L = 64 x FR_LS samples; a wave owns one
// (channel, big block) and each lane one FR_LS-sample sub-block.  Inside the
// wave the sub-block states are combined by log-step scans over the lanes
// with the zero-input transition over FR_LS * 2^i samples (PhiP[i]; the
// reverse pass runs the same cascade on the reversed signal, so it shares
// it).  Between the two wave passes k_fullrate_scan walks the big
// blocks per channel:  S_f(k+1) = PhiL S_f(k) + e_f(k),
// T(k) = PhiL T(k+1) + e_r(k) + M S_f(k)  (T(k): reverse state after sample
// k * FR_L).
constexpr int FR_LS = 32;
constexpr int FR_L = 64 * FR_LS;
// Medium blocks of the matrix-core functionals pass (time-contiguous rows):
// FR_LB samples, 4 per big block; their functionals (forward exit A and
// zero-state reverse exit Z, 2N values) are a fp64-MFMA product with a
// 2N x FR_LB tap table (k_block_functionals_mfma), and the segmented scan
// (k_fullrate_scan_seg) walks them.
constexpr int FR_LB = 16 * FR_LS;
struct FRConst {
  SosCoef cf;
  ZiVec zi;                       // sosfilt_zi (unit step steady state)
  double PhiP[6][MAX_N * MAX_N];  // row-major, stride MAX_N
  double PhiL[MAX_N * MAX_N];     // over FR_L samples
  double M[MAX_N * MAX_N];        // reverse exit state over a big block per forward state entering it
  double MB[MAX_N * MAX_N];       // the same over a medium block (FR_LB samples; PhiP[4] is its transition)
  double M32[MAX_N * MAX_N];      // the same over one sub-block
  double H[FR_LS][MAX_N];         // zero-input output i steps after unit state e_n
  double Rh[FR_LS][MAX_N];        // zero-state reverse output at i of H's forward output
  // output table Q[i][kk] = (Rh[i][kk] | H[31 - i][kk - N]) as the A operand of
  // v_mfma_f64_16x16x4 per 16-row tile mt and k-step ks:
  // QA[mt][ks][l] = Q[16 mt + (l & 15)][4 ks + (l >> 4)]
  double QA[2][4][64];
  // functional taps: row c < N the forward exit state A, N <= c < 2N the
  // zero-state reverse exit Z0 of a sub-block per unit sample p (rows >= 2N
  // zero), as the A operand per k-step: KAZ[ks][l] = Kaz[l & 15][4 ks + (l >> 4)]
  double KAZ[FR_LS / 4][64];
  // zero-state response of a sub-block (forward, then reverse over its
  // output): r0[i] = sum_p Kr[i][p] x[p], as the A operand per row tile mt
  // and k-step ks: KRA[mt][ks][l] = Kr[16 mt + (l & 15)][4 ks + (l >> 4)]
  double KRA[2][FR_LS / 4][64];
};
// Layouts (channel fastest, so the scan's per-channel threads coalesce):
//   F [k][2N][ch] (e_f then e_r), SF / ST [k][N][ch] for k in [0, nb].

// Launchers (lfd_kernels.hip).  All return hipError_t of the launch.
// Full-rate wave kernels: out == false writes the big blocks' functionals F;
// out == true reads the scan's SF / ST and writes y[ch, 0 : nb * FR_L].
// mb (out only): SF / ST are the medium-block states of k_fullrate_scan_seg
// over n_mb medium blocks; nb = ceil(n_mb / 4) big blocks (the last partial).
hipError_t launch_fullrate_blocks(int n_sec, bool out, const float *x, int64_t s_ch, int64_t s_t,
                                  int64_t n_ch, int64_t nb, const FRConst *fc, const double *SF,
                                  const double *ST, double *F, double *y, int64_t ys_ch, int64_t ys_t,
                                  hipStream_t st, bool mb = false, int64_t n_mb = 0);
// Segmented scan over the medium blocks (FR_LB) of the matrix-core
// functionals F2 (f_index layout, nF = 2N over 4 nb blocks): a workgroup =
// cw channels (16, or 8 when fewer 16-channel groups than CUs) x G <= 512 / cw
// segments of `seglen` medium blocks; per segment a zero-state
// aggregate, a combine across the segments (powers pseg = PhiB^seglen, plast
// = PhiB^lastlen), the true states; forward then reverse.  Writes SFm / STm
// (the states at every medium block: the output pass's inputs), TP and the
// tail outputs, like k_fullrate_scan.
struct FRSeg {
  double pseg[MAX_N * MAX_N], plast[MAX_N * MAX_N];
  int seglen, lastlen, G, Gu, cw;
};
hipError_t launch_fullrate_scan_seg(int n_sec, const float *x, int64_t s_ch, int64_t s_t, int64_t n_ch, int64_t n_t,
                                    int64_t M, int padlen, const FRConst *fc, const double *F2, double *SFm,
                                    double *STm, double *TP, double *y, int64_t ys_ch, int64_t ys_t,
                                    const FRSeg &sg, hipStream_t st);
// Per-channel walk over the big blocks + both edges (odd extension, zi) and
// the outputs of the tail [nb * FR_L, n_t).  TP: (n_t - nb * FR_L + padlen) x n_ch.
hipError_t launch_fullrate_scan(int n_sec, const float *x, int64_t s_ch, int64_t s_t, int64_t n_ch,
                                int64_t n_t, int64_t nb, int padlen, const FRConst *fc, const double *F,
                                double *SF, double *ST, double *TP, double *y, int64_t ys_ch, int64_t ys_t,
                                hipStream_t st);
// MFMA block functionals: s_t == 1 (any channel stride).
hipError_t launch_block_functionals_mfma(const float *x, int64_t s_ch, int64_t n_t,
                                         const BlockGeom &g, const double *taps,
                                         const TapGeom &tg, double *F, hipStream_t st);
hipError_t launch_block_runs_mfma(const float *x, int64_t s_ch, int64_t n_t, const BlockGeom &g,
                                  const double *taps, const TapGeom &tg, const RunGeom &rg,
                                  double *Y0, double *AG, hipStream_t st);
// Run-mode MFMA K1 for (time, channel) storage (s_ch == 1, row stride s_t):
// tap table with row shift 0 (tg.nvar == 1, tg.v0 == 0).
hipError_t launch_block_runs_mfma_tm(const float *x, int64_t s_t, int64_t n_t, const BlockGeom &g,
                                     const double *taps, const TapGeom &tg, const RunGeom &rg, double *Y0,
                                     double *AG, hipStream_t st);
// Run epilogue applied to per-block functionals F (K1 kernels without run
// mode): F -> Y0, AG (n_sec == 2).
// Lattice one-pass K1 (tg.nc = 8 + n_off output offsets, every run's first
// block an output block): per run, y0 of its first block at every offset
// into Y0 + d * (ceil(n_ch / 16) * nb * 16), and the run aggregates.
hipError_t launch_block_runs_mfma_lat(const float *x, int64_t s_ch, int64_t n_t, const BlockGeom &g,
                                      const double *taps, const TapGeom &tg, const RunGeom &rg, double *Y0,
                                      double *AG, hipStream_t st);
// Lattice one-pass scan: the state scan once (deferred outputs: SR, TR, CR),
// then k_lat_outputs: every offset d (RunConst rc_off[d], chunk outputs
// cg_off[d * n_chunks ..], Y0 slice d) into the slot-major scratch
// y[(d * y_off + j) * n_ch + ch] (y_off = grid points per offset; ys_ch unused).
hipError_t launch_lattice_scan(const float *x, int64_t s_ch, int64_t s_t, const BlockGeom &g, int padlen,
                               const ScanConst &sc, const RunGeom &rg, const ChunkGeom *cg, int64_t n_chunks,
                               const double *Y0, const double *AG, double *SR, double *TP, int64_t tp_len,
                               double *TR, double *CR, const int *slot_chunk, int n_off, const RunConst *rc_off,
                               const ChunkGeom *cg_off, double *y, int64_t ys_ch, int64_t y_off, hipStream_t st,
                               const SegGeom *seg = nullptr, int seg_max = 0, double *SC = nullptr,
                               int *scan_used = nullptr);
hipError_t launch_fold_runs(const double *F, const BlockGeom &g, const RunGeom &rg, double *Y0,
                            double *AG, hipStream_t st);
// Run-mode scan.  With TR / CR / slot_chunk (per run slot: its chunk) the
// outputs are deferred to k_run_outputs (TR: T entering every run, SR's
// layout; CR: [chunk][ch64] p0 corrections).  seg_fu / nw_fu: the fused
// one-launch scan's table ([n_chunks][FU_SEG_HOST]; nw_fu = FU_SEG_HOST when
// every chunk fits, else 0).
hipError_t launch_chunk_scan_runs(const float *x, int64_t s_ch, int64_t s_t, const BlockGeom &g,
                                  int padlen, const ScanConst &sc, const RunGeom &rg,
                                  const ChunkGeom *cg_dev, int64_t n_chunks, const double *Y0,
                                  const double *AG, double *SR, double *TP, int64_t tp_len,
                                  double *y, int64_t ys_ch, int64_t ys_t, hipStream_t st, double *TR = nullptr,
                                  double *CR = nullptr, const int *slot_chunk = nullptr,
                                  const SegGeom *seg = nullptr, int seg_max = 0, double *SC = nullptr,
                                  const SegGeom *seg_fu = nullptr, int nw_fu = 0, int *scan_used = nullptr);
hipError_t launch_block_functionals(int n_sec, bool fir32, const float *x, int64_t s_ch,
                                    int64_t s_t, const BlockGeom &g,
                                    const BlockConst &kc, double *F,
                                    hipStream_t st);
hipError_t launch_chunk_scan(int n_sec, bool fir32, const float *x, int64_t s_ch,
                             int64_t s_t, const BlockGeom &g, int padlen,
                             const ScanConst &sc, const ChunkGeom *cg_dev,
                             int64_t n_chunks, const double *F, double *SF,
                             double *TP, int64_t tp_len, double *y,
                             int64_t ys_ch, int64_t ys_t, hipStream_t st);
hipError_t launch_sosfiltfilt(int n_sec, const float *x, int64_t n_ch,
                              int64_t n_t, int64_t s_ch, int64_t s_t,
                              const SosCoef &c, const ZiVec &zi,
                              int padlen, double *ws, double *y, int64_t ys_ch,
                              int64_t ys_t, hipStream_t st);
hipError_t launch_interp_linear(const double *x, int64_t n_ch, int64_t n_t,
                                int64_t s_ch, int64_t s_t, const int64_t *lo,
                                const double *w, int64_t n_out, double *y,
                                int64_t ys_ch, int64_t ys_t, hipStream_t st);
hipError_t launch_rolling_mean(const float *x, int64_t n_ch, int64_t n_t,
                               int64_t s_ch, int64_t s_t, int64_t W, int64_t S,
                               float *y, int64_t ys_ch, int64_t ys_t,
                               hipStream_t st);
// FIR decimation: y[k] = sum_i h[i] x[k q + delay - i] (x = 0 outside the
// record), k < ceil(n_t / q); h on the device, n_taps <= 12,288.
// *kernel_used = 1 for the matrix-core kernel, 0 for the VALU one.
hipError_t launch_fir_decimate(const float *x, int64_t n_ch, int64_t n_t, int64_t s_ch, int64_t s_t,
                               const double *h, int n_taps, int64_t q, int64_t delay, double *y, int64_t ys_ch,
                               int64_t ys_t, hipStream_t st, int *kernel_used);
// Lattice (composite) plans: y[ch, bj[i]] = (1 - bw[i]) tmp[ch, bi[2i]] +
// bw[i] tmp[ch, bi[2i+1]] (bi[2i+1] < 0: tmp[ch, bi[2i]]), tmp rows of T.
// GridGen (dts > 0): the weights of a regular time grid computed on device
// from integer ns (point j at rel0 + j*step ns after the input's sample 0,
// sampled every dts ns) instead of bw.
struct GridGen {
  int64_t rel0 = 0, step = 0, dts = 0;
};
// the same blend from a slot-major scratch tmp[slot * n_ch + ch] (one-pass
// lattice plans), LDS-tiled so that reads and writes are both coalesced
hipError_t launch_blend_grid_sm(const double *tmp, int64_t n_ch, const int64_t *bj, const int64_t *bi,
                                const double *bw, int64_t nb, double *y, int64_t ys_ch, int64_t ys_t, hipStream_t st,
                                const GridGen &gen);
hipError_t launch_blend_grid(const double *tmp, int64_t T, int64_t n_ch, const int64_t *bj, const int64_t *bi,
                             const double *bw, int64_t nb, double *y, int64_t ys_ch, int64_t ys_t, hipStream_t st,
                             const GridGen &gen = GridGen{});
// lfd_lowpass_execute with a generated grid (a lattice plan's weights from
// `gen`; the stream caches lattice plans by structure).  Other plans ignore it.
// scan_stream (lfd_lowpass_execute_split): the scan and outputs there after
// the block pass (an event); nullptr = everything on `stream`.
int lowpass_execute_gen(const ::lfd_lowpass_plan *p, const float *x, int64_t s_ch, int64_t s_t, double *y,
                        int64_t ys_ch, int64_t ys_t, void *workspace, void *stream, const GridGen &gen,
                        void *scan_stream = nullptr);
// dst[c * dp + r] = src[r * sp + c] for r < n_rows, c < n_cols.
hipError_t launch_transpose(const float *src, int64_t n_rows, int64_t n_cols, int64_t sp, float *dst,
                            int64_t dp, hipStream_t st);
// Notebook post-processing (low_pass_dascore.ipynb cells 14-22).
hipError_t launch_demean_scale(const double *x, int64_t n_rows, int64_t n_cols, int64_t s_r, int64_t s_c,
                               int64_t c0, int64_t c1, double scale, double *y, int64_t ys_r, int64_t ys_c,
                               hipStream_t st);
// scipy.ndimage.median_filter(x, size=(k0, k1), mode='reflect'); LDS tile <= 64 KB.
hipError_t launch_median2d(const double *x, int64_t n0, int64_t n1, int64_t s0, int64_t s1, int k0, int k1,
                           double *y, int64_t ys0, int64_t ys1, hipStream_t st);

}  // namespace lfd
