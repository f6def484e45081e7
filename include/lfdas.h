/*
 * lfdas.h — C-ABI of the MI355X-native low-frequency DAS hot path
 * (liblfdas.so, built from low-freq-real-time_amd/csrc/ for gfx950).
 *
 * This is the drop-in boundary for the reference's hot path
 * (DASDAE/low-freq-real-time):
 *
 *   lf_das.py:219-290  LFProc.process_time_range — chunked low-pass + resample
 *   lf_das.py:223-225  DASCore Patch.pass_filter(time=(None, fc))
 *                        .interpolate(time=time_grid[a:b])
 *                        → scipy.signal.sosfiltfilt (scipy/signal/_signaltools.py:4718)
 *                        → scipy.interpolate.interp1d  (scipy/interpolate/_interpolate.py:457)
 *   rolling_mean_dascore.ipynb:148   Patch.rolling(time=w, step=s).mean()
 *
 * The reference binds these through Python (DASCore → SciPy's Cython
 * `_sosfilt`); the Python host in low-freq-real-time_amd/lfdas binds this
 * header with ctypes (INTEGRATION.md shows the stub).
 *
 * Conventions
 *   - every call returns int: LFD_OK (0) or a negative LFD_E* code; the
 *     message of the last failure on the calling thread is lfd_last_error().
 *   - `x`, `y`, `workspace` are DEVICE pointers (hipMalloc / torch CUDA
 *     tensors).  sos / grid / chunk tables are HOST arrays copied at plan
 *     creation.  `stream` is a hipStream_t (NULL = default stream).
 *   - arrays are 2-D (channel, time) addressed through element strides
 *     (s_ch, s_t): DASCore's dims ("distance","time") is s_t == 1, the
 *     real-file layout ("time","distance") is s_ch == 1.
 *   - arithmetic is float64 on device; samples are float32 in, float32 out.
 *   - caller owns x / y / workspace; the library owns plans only.
 *   - entry points are re-entrant per (device, stream); execute functions
 *     do no allocation and no synchronisation (hipGraph-capturable).
 */
#ifndef LFDAS_H
#define LFDAS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LFD_OK 0
#define LFD_EINVAL (-1)       /* bad argument (message says which)              */
#define LFD_EHIP (-2)         /* HIP runtime error                              */
#define LFD_EUNSUPPORTED (-3) /* valid request this plan type cannot express    */
#define LFD_ENOMEM (-4)

/* Thread-local message of the last failing call ("" if none). */
const char *lfd_last_error(void);
/* Library version: major*10000 + minor*100 + patch. */
int lfd_version(void);
/* Number of visible HIP devices (replaces nothing in the reference; used by
 * the multi-GPU channel sharding of the host). */
int lfd_device_count(int *count);

/* ------------------------------------------------------------------------
 * Chunked zero-phase Butterworth low-pass + resample
 *   replaces: lf_das.py:219-290 (process_time_range's chunk loop) with its
 *   per-chunk lf_das.py:223-225 (pass_filter → interpolate).
 *
 * Output grid: n_grid points at sample positions grid_lo[j] + grid_w[j]
 * (global sample index of the input array, 0 <= w < 1).  Chunk c reads the
 * INCLUSIVE sample range [s0, s1] (Spool.select(time=(tg[a], tg[b])) after
 * the merge, lf_das.py:236-240) and produces grid points [g0, g1)
 * (time_grid[bgind:edind], lf_das.py:224).  Each chunk is filtered exactly as
 * scipy.signal.sosfiltfilt(sos, x[s0:s1+1], padtype='odd', padlen=padlen)
 * (padlen < 0 → SciPy's default 3*(2*n_sec+1 - ...)) and linearly
 * interpolated at its grid points.  Chunks may overlap (they do in
 * LFProc); overlapping samples are read from HBM once.
 * ------------------------------------------------------------------------ */
typedef struct lfd_chunk {
  int64_t s0, s1; /* inclusive input sample range                         */
  int64_t g0, g1; /* output grid indices [g0, g1)                         */
} lfd_chunk;

typedef struct lfd_lowpass_plan lfd_lowpass_plan;

int lfd_lowpass_plan_create(lfd_lowpass_plan **plan, const double *sos,
                            int n_sec, int padlen, int64_t n_ch, int64_t n_t,
                            const int64_t *grid_lo, const double *grid_w,
                            int64_t n_grid, const lfd_chunk *chunks,
                            int64_t n_chunks);
/* Workspace bytes needed by lfd_lowpass_execute, block geometry. */
int lfd_lowpass_plan_info(const lfd_lowpass_plan *plan, size_t *workspace_bytes,
                          int64_t *n_blocks, int64_t *block_len);
/* y[ch*ys_ch + j*ys_t] for j in [0, n_grid) that some chunk produces. */
int lfd_lowpass_execute(const lfd_lowpass_plan *plan, const float *x,
                        int64_t s_ch, int64_t s_t, float *y, int64_t ys_ch,
                        int64_t ys_t, void *workspace, void *stream);
/* Per-kernel device time of the last execute on `stream` (ms), measured
 * with HIP events when enabled by lfd_set_timing(1). */
int lfd_lowpass_last_timing(const lfd_lowpass_plan *plan, float *ms_blocks,
                            float *ms_scan);
void lfd_lowpass_plan_destroy(lfd_lowpass_plan *plan);
int lfd_set_timing(int enable);
/* Which block-functional kernel the last execute ran: LFD_K1_MFMA (fp64
 * matrix cores over the plan's block taps; time-contiguous float32 rows,
 * 16-B aligned, channel stride a multiple of 4) or LFD_K1_RECURRENCE (any
 * strides, or cascades above 6th order); 0 before the first execute. */
#define LFD_K1_RECURRENCE 1
#define LFD_K1_MFMA 2
#define LFD_K1_MFMA_RUNS 3 /* MFMA + in-register run folding (4th-order cascades) */
int lfd_lowpass_last_kernel(const lfd_lowpass_plan *plan);
/* Testing hook: the plan's block taps Kx[n_comp][row_len] in natural layout,
 * F_c(k) = sum_p Kx[c][p] x[base + k*L - J + p] (row_len = L + J).  With
 * taps == NULL only the sizes are returned.  LFD_EUNSUPPORTED when the plan
 * runs the recurrence kernel only. */
int lfd_debug_block_taps(const lfd_lowpass_plan *plan, double *taps, size_t n_taps,
                         int *n_comp, int64_t *row_len);
/* Testing hook: the run table (first block, length of every run) and the
 * run-mode constants (lfd::RunConst of csrc/lfd_internal.h).  NULL arrays
 * are skipped.  LFD_EUNSUPPORTED when the plan has no run mode. */
int lfd_debug_runs(const lfd_lowpass_plan *plan, int64_t *run_ks, int *run_len,
                   int64_t max_runs, int64_t *n_runs, void *run_const, size_t rc_bytes);
/* Testing hook (not a stable interface): copies the plan's kernel constants
 * (lfd::BlockConst, lfd::ScanConst, lfd::ChunkGeom[n_chunks] of
 * csrc/lfd_internal.h) so CPU tests can check the host math without a GPU.
 * A plan created where no device is visible is host-only: execute fails. */
int lfd_debug_plan_constants(const lfd_lowpass_plan *plan, void *block_const,
                             size_t bc_bytes, void *scan_const, size_t sc_bytes,
                             void *chunk_geom, size_t cg_bytes);

/* One-shot form for a single patch: Patch.pass_filter(time=(None,fc))
 * .interpolate(time=t) (lf_das.py:40-42, :223-225).  Allocates its own
 * workspace (not graph-capturable). */
int lfd_sos_filtfilt_resample_f32(const float *x, int64_t n_ch, int64_t n_t,
                                  int64_t s_ch, int64_t s_t, const double *sos,
                                  int n_sec, int padlen, const int64_t *lo,
                                  const double *w, int64_t n_out, float *y,
                                  int64_t ys_ch, int64_t ys_t, void *stream);

/* ------------------------------------------------------------------------
 * Full-rate zero-phase filter: DASCore Patch.pass_filter(..., zerophase=True)
 * alone → scipy.signal.sosfiltfilt (scipy/signal/_signaltools.py:4718-4828).
 * y is float64 (SciPy's result dtype, _signaltools.py:4684).
 * workspace: lfd_sosfiltfilt_workspace_bytes(n_ch, n_t, padlen) bytes.
 * ------------------------------------------------------------------------ */
size_t lfd_sosfiltfilt_workspace_bytes(int64_t n_ch, int64_t n_t, int padlen,
                                       int n_sec);
int lfd_sosfiltfilt_f32(const float *x, int64_t n_ch, int64_t n_t,
                        int64_t s_ch, int64_t s_t, const double *sos,
                        int n_sec, int padlen, double *y, int64_t ys_ch,
                        int64_t ys_t, void *workspace, void *stream);

/* Linear interpolation of a device float64 array along time at positions
 * lo[j] + w[j] (DASCore Patch.interpolate → interp1d, _interpolate.py:457). */
int lfd_interp_linear_f64(const double *x, int64_t n_ch, int64_t n_t,
                          int64_t s_ch, int64_t s_t, const int64_t *lo_dev,
                          const double *w_dev, int64_t n_out, float *y,
                          int64_t ys_ch, int64_t ys_t, void *stream);

/* ------------------------------------------------------------------------
 * Rolling mean: DASCore Patch.rolling(time=W*dt, step=S*dt, engine='numpy')
 * .mean() (rolling_mean_dascore.ipynb:148, _edge.ipynb:193,213):
 *   y[k] = mean(x[k*S-W+1 : k*S+1]) for k*S >= W-1, else NaN,
 *   k in [0, ceil(n_t/S)).  Sum in float64, result rounded to float32.
 * ------------------------------------------------------------------------ */
int lfd_rolling_mean_f32(const float *x, int64_t n_ch, int64_t n_t,
                         int64_t s_ch, int64_t s_t, int64_t window,
                         int64_t step, float *y, int64_t ys_ch, int64_t ys_t,
                         void *stream);

#ifdef __cplusplus
}
#endif
#endif /* LFDAS_H */
