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
 *   - arithmetic is float64 on device; samples are float32 in.  Low-pass
 *     outputs are float64 (SciPy's sosfiltfilt result dtype,
 *     scipy/signal/_signaltools.py:4684, which lf_das.py:223-232 interpolates
 *     and writes); rolling means are float32.
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

/* Kernel-selection overrides (process-wide; 0 = the library's own choice).
 * Every alternative computes the same outputs within the path's parity
 * tolerance (most bit-identically); they exist so tests can drive the
 * fallback kernels on inputs the default would not send there.  The library
 * reads NO environment variable: its results and kernel choices depend only
 * on the arguments and these options.  (Tuning and diagnostic A/B knobs exist
 * only in the separately built liblfdas_diag.so, -DLFD_DIAG, used by tools/.) */
#define LFD_OPT_NO_RUNS 1         /* block plans: per-block functionals, no run folding   */
#define LFD_OPT_K1_RECURRENCE 2   /* block plans: recurrence K1 instead of fp64 MFMA      */
#define LFD_OPT_TM_NO_PAIRS 3     /* time-major MFMA K1: one dword per channel, no pairs  */
#define LFD_OPT_SCAN_DEFER 4      /* run scan: 1 outputs in the chain, 2 deferred, 3 deferred + segmented chains, 4 fused segmented (one launch) */
#define LFD_OPT_FULLRATE_SERIAL 5 /* lfd_sosfiltfilt_f32: one thread per channel          */
#define LFD_OPT_NO_LATTICE 6      /* drifting grids: LFD_EUNSUPPORTED (per-chunk path)    */
#define LFD_OPT_NO_HEAD_SKIP 7    /* off-sample grids: walk chunk heads                   */
#define LFD_OPT_FIR_VALU 8        /* lfd_fir_decimate_f32: VALU kernel, not matrix cores  */
#define LFD_OPT_FULLRATE_BIGBLOCK 9 /* lfd_sosfiltfilt_f32: big-block functionals + serial scan */
#define LFD_OPT_LATTICE_PHASES 10   /* lattice plans: one block plan per phase, not one pass */
int lfd_set_option(int option, int64_t value);
int lfd_get_option(int option, int64_t *value);

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
 * Grids: uniform spacing with one fraction w (one block plan), or a slowly
 * drifting fraction / spacing (a lattice plan: one block sub-plan per
 * lattice phase + an interp1d blend; e.g. 3 kHz data on integer-ns times).
 * LFD_EUNSUPPORTED for other grids (the caller uses the per-chunk
 * lfd_sos_filtfilt_resample_f32).  For a lattice plan, lfd_lowpass_last_timing
 * reports (all sub-plans, the blend).
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
/* y[ch*ys_ch + j*ys_t] (float64) for j in [0, n_grid) that some chunk produces. */
int lfd_lowpass_execute(const lfd_lowpass_plan *plan, const float *x,
                        int64_t s_ch, int64_t s_t, double *y, int64_t ys_ch,
                        int64_t ys_t, void *workspace, void *stream);
/* Two-stream execute for batch pipelines: the block pass (K1) runs on
 * `block_stream`, the chunk scan and the outputs on `scan_stream` after it
 * (an event), so y is complete in scan_stream order and the workspace is
 * free again once scan_stream has passed this call.  Consecutive executes
 * on two workspaces then overlap one execute's scan and its block pass's
 * drain with the next block pass (lfdas.plan.LowpassPipeline, bench.py).
 * Plans with no separate scan launch (lattice / sub-plan grids) run whole
 * on block_stream and scan_stream waits for them.  Replaces nothing in the
 * reference (LFProc.process_time_range, lf_das.py:219-290, filters one
 * range per call); it is the same computation as lfd_lowpass_execute. */
int lfd_lowpass_execute_split(const lfd_lowpass_plan *plan, const float *x,
                              int64_t s_ch, int64_t s_t, double *y,
                              int64_t ys_ch, int64_t ys_t, void *workspace,
                              void *block_stream, void *scan_stream);
/* Per-kernel device time of the last execute on `stream` (ms), measured
 * with HIP events when enabled by lfd_set_timing(1). */
int lfd_lowpass_last_timing(const lfd_lowpass_plan *plan, float *ms_blocks,
                            float *ms_scan);
/* With lfd_set_timing(n), n > 1: the device times of the last n timed
 * executes of this plan, oldest first (a ring of n event triples, so timed
 * executes need no host synchronisation between them; bench.py). */
int lfd_lowpass_timings(const lfd_lowpass_plan *plan, float *ms_blocks,
                        float *ms_scan, int64_t n);
void lfd_lowpass_plan_destroy(lfd_lowpass_plan *plan);
/* 0: off; 1: time every execute / push / full-rate call; n > 1: also keep
 * the last n low-pass executes' times per plan (lfd_lowpass_timings). */
int lfd_set_timing(int enable);
/* Which block-functional kernel the last execute ran: LFD_K1_MFMA (fp64
 * matrix cores over the plan's block taps; time-contiguous float32 rows,
 * any channel stride) or LFD_K1_RECURRENCE (strided time, or cascades above
 * 6th order); 0 before the first execute. */
#define LFD_K1_RECURRENCE 1
#define LFD_K1_MFMA 2
#define LFD_K1_MFMA_RUNS 3 /* MFMA + in-register run folding (4th-order cascades) */
/* 4th-order cascades whose K1 emits per-block functionals (recurrence K1, or
 * MFMA taps too long for the in-register run buffers, e.g. L = 2000): a
 * separate fold kernel turns them into runs before the scan. */
#define LFD_K1_RECURRENCE_FOLD 4
#define LFD_K1_MFMA_FOLD 5
/* (time, channel) rows (s_ch == 1, the real files' layout): fp64 MFMA over
 * 32-channel row lines, in-register run folding (4th-order cascades). */
#define LFD_K1_MFMA_RUNS_TM 6
int lfd_lowpass_last_kernel(const lfd_lowpass_plan *plan);
/* Which chunk scan the last execute ran: LFD_SCAN_BLOCKS (per-block scan of
 * plans without run folding) or, for run-mode plans, the outputs inside the
 * backward run chain (IN_CHAIN), deferred to a parallel output kernel
 * (DEFERRED), segmented chains (SEGMENTED) or the one-launch fused segmented
 * scan (FUSED); -1 before the first execute.  Testing hook for
 * LFD_OPT_SCAN_DEFER (options 3 / 4 fall back to the default choice when the
 * plan's segment tables do not fit). */
#define LFD_SCAN_BLOCKS 0
#define LFD_SCAN_IN_CHAIN 1
#define LFD_SCAN_DEFERRED 2
#define LFD_SCAN_SEGMENTED 3
#define LFD_SCAN_FUSED 4
int lfd_lowpass_last_scan(const lfd_lowpass_plan *plan);
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
/* Testing hook: a lattice (composite) plan's one-pass form.  *n_offsets =
 * its output offsets (0: the plan has no one-pass form and runs one block
 * plan per phase), *last_onepass = whether the last execute ran it, and
 * *one_pass = the inner block plan (for lfd_debug_block_taps / _runs /
 * _plan_constants; owned by the plan).  NULL outputs are skipped. */
int lfd_debug_lattice(const lfd_lowpass_plan *plan, int64_t *n_offsets, int *last_onepass,
                      const lfd_lowpass_plan **one_pass);
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
                                  const double *w, int64_t n_out, double *y,
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
/* With lfd_set_timing(1): the last blocked lfd_sosfiltfilt_f32's kernel times
 * (ms; waits for them): big-block functionals, per-channel scan, output pass.
 * LFD_EINVAL when that call was untimed or took the serial kernel. */
int lfd_sosfiltfilt_last_timing(float *ms_functionals, float *ms_scan,
                                float *ms_output);

/* Linear interpolation of a device float64 array along time at positions
 * lo[j] + w[j] (DASCore Patch.interpolate → interp1d, _interpolate.py:457). */
int lfd_interp_linear_f64(const double *x, int64_t n_ch, int64_t n_t,
                          int64_t s_ch, int64_t s_t, const int64_t *lo_dev,
                          const double *w_dev, int64_t n_out, double *y,
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

/* ------------------------------------------------------------------------
 * FIR decimation: DASCore Patch.decimate(time=q, filter_type='fir')
 *   (dascore/proc/resample.py, external) = scipy.signal.decimate(x, q,
 *   ftype='fir', zero_phase=True) = resample_poly(x, 1, q, window=h) with
 *   h = firwin(20q+1, 1/q, window='hamming')
 *   (scipy/signal/_signaltools.py decimate, _upfirdn.py):
 *     y[k] = sum_{i < n_taps} taps[i] x[k*q + delay - i], x = 0 outside
 *     [0, n_t), k in [0, ceil(n_t/q));  delay = resample_poly's centring
 *     (10q for decimate's filter).  taps: device float64; y: device float64.
 * ------------------------------------------------------------------------ */
int lfd_fir_decimate_f32(const float *x, int64_t n_ch, int64_t n_t,
                         int64_t s_ch, int64_t s_t, const double *taps_dev,
                         int64_t n_taps, int64_t q, int64_t delay, double *y,
                         int64_t ys_ch, int64_t ys_t, void *stream);
/* Kernel of this thread's last lfd_fir_decimate_f32: 1 = fp64 matrix cores
 * (k_fir_decimate_mfma: time-contiguous rows, q in {4, 5, 6, 8, 10}, n_taps <= 21q + 1),
 * 0 = the VALU kernel (longer filters, or LFD_FIR_VALU=1), -1 = none yet. */
int lfd_fir_decimate_last_kernel(void);

/* ------------------------------------------------------------------------
 * LFProc chunk schedule (host arithmetic, no device): the index loop of
 *   lf_das.py:258-290.  rows[4*i..4*i+3] = (read_first, read_last, out_begin,
 *   out_end) grid indices of chunk i: it selects time_grid[read_first] ..
 *   time_grid[read_last] (inclusive) and writes time_grid[out_begin:out_end].
 *   LFD_EINVAL when the loop cannot progress (process_patch_size <=
 *   2*edge_buff_size; the reference loops forever there) or n_grid < 2.
 * ------------------------------------------------------------------------ */
int lfd_lfproc_schedule(int64_t n_grid, int64_t patch_size, int64_t buff_size,
                        int64_t *rows, int64_t max_rows, int64_t *n_rows);

/* ------------------------------------------------------------------------
 * Streaming low-pass + decimate with a device-resident sample arena.
 *   replaces the real-time loop of low_pass_dascore_edge.ipynb cell 11
 *   (:199-235): every new file triggers a fresh LFProc.process_time_range
 *   (t_1, t_2) (lf_das.py:219-290) with t_2 = newest time_max and
 *   t_1 = get_last_processed_time() (lf_das.py:214-217) - buffer, re-reading
 *   the 2*edge overlap from the archive.  Here the overlap never leaves HBM:
 *   pushes append to a per-channel arena (ping-pong compaction keeps only
 *   what a later run reads), host->HBM copies run on their own HIP stream
 *   (direct DMA from pinned memory, double-buffered pinned staging
 *   otherwise), and each run is one lfd_lowpass_plan execute over all of its
 *   chunks (plans cached by geometry).
 *
 * Modes
 *   LFD_STREAM_EDGE        each push runs process_time_range(t_1, t_hi):
 *                          t_hi = time of the newest sample; t_1 =
 *                          t_start_ns on the first run, afterwards
 *                          last output time - resume_back_ns (the notebook's
 *                          buffer = int((ceil(edge/dt)-1)*dt) s).  Results are
 *                          those of the notebook loop with one file per push.
 *   LFD_STREAM_CONTINUOUS  one process_time_range(t_start_ns, t_end_ns) over
 *                          a spool too large for HBM (out-of-core): chunk i
 *                          runs as soon as time_grid[read_last] has arrived;
 *                          lfd_stream_flush runs what remains.
 * A run that cannot produce an output (time grid of <= 2*B+1 points) is
 * deferred to the next push (the reference indexes out of range there).
 * Pushes must be contiguous in time (next t0 = previous t0 + n_t*sample_ns);
 * otherwise the push fails with "patch merge failed! Gap in data exists"
 * (_check_merge, lf_das.py:16-20).
 * ------------------------------------------------------------------------ */
#define LFD_STREAM_EDGE 0
#define LFD_STREAM_CONTINUOUS 1
#define LFD_STREAM_DRY_RUN 1 /* flags: host bookkeeping only (no device, x may be NULL) */

typedef struct lfd_stream_config {
  int64_t n_ch;                   /* channels of every push                      */
  int64_t sample_ns;              /* input sampling interval, ns                 */
  double output_sample_interval;  /* dt, s; grid step int(dt*1000) ms (lf_das.py:255) */
  int64_t process_patch_size;     /* P (lf_das.py:199)                          */
  int64_t edge_buff_size;         /* B (lf_das.py:200)                          */
  int mode;                       /* LFD_STREAM_EDGE | LFD_STREAM_CONTINUOUS    */
  int flags;                      /* LFD_STREAM_DRY_RUN                         */
  int64_t t_start_ns;             /* edge: first run's t_1; continuous: bgtime  */
  int64_t t_end_ns;               /* continuous: edtime (exclusive)             */
  int64_t resume_back_ns;         /* edge: t_1 = last output - resume_back_ns   */
  int64_t capacity;               /* arena samples per channel (0: automatic)   */
} lfd_stream_config;

typedef struct lfd_stream lfd_stream;

/* Device streams, events and the arena live on the current device. */
int lfd_stream_open(lfd_stream **s, const lfd_stream_config *cfg, const double *sos,
                    int n_sec, int padlen);
/* Allocate the arena (capacity max(cfg capacity, 4*max_push)) and the
 * staging buffer for pushes of up to max_push samples now, so that no push
 * allocates (device allocation after large frees can take seconds). */
int lfd_stream_reserve(lfd_stream *s, int64_t max_push);
/* Append n_t samples of every channel starting at time t0_ns.  x is a HOST
 * array addressed by element strides (s_t == 1: (channel, time) rows;
 * s_ch == 1: (time, channel) rows, transposed on device).  Pinned x
 * (hipHostMalloc / hipHostRegister / lfd_host_alloc) is copied by DMA
 * directly and asynchronously: keep it unchanged until lfd_stream_fetch or
 * lfd_stream_synchronize returns.  Pageable x is staged through two pinned
 * buffers and may be reused on return.  Returns once the copy and the run
 * are enqueued. */
int lfd_stream_push(lfd_stream *s, const float *x, int64_t n_t, int64_t s_ch, int64_t s_t,
                    int64_t t0_ns);
/* Continuous mode: run the chunks still pending (the schedule's tail) on
 * the data received so far.  No-op in edge mode. */
int lfd_stream_flush(lfd_stream *s);

typedef struct lfd_stream_output {
  int64_t n_out;        /* output samples per channel produced by the last push/flush */
  int64_t t_first_ns;   /* time of the first output sample                           */
  int64_t t_step_ns;    /* spacing (int(dt*1000) ms)                                 */
  int64_t n_chunks;     /* LFProc chunks (reference output files) completed          */
  int64_t n_runs;       /* process_time_range runs executed so far                   */
  const double *y;      /* device (n_ch, n_out), row stride ys_ch; valid until the
                           second-next push                                          */
  int64_t ys_ch;
} lfd_stream_output;
int lfd_stream_last_output(const lfd_stream *s, lfd_stream_output *out);
/* Per-chunk output counts of the last push (chunk i holds counts[i] samples). */
int lfd_stream_last_chunks(const lfd_stream *s, int64_t *counts, int64_t max_chunks,
                           int64_t *n_chunks);
/* Wait for the last push (its host->HBM copy and its outputs) and copy the
 * outputs to host y[ch*ys_ch + j*ys_t] (nothing to copy when n_out == 0). */
int lfd_stream_fetch(lfd_stream *s, double *y, int64_t ys_ch, int64_t ys_t);
/* Wait until the last push's host buffer has been read (its host->HBM copy
 * is done; the run may still be executing).  A pinned ring of host buffers is
 * refilled after this returns. */
int lfd_stream_wait_copy(lfd_stream *s);
/* Wait for all enqueued work of the stream. */
int lfd_stream_synchronize(lfd_stream *s);
/* Device time of the last push (ms; needs lfd_set_timing(1)): host->HBM copy
 * (+ transpose) and the low-pass run. */
int lfd_stream_last_timing(const lfd_stream *s, float *ms_copy, float *ms_run);
/* Arena geometry: capacity (samples per channel) and valid columns. */
int lfd_stream_info(const lfd_stream *s, int64_t *capacity, int64_t *held_samples,
                    int64_t *t_first_held_ns);
void lfd_stream_close(lfd_stream *s);
/* Testing hook: low-pass plans this stream has built and plan-cache hits.
 * Uniform grids are cached by (first point, spacing, fraction); lattice grids
 * (3 kHz on integer-ns times) by their structure alone, the fractions being
 * computed on device per run, so a steady stream builds only a few plans. */
int lfd_debug_stream_plans(const lfd_stream *s, int64_t *created, int64_t *hits);

/* Pinned host memory for pushes (hipHostMalloc). */
int lfd_host_alloc(void **p, size_t bytes);
void lfd_host_free(void *p);
/* Page-lock an existing host range (hipHostRegister), e.g. one rank's rows
 * of a full-width host block that several ranks read (lfdas.shard.pin_rows,
 * the cfg5 form of lf_das.py:236-240's per-chunk read across 8 GPUs); pushes
 * from it are then DMA'd directly.  Unregister with the same start pointer. */
int lfd_host_register(void *p, size_t bytes);
int lfd_host_unregister(void *p);

/* ------------------------------------------------------------------------
 * Post-processing of the decimated output (low_pass_dascore.ipynb cells
 * 14-22, notebook numpy/scipy code run on device):
 *   lfd_demean_scale_f64: y[r, c] = (x[r, c] - mean(x[r, c0:c1])) * scale per
 *     time row r ((time, distance) rows: the notebook's
 *     (filtered - mean(filtered[:, c0:c1], axis=1)) * scale_iDAS).
 *   lfd_median_filter_f64: scipy.ndimage.median_filter(x, size=(k0, k1)) with
 *     mode 'reflect', origin 0, rank = k0*k1 // 2 (bit-exact: the output is an
 *     input value; NaN-free input).  1-D traces: n0 = 1, k0 = 1.
 * ------------------------------------------------------------------------ */
int lfd_demean_scale_f64(const double *x, int64_t n_rows, int64_t n_cols, int64_t s_r, int64_t s_c,
                         int64_t c0, int64_t c1, double scale, double *y, int64_t ys_r, int64_t ys_c,
                         void *stream);
int lfd_median_filter_f64(const double *x, int64_t n0, int64_t n1, int64_t s0, int64_t s1, int k0, int k1,
                          double *y, int64_t ys0, int64_t ys1, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* LFDAS_H */
