/*
 * C caller of liblfdas.so through include/lfdas.h only (no Python): what a
 * C/C++ host that replaces lf_das.py's compute would do.  Exercises the plan
 * API (lfd_lowpass_plan_create / execute) and the stream API on constant and
 * ramp inputs whose zero-phase low-pass is known in closed form:
 *   - a constant c stays c (DC gain 1; SciPy's odd extension of a constant is
 *     the constant, zi makes the start steady);
 *   - a ramp a + b*t stays a ramp away from the ends (odd extension of a line
 *     is the same line, and a unit-DC-gain zero-phase filter passes lines).
 * Exit status 0 = pass.  Built by __graft_entry__.build() with gcc against the
 * HIP runtime; run by tests/test_capi.py on the GPU.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/lfdas.h"

#define CHECK(x)                                                              \
  do {                                                                        \
    int rc_ = (x);                                                            \
    if (rc_ != LFD_OK) {                                                      \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_,   \
              lfd_last_error());                                              \
      return 1;                                                               \
    }                                                                         \
  } while (0)
#define HIPCHECK(x)                                                           \
  do {                                                                        \
    if ((x) != hipSuccess) {                                                  \
      fprintf(stderr, "%s:%d %s failed\n", __FILE__, __LINE__, #x);           \
      return 1;                                                               \
    }                                                                         \
  } while (0)

/* scipy.signal.zpk2sos(iirfilter(4, 0.45/250, 'lowpass', 'butter', 'zpk'))
 * (fs = 500 Hz, fc = 0.45 Hz: cfg3), as lfdas.design.lowpass_sos gives it. */
static const double SOS[12] = {
    6.344032428057516e-11, 1.2688064856115032e-10, 6.344032428057516e-11, 1.0, -1.9895737178486945, 0.9896055290874918,
    1.0, 2.0, 1.0, 1.0, -1.9956494127028517, 0.9956813210857649};

static int lowpass_plan_case(void) {
  const int64_t n_ch = 40, n_t = 500 * 400, L = 500; /* 400 s @ 500 Hz, decimate to 1 Hz */
  const int64_t n_grid = n_t / L;
  int64_t *lo = malloc(sizeof(int64_t) * n_grid);
  double *w = calloc(n_grid, sizeof(double));
  for (int64_t j = 0; j < n_grid; ++j) lo[j] = j * L;
  /* LFProc chunks with P = 100, B = 7 (lf_das.py:258-290) */
  int64_t rows[4 * 16], nr = 0;
  CHECK(lfd_lfproc_schedule(n_grid, 100, 7, rows, 16, &nr));
  lfd_chunk ck[16];
  for (int64_t i = 0; i < nr; ++i) {
    ck[i].s0 = lo[rows[4 * i]];
    ck[i].s1 = lo[rows[4 * i + 1]];
    ck[i].g0 = rows[4 * i + 2];
    ck[i].g1 = rows[4 * i + 3];
  }
  lfd_lowpass_plan *plan = NULL;
  CHECK(lfd_lowpass_plan_create(&plan, SOS, 2, -1, n_ch, n_t, lo, w, n_grid, ck, nr));
  size_t ws_bytes = 0;
  int64_t nb = 0, bl = 0;
  CHECK(lfd_lowpass_plan_info(plan, &ws_bytes, &nb, &bl));
  float *hx = malloc(sizeof(float) * n_ch * n_t);
  for (int64_t c = 0; c < n_ch; ++c)
    for (int64_t t = 0; t < n_t; ++t)
      hx[c * n_t + t] = (c % 2) ? (float)(3.0 + 0.25 * c) : (float)(-1.0 + 1e-4 * (double)t);
  float *dx;
  double *dy; /* float64 outputs (SciPy's sosfiltfilt result dtype) */
  void *dws;
  HIPCHECK(hipMalloc((void **)&dx, sizeof(float) * n_ch * n_t));
  HIPCHECK(hipMalloc((void **)&dy, sizeof(double) * n_ch * n_grid));
  HIPCHECK(hipMalloc(&dws, ws_bytes > 256 ? ws_bytes : 256));
  HIPCHECK(hipMemcpy(dx, hx, sizeof(float) * n_ch * n_t, hipMemcpyHostToDevice));
  HIPCHECK(hipMemset(dy, 0, sizeof(double) * n_ch * n_grid));
  CHECK(lfd_lowpass_execute(plan, dx, n_t, 1, dy, n_grid, 1, dws, NULL));
  HIPCHECK(hipDeviceSynchronize());
  double *hy = malloc(sizeof(double) * n_ch * n_grid);
  HIPCHECK(hipMemcpy(hy, dy, sizeof(double) * n_ch * n_grid, hipMemcpyDeviceToHost));
  /* constants are exact up to rounding; ramps carry the decayed start-up
   * transient of sosfilt_zi (steady state of a constant, not of a ramp) B = 7
   * outputs into each chunk */
  double worst = 0.0, worst_ramp = 0.0;
  for (int64_t i = 0; i < nr; ++i)
    for (int64_t j = ck[i].g0; j < ck[i].g1; ++j)
      for (int64_t c = 0; c < n_ch; ++c) {
        const double want = (c % 2) ? 3.0 + 0.25 * c : -1.0 + 1e-4 * (double)lo[j];
        const double err = fabs(hy[c * n_grid + j] - want) / fabs(want);
        if (c % 2 && err > worst) worst = err;
        if (!(c % 2) && fabs(hy[c * n_grid + j] - want) > worst_ramp) worst_ramp = fabs(hy[c * n_grid + j] - want);
      }
  printf("plan: %lld chunks, %lld blocks of %lld, kernel %d, constant rel err %.3e, ramp abs err %.3e\n",
         (long long)nr, (long long)nb, (long long)bl, lfd_lowpass_last_kernel(plan), worst, worst_ramp);
  lfd_lowpass_plan_destroy(plan);
  hipFree(dx);
  hipFree(dy);
  hipFree(dws);
  free(hx);
  free(hy);
  free(lo);
  free(w);
  return (worst < 1e-10 && worst_ramp < 1e-3) ? 0 : 1;
}

static int stream_case(void) {
  const int64_t n_ch = 8, push = 500 * 30; /* 30 s files @ 500 Hz */
  lfd_stream_config cfg = {0};
  cfg.n_ch = n_ch;
  cfg.sample_ns = 2000000;
  cfg.output_sample_interval = 1.0;
  cfg.process_patch_size = 125;
  cfg.edge_buff_size = 7;
  cfg.mode = LFD_STREAM_EDGE;
  cfg.t_start_ns = 1679464800000000000LL;
  cfg.resume_back_ns = 6000000000LL;
  lfd_stream *s = NULL;
  CHECK(lfd_stream_open(&s, &cfg, SOS, 2, -1));
  CHECK(lfd_stream_reserve(s, push));
  float *hx = NULL;
  CHECK(lfd_host_alloc((void **)&hx, sizeof(float) * n_ch * push));
  double hy[8 * 64];
  int64_t total = 0, last_t = 0;
  double worst = 0.0;
  for (int k = 0; k < 6; ++k) {
    for (int64_t c = 0; c < n_ch; ++c)
      for (int64_t t = 0; t < push; ++t) hx[c * push + t] = (float)(10.0 + c);
    CHECK(lfd_stream_push(s, hx, push, push, 1, cfg.t_start_ns + (int64_t)k * push * cfg.sample_ns));
    lfd_stream_output o;
    CHECK(lfd_stream_last_output(s, &o));
    if (o.n_out > 64) return 1;
    CHECK(lfd_stream_fetch(s, hy, o.n_out, 1));
    if (o.n_out && total && o.t_first_ns != last_t + o.t_step_ns) {
      fprintf(stderr, "outputs not contiguous across pushes\n");
      return 1;
    }
    for (int64_t c = 0; c < n_ch; ++c)
      for (int64_t j = 0; j < o.n_out; ++j) {
        const double err = fabs(hy[c * o.n_out + j] - (10.0 + c)) / (10.0 + c);
        if (err > worst) worst = err;
      }
    if (o.n_out) last_t = o.t_first_ns + (o.n_out - 1) * o.t_step_ns;
    total += o.n_out;
  }
  int64_t cap = 0, held = 0, t_held = 0;
  CHECK(lfd_stream_info(s, &cap, &held, &t_held));
  printf("stream: %lld outputs over 6 pushes, arena %lld held %lld, worst rel err %.3e\n",
         (long long)total, (long long)cap, (long long)held, worst);
  lfd_stream_close(s);
  lfd_host_free(hx);
  return (worst < 1e-10 && total > 100) ? 0 : 1;
}

int main(void) {
  int n = 0;
  CHECK(lfd_device_count(&n));
  if (n < 1) {
    fprintf(stderr, "no HIP device\n");
    return 2;
  }
  if (lowpass_plan_case()) return 1;
  if (stream_case()) return 1;
  printf("capi smoke ok (liblfdas %d)\n", lfd_version());
  return 0;
}
