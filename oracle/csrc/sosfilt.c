/*
 * ORACLE — test infrastructure only. Never linked into the product library.
 *
 * Plain-C restatement of SciPy's second-order-section IIR kernel `_sosfilt`
 * (Cython, shipped compiled as scipy/signal/_sosfilt.cpython-310-*.so; its
 * Python caller is scipy/signal/_signaltools.py:4706, dtype promotion at
 * :4684, moveaxis/copy at :4699-4704).  The reference path reaches it through
 * DASCore Patch.pass_filter -> scipy.signal.sosfiltfilt (lf_das.py:223, :40).
 *
 * Per signal, per sample, per section (transposed direct form II):
 *     y      = b0*x + z0
 *     z0     = b1*x - a1*y + z1
 *     z1     = b2*x - a2*y
 * evaluated left to right with no fused multiply-add, so results are
 * bit-identical to SciPy on x86-64 (checked against scipy.signal.sosfilt in
 * tests/test_oracle.py).  Build with -ffp-contract=off (oracle/Makefile).
 */
#include <stdint.h>

/* x: (n_sig, n_t) row-major float64, filtered in place.
 * zi: (n_sig, n_sec, 2) row-major, updated in place (final state).
 * sos: (n_sec, 6) row-major [b0 b1 b2 a0 a1 a2], a0 == 1. */
void oracle_sosfilt_f64(const double *sos, int n_sec, double *x, int64_t n_sig,
                        int64_t n_t, double *zi) {
  for (int64_t i = 0; i < n_sig; ++i) {
    double *row = x + i * n_t;
    double *z = zi + i * (int64_t)n_sec * 2;
    for (int64_t n = 0; n < n_t; ++n) {
      double x_cur = row[n];
      for (int s = 0; s < n_sec; ++s) {
        const double *c = sos + 6 * s;
        double x_new = c[0] * x_cur + z[2 * s];
        z[2 * s] = c[1] * x_cur - c[4] * x_new + z[2 * s + 1];
        z[2 * s + 1] = c[2] * x_cur - c[5] * x_new;
        x_cur = x_new;
      }
      row[n] = x_cur;
    }
  }
}

/* Channel-block sosfiltfilt driver used only by bench.py's cpu_baseline leg:
 * one call filters `n_sig` rows of float32 input (row stride `s_row` floats)
 * exactly as scipy.signal.sosfiltfilt(sos, x, padtype='odd', padlen=padlen)
 * (scipy/signal/_signaltools.py:4718-4828; odd_ext _arraytools.py:57-107) and
 * writes the float64 result rows (length n_t) to y.  `work` must hold
 * n_t + 2*padlen doubles; `zi` is sosfilt_zi(sos), (n_sec, 2). */
void oracle_sosfiltfilt_rows_f32(const double *sos, int n_sec, const double *zi,
                                 int padlen, const float *x, int64_t n_sig,
                                 int64_t n_t, int64_t s_row, double *y,
                                 double *work) {
  const int64_t n_ext = n_t + 2 * (int64_t)padlen;
  double z[16];
  for (int64_t i = 0; i < n_sig; ++i) {
    const float *xr = x + i * s_row;
    /* odd extension, evaluated in float32 like numpy does for a float32 x */
    for (int k = 0; k < padlen; ++k) {
      float v = 2.0f * xr[0] - xr[padlen - k];
      work[k] = (double)v;
    }
    for (int64_t n = 0; n < n_t; ++n) work[padlen + n] = (double)xr[n];
    for (int k = 0; k < padlen; ++k) {
      float v = 2.0f * xr[n_t - 1] - xr[n_t - 2 - k];
      work[padlen + n_t + k] = (double)v;
    }
    double x0 = work[0];
    for (int s = 0; s < n_sec; ++s) {
      z[2 * s] = zi[2 * s] * x0;
      z[2 * s + 1] = zi[2 * s + 1] * x0;
    }
    oracle_sosfilt_f64(sos, n_sec, work, 1, n_ext, z);
    /* reverse pass on the reversed forward output */
    double y0 = work[n_ext - 1];
    for (int64_t a = 0, b = n_ext - 1; a < b; ++a, --b) {
      double t = work[a]; work[a] = work[b]; work[b] = t;
    }
    for (int s = 0; s < n_sec; ++s) {
      z[2 * s] = zi[2 * s] * y0;
      z[2 * s + 1] = zi[2 * s + 1] * y0;
    }
    oracle_sosfilt_f64(sos, n_sec, work, 1, n_ext, z);
    double *yr = y + i * n_t;
    for (int64_t n = 0; n < n_t; ++n) yr[n] = work[n_ext - 1 - padlen - n];
  }
}
