// C-ABI of liblfdas.so (include/lfdas.h): plan construction (host math in
// x87 extended precision), workspace layout and kernel sequencing.
//
// The per-chunk semantics replicate scipy.signal.sosfiltfilt with odd padding
// (scipy/signal/_signaltools.py:4718-4828) followed by linear interp1d at the
// chunk's output grid (scipy/interpolate/_interpolate.py:457-484), as DASCore's
// Patch.pass_filter(...).interpolate(...) does at lf_das.py:223-225, for every
// chunk of LFProc.process_time_range (lf_das.py:252-290).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/lfdas.h"
#include "lfd_internal.h"

using lfd::MAX_N;
using lfd::MAX_SEC;

namespace {
thread_local std::string g_err;
}  // namespace

int lfd::fail(int code, const std::string &m) {
  g_err = m;
  return code;
}

namespace {
using lfd::fail;
std::atomic<int> g_timing{0};
}  // namespace

bool lfd::timing_enabled() { return g_timing.load() != 0; }

namespace {
constexpr int N_OPT = 11;  // LFD_OPT_* ids are 1 .. N_OPT - 1
std::atomic<int64_t> g_opt[N_OPT];
// set explicitly through lfd_set_option (then the diagnostic build's
// environment names are not read, so lfd_set_option(id, 0) restores the
// library's choice even while an A/B variable is exported)
std::atomic<bool> g_opt_set[N_OPT];
#ifdef LFD_DIAG
// the A/B environment names the tools/ recipes of rounds 1-3 use
const char *const k_opt_env[N_OPT] = {nullptr,          "LFD_NO_RUNS",    "LFD_K1_REC",
                                      "LFD_TM_NO_X2",   "LFD_SCAN_DEFER", "LFD_FULLRATE_SERIAL",
                                      "LFD_NO_LATTICE", "LFD_NO_HSKIP",   "LFD_FIR_VALU",
                                      "LFD_FULLRATE_BIGBLOCK", "LFD_LATTICE_PHASES"};
#endif
}  // namespace

int64_t lfd::option(int id) {
  if (id <= 0 || id >= N_OPT) return 0;
  const int64_t v = g_opt[id].load(std::memory_order_relaxed);
#ifdef LFD_DIAG
  if (!g_opt_set[id].load(std::memory_order_relaxed) && k_opt_env[id]) {
    if (const char *e = std::getenv(k_opt_env[id])) {
      // LFD_SCAN_DEFER=0/1 meant in-chain / deferred (3: segmented chains,
      // 4: the fused one-launch segmented scan)
      if (id == LFD_OPT_SCAN_DEFER) {
        const int d = std::atoi(e);
        return d == 3 || d == 4 ? d : (d != 0 ? 2 : 1);
      }
      return std::atoll(e);
    }
  }
#endif
  return v;
}

namespace {

#define LFD_HIP(call)                                                      \
  do {                                                                     \
    hipError_t e_ = (call);                                                \
    if (e_ != hipSuccess)                                                  \
      return fail(LFD_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

typedef long double R;

struct Cascade {
  int ns = 0;
  double b0[MAX_SEC], b1[MAX_SEC], b2[MAX_SEC], a1[MAX_SEC], a2[MAX_SEC];
};

// scipy/signal/_filter_design.py:728 `_validate_sos`: shape (n, 6), a0 == 1.
int load_sos(const double *sos, int n_sec, Cascade &c) {
  if (!sos) return fail(LFD_EINVAL, "sos is NULL");
  if (n_sec < 1 || n_sec > MAX_SEC)
    return fail(LFD_EINVAL, "n_sec must be in [1, " + std::to_string(MAX_SEC) + "]");
  c.ns = n_sec;
  for (int s = 0; s < n_sec; ++s) {
    const double *r = sos + 6 * s;
    for (int i = 0; i < 6; ++i)
      if (!std::isfinite(r[i])) return fail(LFD_EINVAL, "sos has non-finite coefficients");
    if (r[3] != 1.0) return fail(LFD_EINVAL, "sos[:, 3] should be all ones");
    c.b0[s] = r[0];
    c.b1[s] = r[1];
    c.b2[s] = r[2];
    c.a1[s] = r[4];
    c.a2[s] = r[5];
  }
  return LFD_OK;
}

// scipy/signal/_signaltools.py:4811-4813
int default_padlen(const Cascade &c) {
  int nb2 = 0, na2 = 0;
  for (int s = 0; s < c.ns; ++s) {
    nb2 += c.b2[s] == 0.0;
    na2 += c.a2[s] == 0.0;
  }
  return 3 * (2 * c.ns + 1 - std::min(nb2, na2));
}

// scipy/signal/_signaltools.py:4103-4175 (sosfilt_zi) with lfilter_zi's 2x2
// solve of (I - companion(a).T) zi = b[1:] - a[1:] b0.
void sosfilt_zi(const Cascade &c, double *zi) {
  R scale = 1.0L;
  for (int s = 0; s < c.ns; ++s) {
    const R b0 = c.b0[s], b1 = c.b1[s], b2 = c.b2[s], a1 = c.a1[s], a2 = c.a2[s];
    const R r0 = b1 - a1 * b0, r1 = b2 - a2 * b0;
    const R det = (1.0L + a1) + a2;
    const R z0 = (r0 + r1) / det;
    const R z1 = ((1.0L + a1) * r1 - a2 * r0) / det;
    zi[2 * s] = (double)(scale * z0);
    zi[2 * s + 1] = (double)(scale * z1);
    scale *= (b0 + b1 + b2) / ((1.0L + a1) + a2);
  }
}

struct Mat {
  int n;
  R a[MAX_N][MAX_N];
  explicit Mat(int n_ = 0) : n(n_) {
    for (int i = 0; i < MAX_N; ++i)
      for (int j = 0; j < MAX_N; ++j) a[i][j] = 0;
  }
  static Mat eye(int n) {
    Mat m(n);
    for (int i = 0; i < n; ++i) m.a[i][i] = 1;
    return m;
  }
  Mat operator*(const Mat &o) const {
    Mat r(n);
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < n; ++k)
        for (int j = 0; j < n; ++j) r.a[i][j] += a[i][k] * o.a[k][j];
    return r;
  }
};

Mat mpow(const Mat &A, int64_t e) {
  Mat r = Mat::eye(A.n), b = A;
  while (e > 0) {
    if (e & 1) r = r * b;
    b = b * b;
    e >>= 1;
  }
  return r;
}

bool minv(const Mat &A, Mat &out) {
  const int n = A.n;
  R w[MAX_N][2 * MAX_N];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 2 * n; ++j) w[i][j] = j < n ? A.a[i][j] : (j - n == i);
  for (int col = 0; col < n; ++col) {
    int p = col;
    for (int i = col + 1; i < n; ++i)
      if (std::fabs(w[i][col]) > std::fabs(w[p][col])) p = i;
    if (w[p][col] == 0) return false;
    for (int j = 0; j < 2 * n; ++j) std::swap(w[p][j], w[col][j]);
    const R d = w[col][col];
    for (int j = 0; j < 2 * n; ++j) w[col][j] /= d;
    for (int i = 0; i < n; ++i)
      if (i != col) {
        const R f = w[i][col];
        for (int j = 0; j < 2 * n; ++j) w[i][j] -= f * w[col][j];
      }
  }
  out = Mat(n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) out.a[i][j] = w[i][j + n];
  return true;
}

// ---------------------------------------------------------------------------
// Realization R (lfd_internal.h): factored numerator FIR + all-pole sections.
// Every kernel constant is obtained by simulating the same recurrences in
// extended precision (so host and device agree on coordinates by
// construction).
// ---------------------------------------------------------------------------
struct RModel {
  int ns = 0, J = 0;
  R a1[MAX_SEC], a2[MAX_SEC];
  R c[lfd::MAX_J + 1];
  R G = 0;
};

int make_rmodel(const Cascade &cs, RModel &m) {
  m.ns = cs.ns;
  m.J = 2 * cs.ns;
  R N[lfd::MAX_J + 1] = {0};
  N[0] = 1;
  int deg = 0;
  for (int s = 0; s < cs.ns; ++s) {
    const R b[3] = {cs.b0[s], cs.b1[s], cs.b2[s]};
    R out[lfd::MAX_J + 1] = {0};
    for (int i = 0; i <= deg; ++i)
      for (int j = 0; j < 3; ++j) out[i + j] += N[i] * b[j];
    deg += 2;
    for (int i = 0; i <= deg; ++i) N[i] = out[i];
  }
  if (N[0] == 0) return fail(LFD_EUNSUPPORTED, "numerator with a zero leading coefficient");
  m.G = N[0];
  for (int j = 0; j <= m.J; ++j) m.c[j] = N[j] / N[0];
  for (int s = 0; s < cs.ns; ++s) {
    m.a1[s] = cs.a1[s];
    m.a2[s] = cs.a2[s];
    if (cs.a2[s] == 0.0)
      return fail(LFD_EUNSUPPORTED, "a section with a2 == 0 (odd order) needs the full-rate path");
    if ((1.0L + m.a1[s]) + m.a2[s] == 0)
      return fail(LFD_EUNSUPPORTED, "a section with a pole at z = 1");
  }
  return LFD_OK;
}

// forward all-pole (S[2s] = v_s[n-1], S[2s+1] = v_s[n-2]); returns v_last
R r_allpole(const RModel &m, R *S, R v) {
  for (int s = 0; s < m.ns; ++s) {
    const R vn = v - m.a1[s] * S[2 * s] - m.a2[s] * S[2 * s + 1];
    S[2 * s + 1] = S[2 * s];
    S[2 * s] = vn;
    v = vn;
  }
  return v;
}

struct BlockSim {
  R ef[MAX_N], er0[MAX_N], p0;
};

// One block of L samples with given initial forward state, reverse state
// entering from the right and an optional unit impulse in w at offset imp.
// p0 is the output functional: (1 - ow) y[off] + ow y[off + 1] (ow > 0 needs
// L >= off + J + 2; off > 0: the lattice plans' output offsets).
BlockSim sim_block(const RModel &m, int L, const R *Sf0, const R *Tr0, int imp, R ow, int off = 0) {
  const int n = 2 * m.ns;
  R S[MAX_N], T[MAX_N];
  for (int i = 0; i < n; ++i) {
    S[i] = Sf0 ? Sf0[i] : 0;
    T[i] = Tr0 ? Tr0[i] : 0;
  }
  std::vector<R> yf(L), ql(L);
  for (int k = 0; k < L; ++k) yf[k] = m.G * r_allpole(m, S, k == imp ? 1.0L : 0.0L);
  for (int k = L - 1; k >= 0; --k) ql[k] = r_allpole(m, T, yf[k]);
  BlockSim o;
  for (int i = 0; i < n; ++i) {
    o.ef[i] = S[i];
    o.er0[i] = T[i];
  }
  R acc0 = 0, acc1 = 0;
  for (int j = 0; j <= m.J; ++j) {
    acc0 += m.c[j] * ql[off + j];
    if (ow != 0) acc1 += m.c[j] * ql[off + j + 1];
  }
  o.p0 = m.G * ((1.0L - ow) * acc0 + ow * acc1);
  return o;
}

// Weights e[i] (i <= J + 1) of the reverse outputs q_last[i] in the output
// functional: (1 - ow) sum_j c_j q[j] + ow sum_j c_j q[j + 1].
void out_weights(const RModel &m, R ow, R *e) {
  for (int i = 0; i <= m.J + 1; ++i) {
    e[i] = 0;
    if (i <= m.J) e[i] += (1.0L - ow) * m.c[i];
    if (i >= 1) e[i] += ow * m.c[i - 1];
  }
}

// Device coefficients of realization R; fir32 = no negative FIR tap.
void make_rcoef(const RModel &m, lfd::RCoef &rc, bool &fir32) {
  R csum = 0;
  fir32 = true;
  for (int j = 0; j <= m.J; ++j) {
    rc.c64[j] = (double)m.c[j];
    rc.c32[j] = (float)m.c[j];
    csum += m.c[j];
    if (m.c[j] < 0) fir32 = false;  // cancellation: keep the FIR in float64
  }
  rc.G = (double)m.G;
  rc.csum = (double)csum;
  for (int s = 0; s < m.ns; ++s) {
    rc.na1[s] = (double)-m.a1[s];
    rc.na2[s] = (double)-m.a2[s];
    rc.nia2[s] = (double)(-1.0L / m.a2[s]);
    rc.nra[s] = (double)(-m.a1[s] / m.a2[s]);
    rc.dcg[s] = (double)(1.0L / ((1.0L + m.a1[s]) + m.a2[s]));
  }
}

// Full-rate constants (lfd_internal.h FRConst): SciPy's TDF-II cascade
// (_sosfilt, scipy/signal/_signaltools.py:4706) simulated in extended
// precision.
R tdf2_step(const Cascade &c, R *z, R v) {
  for (int s = 0; s < c.ns; ++s) {
    const R yv = c.b0[s] * v + z[2 * s];
    z[2 * s] = c.b1[s] * v - c.a1[s] * yv + z[2 * s + 1];
    z[2 * s + 1] = c.b2[s] * v - c.a2[s] * yv;
    v = yv;
  }
  return v;
}

void fullrate_constants(const Cascade &cs, lfd::FRConst &fc) {
  const int n = 2 * cs.ns;
  std::memset(&fc, 0, sizeof(fc));
  for (int s = 0; s < cs.ns; ++s) {
    fc.cf.b0[s] = cs.b0[s];
    fc.cf.b1[s] = cs.b1[s];
    fc.cf.b2[s] = cs.b2[s];
    fc.cf.a1[s] = cs.a1[s];
    fc.cf.a2[s] = cs.a2[s];
  }
  sosfilt_zi(cs, fc.zi.v);
  Mat P(n);
  for (int c = 0; c < n; ++c) {
    R z[MAX_N] = {0};
    z[c] = 1;
    for (int t = 0; t < lfd::FR_LS; ++t) (void)tdf2_step(cs, z, 0);
    for (int r = 0; r < n; ++r) P.a[r][c] = z[r];
  }
  for (int i = 0; i < 6; ++i) {
    for (int r = 0; r < n; ++r)
      for (int c = 0; c < n; ++c) fc.PhiP[i][r * MAX_N + c] = (double)P.a[r][c];
    P = P * P;
  }
  for (int r = 0; r < n; ++r)  // P = PhiP[5]^2: FR_L samples
    for (int c = 0; c < n; ++c) fc.PhiL[r * MAX_N + c] = (double)P.a[r][c];
  std::vector<R> yv(lfd::FR_L);
  for (int c = 0; c < n; ++c) {
    R z[MAX_N] = {0};
    z[c] = 1;
    for (int i = 0; i < lfd::FR_L; ++i) {
      yv[i] = tdf2_step(cs, z, 0);
      if (i < lfd::FR_LS) fc.H[i][c] = (double)yv[i];
    }
    R t[MAX_N] = {0};
    for (int i = lfd::FR_L - 1; i >= 0; --i) (void)tdf2_step(cs, t, yv[i]);
    for (int r = 0; r < n; ++r) fc.M[r * MAX_N + c] = (double)t[r];
    R tb[MAX_N] = {0};
    for (int i = lfd::FR_LB - 1; i >= 0; --i) (void)tdf2_step(cs, tb, yv[i]);
    for (int r = 0; r < n; ++r) fc.MB[r * MAX_N + c] = (double)tb[r];
    R u[MAX_N] = {0};
    for (int i = lfd::FR_LS - 1; i >= 0; --i) fc.Rh[i][c] = (double)tdf2_step(cs, u, yv[i]);
    for (int r = 0; r < n; ++r) fc.M32[r * MAX_N + c] = (double)u[r];
  }
  {
    R kaz[16][lfd::FR_LS] = {{0}};
    for (int p = 0; p < lfd::FR_LS; ++p) {
      R z[MAX_N] = {0}, yo[lfd::FR_LS];
      for (int i = 0; i < lfd::FR_LS; ++i) yo[i] = tdf2_step(cs, z, i == p ? 1.0L : 0.0L);
      R t[MAX_N] = {0};
      for (int i = lfd::FR_LS - 1; i >= 0; --i) (void)tdf2_step(cs, t, yo[i]);
      for (int c = 0; c < n; ++c) {
        kaz[c][p] = z[c];
        kaz[n + c][p] = t[c];
      }
    }
    for (int ks = 0; ks < lfd::FR_LS / 4; ++ks)
      for (int l = 0; l < 64; ++l) fc.KAZ[ks][l] = (double)kaz[l & 15][4 * ks + (l >> 4)];
  }
  {
    R kr[lfd::FR_LS][lfd::FR_LS] = {{0}};  // kr[i][p]
    for (int p = 0; p < lfd::FR_LS; ++p) {
      R z[MAX_N] = {0}, yo[lfd::FR_LS];
      for (int i = 0; i < lfd::FR_LS; ++i) yo[i] = tdf2_step(cs, z, i == p ? 1.0L : 0.0L);
      R t[MAX_N] = {0};
      for (int i = lfd::FR_LS - 1; i >= 0; --i) kr[i][p] = tdf2_step(cs, t, yo[i]);
    }
    for (int mt = 0; mt < 2; ++mt)
      for (int ks = 0; ks < lfd::FR_LS / 4; ++ks)
        for (int l = 0; l < 64; ++l) fc.KRA[mt][ks][l] = (double)kr[16 * mt + (l & 15)][4 * ks + (l >> 4)];
  }
  for (int mt = 0; mt < 2; ++mt)
    for (int ks = 0; ks < 4; ++ks)
      for (int l = 0; l < 64; ++l) {
        const int i = 16 * mt + (l & 15), kk = 4 * ks + (l >> 4);
        fc.QA[mt][ks][l] = kk < n ? fc.Rh[i][kk] : (kk < 2 * n ? fc.H[lfd::FR_LS - 1 - i][kk - n] : 0.0);
      }
}

// Taps of the medium-block functionals (lfd_internal.h FR_LB), packed as the
// MFMA kernel's tap table (TapGeom{FR_LB, 0, 2N, 1, 0}):  for a unit sample at
// p, A = the forward exit state after the block = st[LB-1-p] (st[i]: state
// after i + 1 steps of the impulse response h), Z = the zero-state reverse
// exit over the forward output h[i - p] = sum_{i >= p} st[i] h[i - p] (the
// reverse pass runs the same cascade).
std::vector<double> fullrate_medium_taps(const Cascade &cs) {
  const int n = 2 * cs.ns, LB = lfd::FR_LB;
  std::vector<R> h(LB);
  std::vector<std::array<R, MAX_N>> st(LB);
  {
    R z[MAX_N] = {0};
    for (int i = 0; i < LB; ++i) {
      h[i] = tdf2_step(cs, z, i == 0 ? 1.0L : 0.0L);
      for (int c = 0; c < MAX_N; ++c) st[i][c] = z[c];
    }
  }
  std::vector<R> K((size_t)2 * n * LB, 0.0L);  // K[c][p]
  for (int p = 0; p < LB; ++p)
    for (int c = 0; c < n; ++c) {
      K[(size_t)c * LB + p] = st[LB - 1 - p][c];
      R acc = 0;
      for (int i = p; i < LB; ++i) acc += st[i][c] * h[i - p];
      K[(size_t)(n + c) * LB + p] = acc;
    }
  const int nc = 2 * n;
  std::vector<double> dev((size_t)LB * nc, 0.0);
  for (int t = 0; t < LB / 16; ++t)
    for (int q = 0; q < 4; ++q)
      for (int c = 0; c < nc; ++c)
        for (int el = 0; el < 4; ++el)
          dev[((size_t)(t * 4 + q) * nc + c) * 4 + el] = (double)K[(size_t)c * LB + 16 * t + 4 * q + el];
  return dev;
}

// Segment plan of k_fullrate_scan_seg for M medium blocks: G segments of
// seglen blocks (Gu non-empty), PhiB^seglen and PhiB^lastlen in extended
// precision.
// Segments of the full-rate scan: 16 channels x <= 32 segments per
// workgroup, >= 4 medium blocks per segment.  (8 channels x <= 64 segments,
// twice the workgroups for 2,000 channels = 125 groups on 256 CUs, measured
// 0.49 vs 0.48 ms: the diag A/B LFD_FR_SEG_CW=8, profiles/r04s_fr_seg_cw.txt.)
lfd::FRSeg fullrate_segments(const Cascade &cs, int64_t M, int64_t n_ch) {
  lfd::FRSeg sg{};
  const int n = 2 * cs.ns;
  (void)n_ch;
  sg.cw = 16;
  if (const char *v = lfd::knob("LFD_FR_SEG_CW")) sg.cw = std::atoi(v) == 8 ? 8 : 16;  // (diag A/B)
  const int64_t G = std::max<int64_t>(1, std::min<int64_t>(512 / sg.cw, M / 4));
  sg.seglen = (int)((M + G - 1) / G);
  sg.Gu = (int)((M + sg.seglen - 1) / sg.seglen);
  sg.G = (int)G;
  sg.lastlen = (int)(M - (int64_t)(sg.Gu - 1) * sg.seglen);
  Mat P1(n);
  for (int c = 0; c < n; ++c) {
    R z[MAX_N] = {0};
    z[c] = 1;
    (void)tdf2_step(cs, z, 0);
    for (int r = 0; r < n; ++r) P1.a[r][c] = z[r];
  }
  const Mat PB = mpow(P1, lfd::FR_LB);
  const Mat ps = mpow(PB, sg.seglen), pl = mpow(PB, sg.lastlen);
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < n; ++c) {
      sg.pseg[r * MAX_N + c] = (double)ps.a[r][c];
      sg.plast[r * MAX_N + c] = (double)pl.a[r][c];
    }
  return sg;
}

// Fill the block-functional and scan constants for block length L and output
// weight ow (the grid's constant fractional sample position).
int block_constants(const Cascade &cs, int L, R ow, lfd::BlockConst &kc, lfd::ScanConst &sc,
                    bool &fir32) {
  RModel m;
  if (int e = make_rmodel(cs, m)) return e;
  const int n = 2 * m.ns, J = m.J;
  if (L < J + 1 + (ow != 0 ? 1 : 0)) return fail(LFD_EUNSUPPORTED, "block shorter than the FIR span");
  std::memset(&kc, 0, sizeof(kc));
  std::memset(&sc, 0, sizeof(sc));
  lfd::RCoef rc{};
  make_rcoef(m, rc, fir32);
  kc.r = rc;
  sc.r = rc;
  // reverse state-space in T coordinates (T(m) = A T(m+1) + B y)
  Mat A(n), Ai(n);
  R B[MAX_N];
  for (int j = 0; j < n; ++j) {
    R T[MAX_N] = {0};
    T[j] = 1;
    r_allpole(m, T, 0);
    for (int i = 0; i < n; ++i) A.a[i][j] = T[i];
  }
  {
    R T[MAX_N] = {0};
    r_allpole(m, T, 1);
    for (int i = 0; i < n; ++i) B[i] = T[i];
  }
  if (!minv(A, Ai)) return fail(LFD_EUNSUPPORTED, "singular reverse transition");
  const Mat Tm = mpow(A, L - 1);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) kc.T[i * MAX_N + j] = (double)(m.G * Tm.a[i][j]);
  // p0 as a linear function of (u, y0[0..J]) (unscaled v_last inputs):
  // T(0) = Tm u, T(j) = A^{-j} (T(0) - sum_{q<j} A^q B y0[q]),
  // p0 = G * G * sum_{j <= J+1} e_j T(j)[2(ns-1)]  (out_weights)
  R ew[lfd::MAX_J + 2];
  out_weights(m, ow, ew);
  auto p0_of = [&](const R *u, const R *y0) {
    R T0[MAX_N];
    for (int i = 0; i < n; ++i) {
      T0[i] = 0;
      for (int j = 0; j < n; ++j) T0[i] += Tm.a[i][j] * u[j];
    }
    R val = 0;
    for (int j = 0; j <= J + 1; ++j) {
      if (ew[j] == 0) continue;
      R acc[MAX_N];
      for (int i = 0; i < n; ++i) acc[i] = T0[i];
      Mat Aq = Mat::eye(n);
      for (int q = 0; q < j; ++q) {
        for (int i = 0; i < n; ++i) {
          R t = 0;
          for (int l = 0; l < n; ++l) t += Aq.a[i][l] * B[l];
          acc[i] -= t * y0[q];
        }
        Aq = Aq * A;
      }
      const Mat Aij = mpow(Ai, j);
      R tj = 0;
      for (int l = 0; l < n; ++l) tj += Aij.a[2 * (m.ns - 1)][l] * acc[l];
      val += ew[j] * tj;
    }
    return m.G * m.G * val;
  };
  for (int i = 0; i < n; ++i) {
    R u[MAX_N] = {0}, y0[lfd::MAX_J + 1] = {0};
    u[i] = 1;
    kc.cp[i] = (double)p0_of(u, y0);
  }
  for (int q = 0; q <= J; ++q) {
    R u[MAX_N] = {0}, y0[lfd::MAX_J + 1] = {0};
    y0[q] = 1;
    kc.dp[q] = (double)p0_of(u, y0);
  }
  sc.ow = (double)ow;
  // scan matrices
  for (int i = 0; i < n; ++i) {
    R e[MAX_N] = {0};
    e[i] = 1;
    const BlockSim bf = sim_block(m, L, e, nullptr, -1, ow);
    const BlockSim br = sim_block(m, L, nullptr, e, -1, ow);
    for (int r = 0; r < n; ++r) {
      sc.PhiF[r * MAX_N + i] = (double)bf.ef[r];
      sc.M[r * MAX_N + i] = (double)bf.er0[r];
      sc.PhiR[r * MAX_N + i] = (double)br.er0[r];
    }
    sc.G0[i] = (double)bf.p0;
    sc.H0[i] = (double)br.p0;
  }
  for (int q = 0; q < J; ++q) {
    const BlockSim bi = sim_block(m, L, nullptr, nullptr, q, ow);
    for (int r = 0; r < n; ++r) {
      sc.Kc[r * lfd::MAX_J + q] = (double)bi.ef[r];
      sc.Kc[(n + r) * lfd::MAX_J + q] = (double)bi.er0[r];
    }
    sc.Kc[(2 * n) * lfd::MAX_J + q] = (double)bi.p0;
  }
  return LFD_OK;
}

// The 2n+1 block functionals are linear in the block's extended samples
// x[a-J .. a+L-1] (J samples of FIR history): F_c = sum_p Kx[c][p] x[a-J+p].
// Taps are computed in extended precision from impulse responses (O(L)):
//   hS[t], hv[t]  state / v_last output t samples after a unit impulse;
//   e_f  : Kw[i][k]    = hS[L-1-k][i]
//   e_r0 : Kw[n+i][k]  = G sum_t hv[t] hS[k+t][i]                 (adjoint)
//   p0   : Kw[2n][k]   = G^2 sum_t hv[t] z[k+t],  z[m] = sum_j c_j hv[m-j]
// (sum_t hv[t] s[k+t] is the all-pole cascade run backward over s), and
//   Kx[c][p] = sum_j c_j Kw[c][p-J+j].
// The output at offset 1 is the same backward run over z shifted by one
// sample, so the blended output functional (weight ow) runs it over
// (1 - ow) z[k] + ow z[k-1].
// Same definitions as sim_block (impulse at w[k], zero states).
// n_off > 0 (lattice plans, ow = 0): rows 2n + d, d < n_off, are the outputs
// at offset d, the same backward run over z shifted by d samples.
int block_taps(const Cascade &cs, int L, R ow, std::vector<long double> &Kx, int &nc, int &row, int n_off = 0) {
  RModel m;
  if (int e = make_rmodel(cs, m)) return e;
  const int n = 2 * m.ns, J = m.J;
  nc = 2 * n + (n_off > 0 ? n_off : 1);
  row = L + J;
  std::vector<R> hS((size_t)L * n), hv(L), Kw((size_t)nc * L, 0.0L);
  {
    R S[MAX_N] = {0};
    for (int t = 0; t < L; ++t) {
      hv[t] = r_allpole(m, S, t == 0 ? 1.0L : 0.0L);
      for (int i = 0; i < n; ++i) hS[(size_t)t * n + i] = S[i];
    }
  }
  auto backward = [&](const std::vector<R> &s, R scale, R *out) {
    R T[MAX_N] = {0};
    for (int k = L - 1; k >= 0; --k) out[k] = scale * r_allpole(m, T, s[k]);
  };
  std::vector<R> s(L);
  for (int i = 0; i < n; ++i) {
    for (int k = 0; k < L; ++k) Kw[(size_t)i * L + k] = hS[(size_t)(L - 1 - k) * n + i];
    for (int k = 0; k < L; ++k) s[k] = hS[(size_t)k * n + i];
    backward(s, m.G, &Kw[(size_t)(n + i) * L]);
  }
  std::vector<R> z(L);
  for (int k = 0; k < L; ++k) {
    R acc = 0;
    for (int j = 0; j <= J && j <= k; ++j) acc += m.c[j] * hv[k - j];
    z[k] = acc;
  }
  if (n_off > 0) {
    for (int d = 0; d < n_off; ++d) {
      for (int k = 0; k < L; ++k) s[k] = k >= d ? z[k - d] : 0.0L;
      backward(s, m.G * m.G, &Kw[(size_t)(2 * n + d) * L]);
    }
  } else {
    for (int k = 0; k < L; ++k) s[k] = (1.0L - ow) * z[k] + (k >= 1 ? ow * z[k - 1] : 0.0L);
    backward(s, m.G * m.G, &Kw[(size_t)(2 * n) * L]);
  }
  Kx.assign((size_t)nc * row, 0.0L);
  for (int c = 0; c < nc; ++c)
    for (int p = 0; p < row; ++p) {
      R acc = 0;
      for (int j = 0; j <= J; ++j) {
        const int k = p - J + j;
        if (k >= 0 && k < L) acc += m.c[j] * Kw[(size_t)c * L + k];
      }
      Kx[(size_t)c * row + p] = acc;
    }
  return LFD_OK;
}

// Run-mode constants from the scan matrices (row-major 4x4, extended precision).
void run_constants(const lfd::ScanConst &sc, lfd::RunConst &rc) {
  typedef R M4[4][4];
  auto ld = [](const double *src, int stride, M4 &m) {
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) m[i][j] = src[i * stride + j];
  };
  auto mul = [](const M4 &a, const M4 &b, M4 &o) {
    M4 t;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        R acc = 0;
        for (int k = 0; k < 4; ++k) acc += a[i][k] * b[k][j];
        t[i][j] = acc;
      }
    std::memcpy(o, t, sizeof(M4));
  };
  auto st = [](const M4 &m, double *dst) {
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) dst[i * 4 + j] = (double)m[i][j];
  };
  constexpr int RR = lfd::RUN_R;
  M4 PF, PR, Mm;
  ld(sc.PhiF, MAX_N, PF);
  ld(sc.PhiR, MAX_N, PR);
  ld(sc.M, MAX_N, Mm);
  R G0[4], H0[4];
  for (int j = 0; j < 4; ++j) {
    G0[j] = sc.G0[j];
    H0[j] = sc.H0[j];
  }
  std::vector<M4> Fp(RR + 1), Rp(RR + 1), Q(RR);  // PhiF^j, PhiR^j, M PhiF^m
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) Fp[0][i][j] = Rp[0][i][j] = (i == j);
  for (int j = 1; j <= RR; ++j) {
    mul(PF, Fp[j - 1], Fp[j]);
    mul(PR, Rp[j - 1], Rp[j]);
  }
  for (int m = 0; m < RR; ++m) mul(Mm, Fp[m], Q[m]);
  std::memset(&rc, 0, sizeof(rc));
  for (int j = 0; j <= RR; ++j) {
    st(Fp[j], rc.PhiFp[j]);
    st(Rp[j], rc.PhiRp[j]);
    M4 C = {};
    for (int m = 0; m < j; ++m) {  // C[j] = sum_{m<j} PhiR^m M PhiF^m
      M4 t;
      mul(Rp[m], Q[m], t);
      for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) C[a][b] += t[a][b];
    }
    st(C, rc.C[j]);
  }
  for (int d = 0; d < RR; ++d)
    for (int j = 0; j < 4; ++j) {
      R acc = 0;
      for (int i = 0; i < 4; ++i) acc += H0[i] * Rp[d][i][j];
      rc.B[d][j] = (double)acc;
    }
  for (int len = 1; len <= RR; ++len)
    for (int p = 0; p < len; ++p)
      for (int j = 0; j < 4; ++j) {
        R acc = 0;
        for (int i = 0; i < 4; ++i) acc += G0[i] * Fp[p][i][j];
        for (int m = p + 1; m < len; ++m) {
          M4 t;
          mul(Rp[m - p - 1], Q[m], t);
          for (int i = 0; i < 4; ++i) acc += H0[i] * t[i][j];
        }
        rc.A[len][p][j] = (double)acc;
      }
  st(PF, rc.PhiF);
  st(Mm, rc.M);
  st(PR, rc.PhiR);
  for (int j = 0; j < 4; ++j) {
    rc.G0[j] = sc.G0[j];
    rc.H0[j] = sc.H0[j];
  }
}

inline int64_t floor_div(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}
inline int64_t ceil_div(int64_t a, int64_t b) { return -floor_div(-a, b); }
inline size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// Blocks per grid interval for grid spacing Rg: 1 while Rg <= SUB_L_MAX,
// else the smallest divisor m with Rg/m <= SUB_L_MAX, preferring block
// lengths that are multiples of 4 (one 16-B row alignment: a single tap
// table) and never shorter than the FIR span (+1 for an off-sample grid).
// LFD_SUBBLOCK=0 (A/B knob) keeps L = Rg; another value sets SUB_L_MAX.
constexpr int64_t SUB_L_MAX = 504;  // Lp = 512: taps 36.9 KB + 8 run buffers = 2 groups/CU
int64_t sub_block_step(int64_t Rg, int J, bool off_sample) {
  int64_t lmax = SUB_L_MAX;
  if (const char *v = lfd::knob("LFD_SUBBLOCK")) {
    lmax = std::atoll(v);
    if (lmax <= 0) return 1;
  }
  if (Rg <= lmax) return 1;
  const int64_t lmin = std::max<int64_t>(64, J + 1 + (off_sample ? 1 : 0));
  for (int pass = 0; pass < 2; ++pass)
    for (int64_t m = 2; Rg / m >= lmin; ++m)
      if (Rg % m == 0 && Rg / m <= lmax && (pass == 1 || (Rg / m) % 4 == 0)) return m;
  return 1;
}

}  // namespace

struct lfd_lowpass_plan {
  int device = 0;
  int n_sec = 0, padlen = 0;
  int64_t n_ch = 0, n_t = 0, n_grid = 0, n_chunks = 0;
  int64_t kstep = 1;  // blocks per output-grid interval
  double ow = 0.0;    // the grid's fractional sample position
  lfd::BlockGeom bg{};
  lfd::BlockConst kc{};
  lfd::ScanConst sc{};
  bool fir32 = true;
  std::vector<lfd::ChunkGeom> chunks;
  lfd::ChunkGeom *d_chunks = nullptr;
  // block taps for the MFMA block-functional kernel (empty: recurrence kernel)
  std::vector<double> taps;      // natural layout [nc][L+J]
  lfd::TapGeom tg{};
  double *d_taps = nullptr;      // device layout (lfd_internal.h TapGeom)
  lfd::TapGeom tg_tm{};          // (time, channel) rows: one table, row shift 0
  double *d_taps_tm = nullptr;
  // run mode (lfd_internal.h RunConst): run table, K1 units, constants
  bool run_ok = false;       // run table + constants (4th-order cascades)
  bool run_mfma_ok = false;  // taps + 16 run buffers fit LDS: k_block_runs_mfma
  std::vector<int64_t> run_ks;
  std::vector<int> run_len, group_r0;
  lfd::RunConst rc{};
  int64_t n_sr = 0;
  int64_t *d_run_ks = nullptr;
  int *d_run_len = nullptr, *d_group_r0 = nullptr;
  lfd::RunConst *d_rc = nullptr;
  std::vector<int> slot_chunk;    // run slot (chunk-ordered runs) -> its chunk
  int *d_slot_chunk = nullptr;
  // segmented run chains (lfd_internal.h SegGeom): [n_chunks][seg_max]
  std::vector<lfd::SegGeom> segs;
  lfd::SegGeom *d_segs = nullptr;
  int seg_max = 0;
  // the fused one-launch scan (k_scan_fused): [n_chunks][FU_SEG_HOST] segments
  std::vector<lfd::SegGeom> segs_fu;
  lfd::SegGeom *d_segs_fu = nullptr;
  int nw_fu = 0;
  size_t off_SC = 0;
  // lattice one-pass plan (n_off > 0; built by plan_create_composite): the
  // grid is the lattice at its lowest phase, K1 forms the outputs at offsets
  // 0 .. n_off - 1 of every output block (MFMA rows 8 + d), runs start at
  // output blocks; per offset its run constants (G0/H0 of that offset) and
  // chunk output ranges (the points that need that phase)
  int n_off = 0;
  std::vector<lfd::RunConst> rc_off;
  std::vector<lfd::ChunkGeom> chunks_off;  // [n_off][n_chunks]
  lfd::RunConst *d_rc_off = nullptr;
  lfd::ChunkGeom *d_chunks_off = nullptr;
  size_t off_Y0 = 0, off_AG = 0, off_SR = 0, off_TR = 0, off_CR = 0;
  int64_t sf_blocks = 0, tp_len = 0;
  size_t off_F = 0, off_SF = 0, off_TP = 0, ws_bytes = 0;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  // lfd_set_timing(n > 1): a ring of n event triples, so n timed executes
  // need no host synchronisation between them (lfd_lowpass_timings)
  mutable std::vector<hipEvent_t> ring;
  // split executes: the block-pass -> scan-stream events, reused round-robin
  // (a stream wait binds to the record made before it)
  mutable std::vector<hipEvent_t> split_ev;
  mutable size_t split_i = 0;
  mutable std::mutex split_mu;  // (executes of one plan from several host threads)
  mutable int64_t n_exec = 0;
  mutable int last_ring = 0;  // ring size of the last timed execute (0: ev)
  mutable bool timed = false;
  mutable std::atomic<int> last_k1{0};  // (plans may be executed from several host threads)
  mutable std::atomic<int> last_scan{-1};
  // Composite plan (grids that are not one uniform lattice with one fraction
  // w: 3 kHz data on integer-ns times, jittered archives): one uniform,
  // sample-aligned sub-plan per lattice phase d (positions lo0 + j R + d),
  // each writing its lattice outputs into rows [toff, toff + n) of an
  // [n_ch][comp_T] float64 scratch, then k_blend_grid forms
  // y[j] = (1 - w_j) Y_{d_j}[j] + w_j Y_{d_j + 1}[j] (linear interp1d).
  std::vector<lfd_lowpass_plan *> subs;
  std::vector<int64_t> sub_toff;
  int64_t comp_T = 0, n_blend = 0;
  size_t off_tmp = 0;
  int64_t *d_bj = nullptr, *d_bi = nullptr;  // grid index; scratch index of y[lo], y[lo + 1] (-1: w == 0)
  double *d_bw = nullptr;
  // one-pass alternative (channel-major, time-contiguous rows): one lattice plan
  // for every phase (n_off offsets), slot-major scratch [n_off * n_grid][n_ch]
  lfd_lowpass_plan *lat = nullptr;
  int64_t *d_bi_lat = nullptr;
  size_t off_tmp_lat = 0;
  mutable std::atomic<bool> last_onepass{false};
};

extern "C" {

const char *lfd_last_error(void) { return g_err.c_str(); }
int lfd_version(void) { return 200; }  // 2.0: float64 low-pass outputs

int lfd_device_count(int *count) {
  if (!count) return fail(LFD_EINVAL, "count is NULL");
  LFD_HIP(hipGetDeviceCount(count));
  return LFD_OK;
}

int lfd_set_option(int option, int64_t value) {
  if (option <= 0 || option >= N_OPT) return fail(LFD_EINVAL, "unknown option " + std::to_string(option));
  if (value < 0 || (option == LFD_OPT_SCAN_DEFER ? value > 4 : value > 1))
    return fail(LFD_EINVAL, "option " + std::to_string(option) + ": value out of range");
  g_opt[option].store(value);
  g_opt_set[option].store(true);
  return LFD_OK;
}

int lfd_get_option(int option, int64_t *value) {
  if (option <= 0 || option >= N_OPT) return fail(LFD_EINVAL, "unknown option " + std::to_string(option));
  if (!value) return fail(LFD_EINVAL, "value is NULL");
  *value = g_opt[option].load();
  return LFD_OK;
}

int lfd_set_timing(int enable) {
  g_timing.store(enable > 0 ? enable : 0);
  return LFD_OK;
}

static int plan_create_uniform(lfd_lowpass_plan **out, const double *sos, int n_sec,
                               int padlen, int64_t n_ch, int64_t n_t,
                               const int64_t *grid_lo, const double *grid_w,
                               int64_t n_grid, const lfd_chunk *chunks,
                               int64_t n_chunks, int n_off = 0);
static int plan_create_composite(lfd_lowpass_plan **out, const double *sos, int n_sec,
                                 int padlen, int64_t n_ch, int64_t n_t,
                                 const int64_t *grid_lo, const double *grid_w,
                                 int64_t n_grid, const lfd_chunk *chunks,
                                 int64_t n_chunks);

int lfd_lowpass_plan_create(lfd_lowpass_plan **out, const double *sos, int n_sec,
                            int padlen, int64_t n_ch, int64_t n_t,
                            const int64_t *grid_lo, const double *grid_w,
                            int64_t n_grid, const lfd_chunk *chunks,
                            int64_t n_chunks) {
  const int rc = plan_create_uniform(out, sos, n_sec, padlen, n_ch, n_t, grid_lo, grid_w, n_grid, chunks,
                                     n_chunks);
  if (rc != LFD_EUNSUPPORTED || n_grid < 2 || !grid_lo || !grid_w || !chunks || n_chunks < 1) return rc;
  const std::string why = g_err;
  const int rc2 = plan_create_composite(out, sos, n_sec, padlen, n_ch, n_t, grid_lo, grid_w, n_grid, chunks,
                                        n_chunks);
  if (rc2 == LFD_EUNSUPPORTED) return fail(LFD_EUNSUPPORTED, why + "; lattice plan: " + g_err);
  return rc2;
}

static int plan_create_uniform(lfd_lowpass_plan **out, const double *sos, int n_sec,
                               int padlen, int64_t n_ch, int64_t n_t,
                               const int64_t *grid_lo, const double *grid_w,
                               int64_t n_grid, const lfd_chunk *chunks,
                               int64_t n_chunks, int n_off) {
  if (!out) return fail(LFD_EINVAL, "plan out-pointer is NULL");
  *out = nullptr;
  Cascade c;
  if (int e = load_sos(sos, n_sec, c)) return e;
  if (padlen < 0) padlen = default_padlen(c);
  if (n_ch < 1 || n_t < 1) return fail(LFD_EINVAL, "n_ch and n_t must be >= 1");
  if (n_grid < 2 || !grid_lo || !grid_w)
    return fail(LFD_EUNSUPPORTED, "block plan needs a uniform grid of >= 2 points");
  if (n_chunks < 1 || !chunks) return fail(LFD_EINVAL, "no chunks");
  // uniform grid with one fractional position w for every point (an archive
  // whose samples start off the output grid: t0 = 03:00:00.000372 etc.)
  const int64_t Rg = grid_lo[1] - grid_lo[0];
  const double w0 = grid_w[0];
  for (int64_t j = 0; j < n_grid; ++j) {
    if (!(grid_w[j] >= 0.0 && grid_w[j] < 1.0)) return fail(LFD_EINVAL, "grid weights must be in [0, 1)");
    if (grid_w[j] != w0)
      return fail(LFD_EUNSUPPORTED, "grid points at varying positions between samples need the general path");
    if (j > 0 && grid_lo[j] - grid_lo[j - 1] != Rg)
      return fail(LFD_EUNSUPPORTED, "non-uniform grid spacing needs the general path");
  }
  if (Rg < 2 || Rg > (int64_t)1 << 30)
    return fail(LFD_EUNSUPPORTED, "grid spacing must be in [2, 2^30] samples");
  if (n_off > 0 && (n_off > lfd::LAT_MAX_OFF || n_sec != 2 || w0 != 0.0))
    return fail(LFD_EUNSUPPORTED, "lattice one-pass: 2 sections, sample-aligned lattice, <= 8 offsets");
  // Block length L = Rg / kstep: long grid spacings (Rg > 504: dt = 10 s at
  // 200 Hz - 2 kHz, dt = 1 s at 2 kHz) are cut into sub-blocks of <= 504
  // samples so that the MFMA tap table (L * 72 B) + run buffers fit two
  // 512-thread workgroups per CU; outputs sit at every kstep-th block start.
  const int64_t kstep = sub_block_step(Rg, 2 * n_sec, w0 != 0.0);
  const int L = (int)(Rg / kstep);
  if (n_off > 0 && L < n_off + 2 * n_sec + 1) return fail(LFD_EUNSUPPORTED, "lattice one-pass: block too short");
  const int64_t base0 = ((grid_lo[0] % L) + L) % L;

  auto *p = new lfd_lowpass_plan();
  p->n_sec = n_sec;
  p->padlen = padlen;
  p->n_ch = n_ch;
  p->n_t = n_t;
  p->n_grid = n_grid;
  p->n_chunks = n_chunks;
  int64_t kmin = INT64_MAX, kmax = INT64_MIN;
  p->chunks.resize(n_chunks);
  for (int64_t ci = 0; ci < n_chunks; ++ci) {
    const lfd_chunk &ch = chunks[ci];
    lfd::ChunkGeom &G = p->chunks[ci];
    auto bad = [&](int code, const std::string &m) {
      delete p;
      return fail(code, "chunk " + std::to_string(ci) + ": " + m);
    };
    if (ch.s0 < 0 || ch.s1 >= n_t || ch.s1 < ch.s0) return bad(LFD_EINVAL, "sample range outside the array");
    if (ch.s1 - ch.s0 + 1 <= padlen)
      return bad(LFD_EINVAL, "The length of the input vector x must be greater than padlen, which is " +
                                 std::to_string(padlen) + ".");
    if (ch.g0 < 0 || ch.g1 > n_grid || ch.g1 < ch.g0) return bad(LFD_EINVAL, "grid range outside the grid");
    G.s0 = ch.s0;
    G.s1 = ch.s1;
    G.kb = ceil_div(ch.s0 - base0, L);
    G.ke = floor_div(ch.s1 + 1 - base0, L);
    if (G.ke <= G.kb) return bad(LFD_EUNSUPPORTED, "chunk holds no full block");
    G.head_end = base0 + G.kb * L;
    G.tail_begin = base0 + G.ke * L;
    G.tail_out_j = -1;
    G.tail_out_pos = -1;
    G.kout0 = G.kout1 = G.kb;
    G.jout0 = 0;
    G.kstep = kstep;
    // head skip (run mode): the samples of block kb-1 before s0 and its J
    // samples of FIR history all lie in the left pad
    {
      const int64_t nh = G.head_end - G.s0, lo = G.head_end - L, J = 2 * n_sec;
      const int64_t ncorr = G.s0 - lo + J;
      G.hskip = (nh >= J && lo >= 0 && ncorr <= padlen && ncorr <= lfd::HSKIP_MAX &&
                 !lfd::option(LFD_OPT_NO_HEAD_SKIP)) ? 1 : 0;
    }
    bool any_block = false;
    for (int64_t j = ch.g0; j < ch.g1; ++j) {
      const int64_t pos = grid_lo[j];
      if (n_off > 0 && (pos < ch.s0 || pos + n_off - 1 > ch.s1))
        return bad(LFD_EUNSUPPORTED, "lattice one-pass: output offsets outside the chunk");
      if (pos < ch.s0 || pos > ch.s1 || (w0 != 0.0 && pos + 1 > ch.s1))
        return bad(LFD_EINVAL, "output grid point outside the chunk");
      const int64_t kj = (pos - base0) / L;
      if (kj >= G.kb && kj < G.ke) {
        if (!any_block) {
          G.kout0 = kj;
          G.jout0 = j;
          any_block = true;
        }
        G.kout1 = kj + 1;
      } else if (pos < G.head_end) {
        // unreachable: grid points are block starts and blocks start >= s0
        return bad(LFD_EINVAL, "internal: output grid point inside a chunk head");
      } else {
        if (n_off > 0) return bad(LFD_EUNSUPPORTED, "lattice one-pass: an output in a chunk tail");
        G.tail_out_pos = pos;
        G.tail_out_j = j;
      }
    }
    // (one-pass lattice) the output at block kb would need the FIR-history
    // correction of every offset (CR holds offset 0's)
    if (n_off > 0 && any_block && G.kout0 == G.kb)
      return bad(LFD_EUNSUPPORTED, "lattice one-pass: an output in a chunk's first block");
    kmin = std::min(kmin, G.hskip ? G.kb - 1 : G.kb);
    kmax = std::max(kmax, G.ke);
    const int64_t nhead = G.head_end - G.s0, ntail = G.s1 + 1 - G.tail_begin;
    p->tp_len = std::max(p->tp_len, nhead + ntail + padlen);
  }
  // shift block indices so the plan's blocks are [0, nb)
  int64_t sf = 0;
  for (auto &G : p->chunks) {
    G.kb -= kmin;
    G.ke -= kmin;
    G.kout0 -= kmin;
    G.kout1 -= kmin;
    G.sf_off = sf;
    sf += G.ke - G.kb;
  }
  p->sf_blocks = sf;
  const int n = 2 * n_sec;
  p->bg.n_ch = n_ch;
  p->bg.nb = kmax - kmin;
  p->bg.base = base0 + kmin * L;
  p->bg.L = L;
  p->bg.nF = 2 * n + 1;
  p->kstep = kstep;
  p->ow = w0;
  if (int e = block_constants(c, L, (R)w0, p->kc, p->sc, p->fir32)) {
    delete p;
    return e;
  }
  std::vector<long double> Kx;
  int nc = 0, row = 0;
  if (2 * n + (n_off > 0 ? n_off : 1) <= 16) {
    if (int e = block_taps(c, L, (R)w0, Kx, nc, row, n_off)) {
      delete p;
      return e;
    }
    const int J = 2 * n_sec;
    const int nvar = L % 4 == 0 ? 1 : 4;
    const int v0 = (int)(((p->bg.base - J) % 4 + 4) % 4);
    const int Lp = (row + (nvar == 1 ? v0 : 3) + 63) / 64 * 64;
    if ((size_t)Lp * nc * nvar * sizeof(double) <= (size_t)lfd::TAP_LDS_MAX) {
      p->taps.resize(Kx.size());
      for (size_t i = 0; i < Kx.size(); ++i) p->taps[i] = (double)Kx[i];
      p->tg = lfd::TapGeom{Lp, J, nc, nvar, v0};
    }
  }
  if (n_off > 0 && (p->taps.empty() ||
                    sizeof(double) * ((size_t)p->tg.Lp * p->tg.nc * p->tg.nvar + 224) > (size_t)lfd::TAP_LDS_MAX)) {
    delete p;
    return fail(LFD_EUNSUPPORTED, "lattice one-pass: tap table does not fit LDS");
  }
  p->n_off = n_off;
  p->bg.n_sf = p->sf_blocks;
  // run mode: 4th-order cascades.  The MFMA K1 folds runs in registers when
  // its LDS holds the taps + 16 run buffers; otherwise (and for the recurrence
  // K1) k_fold_runs folds the per-block functionals.
  if (n_sec == 2) {
    p->run_mfma_ok = !p->taps.empty() &&
        sizeof(double) * ((size_t)p->tg.Lp * p->tg.nc * p->tg.nvar + 64 + 8 * lfd::RUN_R * 5 * 16) <=
            (size_t)lfd::TAP_LDS_MAX;
    // (time, channel) rows: k_block_runs_mfma_tm reads each block row from
    // its first sample (no 16-B shift): one table, shift 0; its 512-thread
    // workgroup holds 8 waves x 2 channel tiles of run buffers
    if (!p->taps.empty() && n_off == 0) {
      const int row = (int)(p->taps.size() / p->tg.nc);
      const int Lp_tm = (row + 63) / 64 * 64;
      if (sizeof(double) * ((size_t)Lp_tm * p->tg.nc + 64 + 8 * 2 * lfd::RUN_R * 5 * 16) <= (size_t)lfd::TAP_LDS_MAX)
        p->tg_tm = lfd::TapGeom{Lp_tm, p->tg.J, p->tg.nc, 1, 0};
    }
    std::vector<int64_t> cuts = {0, p->bg.nb};
    for (const auto &G : p->chunks) {
      if (G.hskip) cuts.push_back(G.kb - 1);  // block kb-1 alone: E_f = e_f(kb-1)
      cuts.push_back(G.kb);
      if (G.kb + 1 < G.ke) cuts.push_back(G.kb + 1);
      cuts.push_back(G.ke);
      // (one-pass lattice) every output block starts a run: K1 forms y0 of a
      // run's first block only
      if (n_off > 0)
        for (int64_t k = G.kout0; k < G.kout1; k += kstep) cuts.push_back(k);
    }
    std::sort(cuts.begin(), cuts.end());
    cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
    for (size_t i = 0; i + 1 < cuts.size(); ++i)
      for (int64_t a = cuts[i]; a < cuts[i + 1]; a += lfd::RUN_R) {
        p->run_ks.push_back(a);
        p->run_len.push_back((int)std::min<int64_t>(lfd::RUN_R, cuts[i + 1] - a));
      }
    const int64_t n_runs = (int64_t)p->run_ks.size();
    // K1 units: consecutive runs up to 32 blocks (fewer for narrow arrays, so
    // that >= ~4,096 wave units cover the chip)
    // (k_block_runs_mfma holds a unit's run table one run per lane: a unit of
    // <= 32 blocks has <= 32 runs, well inside the 64 lanes)
    // (at least ~16 rounds of units over the 4,096 resident waves: a
    // 1,250-channel shard (8 GPUs) ran its last, partial round of 32-block
    // units 7 % longer than with 16-block ones, tools/ab_plan.py --replan)
    int64_t unit_cap = 32;
    int64_t unit_min = 16;
    if (const char *v = lfd::knob("LFD_RUN_UNIT")) {
      unit_cap = std::min<int64_t>(32, std::max(lfd::RUN_R, std::atoi(v)));
      unit_min = lfd::RUN_R;
    }
    const int64_t blocks_all = ((n_ch + 15) / 16) * p->bg.nb;
    const int64_t unit_blocks =
        blocks_all / 4096 >= 32
            ? std::max<int64_t>(std::min(unit_min, unit_cap), std::min<int64_t>(unit_cap, blocks_all / (16 * 4096)))
            : std::max<int64_t>(lfd::RUN_R, std::min<int64_t>(unit_cap, blocks_all / 4096));
    // Tail: units are dispatched time-group-major (unit = channel group +
    // n_cg x time group), so the last ~2 rounds of units (2 x 4,096 waves)
    // are the last time groups; making those one run long shortens the
    // kernel's drain, where a few waves each stream alone (LFD_RUN_TAIL=0:
    // off)
    const int64_t n_cg = (n_ch + 15) / 16;
    int64_t tail_rounds = 2;  // LFD_RUN_TAIL=<rounds>, 0: off
    if (const char *v = lfd::knob("LFD_RUN_TAIL")) tail_rounds = std::max(0, std::atoi(v));
    const int64_t tail_blocks =
        std::min<int64_t>(p->bg.nb / 4, tail_rounds * ((4096 + n_cg - 1) / n_cg) * lfd::RUN_R);
    const int64_t tail_k = unit_blocks <= lfd::RUN_R ? p->bg.nb : p->bg.nb - tail_blocks;  // runs starting at or after this block
    int acc = 0;
    for (int64_t r = 0; r < n_runs; ++r) {
      const int64_t cap = p->run_ks[r] >= tail_k ? lfd::RUN_R : unit_blocks;
      if (r == 0 || acc + p->run_len[r] > cap || (p->run_ks[r] >= tail_k && acc > 0)) {
        p->group_r0.push_back((int)r);
        acc = 0;
      }
      acc += p->run_len[r];
    }
    p->group_r0.push_back((int)n_runs);
    for (size_t gi = 0; gi + 1 < p->group_r0.size(); ++gi)
      if (p->group_r0[gi + 1] - p->group_r0[gi] > 64) {
        delete p;
        return fail(LFD_EINVAL, "internal: a K1 unit holds more than 64 runs");
      }
    auto run_at = [&](int64_t k) {
      return (int64_t)(std::lower_bound(p->run_ks.begin(), p->run_ks.end(), k) - p->run_ks.begin());
    };
    int64_t sr = 0;
    for (size_t ci = 0; ci < p->chunks.size(); ++ci) {
      auto &G = p->chunks[ci];
      G.r0 = run_at(G.kb);
      G.r1 = run_at(G.ke);
      G.sr_off = sr;
      sr += G.r1 - G.r0;
      p->slot_chunk.insert(p->slot_chunk.end(), (size_t)(G.r1 - G.r0), (int)ci);
    }
    p->n_sr = sr;
    run_constants(p->sc, p->rc);
    for (int i = 0; i < 4; ++i)
      for (int q = 0; q < lfd::HSKIP_MAX; ++q)
        p->rc.KfH[i][q] = (nc > i && q < row) ? (double)Kx[(size_t)i * row + q] : 0.0;
    // segmented chains: each chunk's runs in <= gmax segments of >= min_runs
    // runs; P / Q = PhiF / PhiR to the segment's block count
    {
      Mat PF(4), PR(4);
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
          PF.a[i][j] = p->sc.PhiF[i * MAX_N + j];
          PR.a[i][j] = p->sc.PhiR[i * MAX_N + j];
        }
      auto build_segs = [&](int64_t gmax, int64_t min_runs, std::vector<lfd::SegGeom> &segs) {
        segs.assign((size_t)(n_chunks * gmax), lfd::SegGeom{});
        for (int64_t ci = 0; ci < n_chunks; ++ci) {
          const auto &G = p->chunks[ci];
          const int64_t nr = G.r1 - G.r0;
          const int64_t gc = std::max<int64_t>(1, std::min<int64_t>(gmax, nr / min_runs));
          const int64_t per = (nr + gc - 1) / gc;
          for (int64_t k = 0; k < gmax; ++k) {
            lfd::SegGeom &sgm = segs[(size_t)(ci * gmax + k)];
            sgm.ra = std::min(G.r1, G.r0 + k * per);
            sgm.rb = std::min(G.r1, sgm.ra + per);
            if (k >= gc || sgm.ra >= sgm.rb) {
              sgm.ra = sgm.rb = G.r1;
              continue;
            }
            sgm.last = (k == gc - 1 || G.r0 + (k + 1) * per >= G.r1) ? 1 : 0;
            const int64_t blocks = p->run_ks[sgm.rb - 1] + p->run_len[sgm.rb - 1] - p->run_ks[sgm.ra];
            const Mat Pk = mpow(PF, (int)blocks), Qk = mpow(PR, (int)blocks);
            for (int i = 0; i < 4; ++i)
              for (int j = 0; j < 4; ++j) {
                sgm.P[i * 4 + j] = (double)Pk.a[i][j];
                sgm.Q[i * 4 + j] = (double)Qk.a[i][j];
              }
          }
        }
      };
      // the multi-launch segmented scan (k_seg_fwd / k_seg_bwd)
      int64_t gmax = 1;
      for (const auto &G : p->chunks)
        gmax = std::max<int64_t>(gmax, std::min<int64_t>(lfd::SEG_MAX, (G.r1 - G.r0) / lfd::SEG_MIN_RUNS));
      p->seg_max = (int)gmax;
      build_segs(gmax, lfd::SEG_MIN_RUNS, p->segs);
      // the fused one-launch scan (k_scan_fused): FU_SEG_HOST segments per
      // chunk, each held in registers (<= FU_SEGR_HOST runs)
      int64_t nr_max = 0;
      for (const auto &G : p->chunks) nr_max = std::max<int64_t>(nr_max, G.r1 - G.r0);
      p->nw_fu = nr_max <= (int64_t)lfd::FU_SEG_HOST * lfd::FU_SEGR_HOST ? lfd::FU_SEG_HOST : 0;
      if (p->nw_fu) build_segs(lfd::FU_SEG_HOST, 1, p->segs_fu);
      // the fused scan's right-edge maps: scan_tail (lfd_kernels.hip) on zero
      // samples from S = e_k, in extended precision — the tail's forward walk
      // over its samples and the odd-extension pad, the reverse from the
      // steady state of the last forward output, the tail output (interp1d
      // between two reverse outputs); the device adds its S = 0 walk
      bool tmap_on = p->nw_fu != 0;
      if (const char *v = lfd::knob("LFD_FU_TAILMAP")) tmap_on = tmap_on && std::atoi(v) != 0;
      RModel tm_m;
      if (tmap_on && make_rmodel(c, tm_m) != LFD_OK) tmap_on = false;
      if (tmap_on && tm_m.ns != 2) tmap_on = false;  // (run mode is 4th order)
      for (int64_t ci = 0; tmap_on && ci < n_chunks; ++ci) {
        const auto &G = p->chunks[ci];
        const int J = tm_m.J;
        const int64_t ntp = G.s1 + 1 - G.tail_begin + padlen;
        R TM[4][4] = {}, tmv[4] = {};
        std::vector<R> tp((size_t)ntp);
        for (int k = 0; k < 4; ++k) {
          R S[4] = {0, 0, 0, 0};
          S[k] = 1;
          R ylast = 0;
          for (int64_t i = 0; i < ntp; ++i) tp[(size_t)i] = ylast = tm_m.G * r_allpole(tm_m, S, 0);
          R T[4], v = ylast;
          for (int sct = 0; sct < 2; ++sct) {
            v *= 1.0L / ((1.0L + tm_m.a1[sct]) + tm_m.a2[sct]);
            T[2 * sct] = T[2 * sct + 1] = v;
          }
          R qw[lfd::MAX_J];
          for (int j = 0; j < J; ++j) qw[j] = v;
          R y_next = 0, y_out = 0;
          for (int64_t i = ntp - 1; i >= 0; --i) {
            const R q = r_allpole(tm_m, T, tp[(size_t)i]);
            if (G.tail_out_j >= 0 && (G.tail_begin + i == G.tail_out_pos || G.tail_begin + i == G.tail_out_pos + 1)) {
              R acc = q;
              for (int j = 1; j <= J; ++j) acc += tm_m.c[j] * qw[j - 1];
              acc *= tm_m.G;
              if (G.tail_begin + i == G.tail_out_pos + 1)
                y_next = acc;
              else
                y_out = acc + (R)p->ow * (y_next - acc);
            }
            for (int j = J - 1; j > 0; --j) qw[j] = qw[j - 1];
            qw[0] = q;
          }
          for (int i = 0; i < 4; ++i) TM[i][k] = T[i];
          tmv[k] = y_out;
        }
        for (int sgi = 0; sgi < lfd::FU_SEG_HOST; ++sgi) {
          lfd::SegGeom &sgm = p->segs_fu[(size_t)(ci * lfd::FU_SEG_HOST + sgi)];
          sgm.tmap = 1;
          for (int i = 0; i < 4; ++i) {
            sgm.tm[i] = (double)tmv[i];
            for (int k = 0; k < 4; ++k) sgm.TM[i * 4 + k] = (double)TM[i][k];
          }
        }
      }
    }
    if (n_off > 0) {
      // per offset d: the output's responses to the states (G0_d, H0_d) and
      // the run constants built on them; H0_d also into the K1 constants
      RModel m;
      if (int e = make_rmodel(c, m)) {
        delete p;
        return e;
      }
      p->rc_off.resize(n_off);
      for (int d = 0; d < n_off; ++d) {
        lfd::ScanConst sd = p->sc;
        for (int i = 0; i < n; ++i) {
          R e[MAX_N] = {0};
          e[i] = 1;
          sd.G0[i] = (double)sim_block(m, L, e, nullptr, -1, 0, d).p0;
          sd.H0[i] = (double)sim_block(m, L, nullptr, e, -1, 0, d).p0;
          p->rc.H0L[d][i] = sd.H0[i];
        }
        run_constants(sd, p->rc_off[d]);
        std::memcpy(p->rc_off[d].KfH, p->rc.KfH, sizeof(p->rc.KfH));
      }
      for (int d = 0; d < n_off; ++d) std::memcpy(p->rc_off[d].H0L, p->rc.H0L, sizeof(p->rc.H0L));
    }
    p->run_ok = true;
  }
  // channel-group-major layouts (lfd_internal.h f_index / sf_index): channels
  // padded to 16 (F) and 64 (SF)
  const size_t ch16 = (size_t)((n_ch + 15) / 16) * 16, ch64 = (size_t)((n_ch + 63) / 64) * 64;
  p->off_F = 0;
  p->off_SF = align256(p->off_F + sizeof(double) * (size_t)p->bg.nF * p->bg.nb * ch16);
  size_t end_F = align256(p->off_SF + sizeof(double) * (size_t)p->sf_blocks * n * ch64);
  if (p->run_ok) {  // run-mode buffers alias SF (unused in run mode); F stays for the fold
    p->off_Y0 = p->off_SF;
    p->off_AG = align256(p->off_Y0 + sizeof(double) * (size_t)p->bg.nb * ch16 * std::max(1, n_off));
    p->off_SR = align256(p->off_AG + sizeof(double) * (size_t)p->run_ks.size() * 8 * ch16);
    p->off_TR = align256(p->off_SR + sizeof(double) * (size_t)p->n_sr * 4 * ch64);
    p->off_CR = align256(p->off_TR + sizeof(double) * (size_t)p->n_sr * 4 * ch64);
    p->off_SC = align256(p->off_CR + sizeof(double) * (size_t)n_chunks * ch64);
    end_F = std::max(end_F, align256(p->off_SC + sizeof(double) * (size_t)n_chunks * lfd::SC_N_HOST * ch64));
  }
  p->off_TP = end_F;
  p->ws_bytes = align256(p->off_TP + sizeof(double) * (size_t)p->tp_len * n_chunks * n_ch);
  // Device state.  Without a visible device the plan stays host-only (its
  // geometry and constants can still be inspected); execute then fails.
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    (void)hipGetLastError();
    p->device = -1;
    *out = p;
    return LFD_OK;
  }
  hipError_t e = hipGetDevice(&p->device);
  if (e == hipSuccess) e = hipMalloc(&p->d_chunks, sizeof(lfd::ChunkGeom) * n_chunks);
  if (e == hipSuccess)
    e = hipMemcpy(p->d_chunks, p->chunks.data(), sizeof(lfd::ChunkGeom) * n_chunks,
                  hipMemcpyHostToDevice);
  // device layout (lfd_internal.h TapGeom): one table per row shift v
  auto upload_taps = [&](const lfd::TapGeom &tg, double **dst) {
    const int row = (int)(p->taps.size() / tg.nc);
    const size_t tab = (size_t)tg.Lp * tg.nc;
    std::vector<double> dev(tab * tg.nvar, 0.0);
    for (int vi = 0; vi < tg.nvar; ++vi) {
      const int v = tg.nvar == 1 ? tg.v0 : vi;
      for (int t = 0; t < tg.Lp / 16; ++t)
        for (int q = 0; q < 4; ++q)
          for (int cc = 0; cc < tg.nc; ++cc)
            for (int el = 0; el < 4; ++el) {
              const int pos = 16 * t + 4 * q + el - v;
              if (pos >= 0 && pos < row)
                dev[vi * tab + ((size_t)(t * 4 + q) * tg.nc + cc) * 4 + el] =
                    p->taps[(size_t)cc * row + pos];
            }
    }
    hipError_t e2 = hipMalloc(dst, dev.size() * sizeof(double));
    if (e2 == hipSuccess)
      e2 = hipMemcpy(*dst, dev.data(), dev.size() * sizeof(double), hipMemcpyHostToDevice);
    return e2;
  };
  if (e == hipSuccess && !p->taps.empty()) e = upload_taps(p->tg, &p->d_taps);
  if (e == hipSuccess && p->tg_tm.Lp > 0) e = upload_taps(p->tg_tm, &p->d_taps_tm);
  if (e == hipSuccess && p->run_ok) {
    e = hipMalloc(&p->d_run_ks, sizeof(int64_t) * p->run_ks.size());
    if (e == hipSuccess) e = hipMalloc(&p->d_run_len, sizeof(int) * p->run_len.size());
    if (e == hipSuccess) e = hipMalloc(&p->d_group_r0, sizeof(int) * p->group_r0.size());
    if (e == hipSuccess) e = hipMalloc(&p->d_rc, sizeof(lfd::RunConst));
    if (e == hipSuccess)
      e = hipMemcpy(p->d_run_ks, p->run_ks.data(), sizeof(int64_t) * p->run_ks.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(p->d_run_len, p->run_len.data(), sizeof(int) * p->run_len.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(p->d_group_r0, p->group_r0.data(), sizeof(int) * p->group_r0.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_rc, &p->rc, sizeof(lfd::RunConst), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&p->d_slot_chunk, sizeof(int) * std::max<size_t>(1, p->slot_chunk.size()));
    if (e == hipSuccess && !p->slot_chunk.empty())
      e = hipMemcpy(p->d_slot_chunk, p->slot_chunk.data(), sizeof(int) * p->slot_chunk.size(),
                    hipMemcpyHostToDevice);
    if (e == hipSuccess && !p->segs.empty()) {
      e = hipMalloc(&p->d_segs, sizeof(lfd::SegGeom) * p->segs.size());
      if (e == hipSuccess)
        e = hipMemcpy(p->d_segs, p->segs.data(), sizeof(lfd::SegGeom) * p->segs.size(), hipMemcpyHostToDevice);
    }
    if (e == hipSuccess && !p->segs_fu.empty()) {
      e = hipMalloc(&p->d_segs_fu, sizeof(lfd::SegGeom) * p->segs_fu.size());
      if (e == hipSuccess)
        e = hipMemcpy(p->d_segs_fu, p->segs_fu.data(), sizeof(lfd::SegGeom) * p->segs_fu.size(),
                      hipMemcpyHostToDevice);
    }
    if (e == hipSuccess && n_off > 0) {
      e = hipMalloc(&p->d_rc_off, sizeof(lfd::RunConst) * n_off);
      if (e == hipSuccess)
        e = hipMemcpy(p->d_rc_off, p->rc_off.data(), sizeof(lfd::RunConst) * n_off, hipMemcpyHostToDevice);
    }
  }
  for (int i = 0; i < 3 && e == hipSuccess; ++i) e = hipEventCreate(&p->ev[i]);
  if (e != hipSuccess) {
    lfd_lowpass_plan_destroy(p);
    return fail(LFD_EHIP, std::string("plan allocation: ") + hipGetErrorString(e));
  }
  *out = p;
  return LFD_OK;
}

// Lattice decomposition of a general grid (see lfd_lowpass_plan::subs):
// nominal spacing R = round((lo_last - lo_0) / (n - 1)), phase of point j
// d_j = lo_j - (lo_0 + j R); point j needs phase d_j (y[lo_j]) and, when
// w_j > 0, phase d_j + 1 (y[lo_j + 1]).  Every phase is a uniform,
// sample-aligned grid, so each sub-plan is an ordinary block plan over the
// original chunks (each chunk filtered with its own edges, as the reference
// filters each chunk); only the lattice points a chunk needs are put in its
// grid range.  At most LATTICE_MAX phases (3 kHz data with integer-ns times
// drift one sample per ~333 s at dt = 1 s).
static int plan_create_composite(lfd_lowpass_plan **out, const double *sos, int n_sec,
                                 int padlen, int64_t n_ch, int64_t n_t,
                                 const int64_t *lo, const double *w,
                                 int64_t n, const lfd_chunk *chunks,
                                 int64_t n_chunks) {
  constexpr int LATTICE_MAX = 32;
  if (lfd::option(LFD_OPT_NO_LATTICE)) return fail(LFD_EUNSUPPORTED, "disabled (LFD_OPT_NO_LATTICE)");
  for (int64_t j = 0; j < n; ++j) {
    if (!(w[j] >= 0.0 && w[j] < 1.0)) return fail(LFD_EINVAL, "grid weights must be in [0, 1)");
    if (j > 0 && lo[j] + w[j] <= lo[j - 1] + w[j - 1]) return fail(LFD_EUNSUPPORTED, "grid not increasing");
  }
  const int64_t R = (int64_t)std::llround((double)(lo[n - 1] - lo[0]) / (double)(n - 1));
  if (R < 2) return fail(LFD_EUNSUPPORTED, "grid spacing below 2 samples");
  auto phase = [&](int64_t j) { return lo[j] - (lo[0] + j * R); };
  // phase -> [j_first, j_last] over the points the chunks need
  std::vector<std::pair<int64_t, std::pair<int64_t, int64_t>>> ph;
  auto need = [&](int64_t d, int64_t j) {
    for (auto &e : ph)
      if (e.first == d) {
        e.second.first = std::min(e.second.first, j);
        e.second.second = std::max(e.second.second, j);
        return;
      }
    ph.push_back({d, {j, j}});
  };
  for (int64_t c = 0; c < n_chunks; ++c) {
    if (chunks[c].g0 < 0 || chunks[c].g1 > n || chunks[c].g1 < chunks[c].g0)
      return fail(LFD_EINVAL, "chunk " + std::to_string(c) + ": grid range outside the grid");
    for (int64_t j = chunks[c].g0; j < chunks[c].g1; ++j) {
      need(phase(j), j);
      if (w[j] != 0.0) need(phase(j) + 1, j);
      if ((int)ph.size() > LATTICE_MAX) return fail(LFD_EUNSUPPORTED, "more than 32 lattice phases");
    }
  }
  if (ph.empty()) return fail(LFD_EUNSUPPORTED, "no output points");
  // every phase re-runs K1 over its chunks: only grids with few phases per
  // point (slow drift) pay off against the per-chunk general path
  int64_t n_pts = 0;
  for (int64_t c = 0; c < n_chunks; ++c) n_pts += chunks[c].g1 - chunks[c].g0;
  if ((int64_t)ph.size() * 8 > n_pts + 16)
    return fail(LFD_EUNSUPPORTED, std::to_string(ph.size()) + " lattice phases for " + std::to_string(n_pts) +
                                      " points");
  std::sort(ph.begin(), ph.end());
  auto *p = new lfd_lowpass_plan();
  p->n_sec = n_sec;
  p->n_ch = n_ch;
  p->n_t = n_t;
  p->n_grid = n;
  p->n_chunks = n_chunks;
  auto bad = [&](int code) {
    lfd_lowpass_plan_destroy(p);
    return code;
  };
  size_t ws_max = 256;
  std::vector<int64_t> jfirst;
  for (const auto &e : ph) {
    const int64_t d = e.first, j0 = e.second.first;
    const int64_t j1 = std::max(e.second.second, j0 + 1);  // a lattice of >= 2 points
    std::vector<int64_t> sl((size_t)(j1 - j0 + 1));
    for (int64_t i = 0; i <= j1 - j0; ++i) sl[i] = lo[0] + (j0 + i) * R + d;
    std::vector<double> sw(sl.size(), 0.0);
    std::vector<lfd_chunk> sc;
    for (int64_t c = 0; c < n_chunks; ++c) {
      int64_t a = INT64_MAX, b = INT64_MIN;
      for (int64_t j = chunks[c].g0; j < chunks[c].g1; ++j)
        if (phase(j) == d || (w[j] != 0.0 && phase(j) + 1 == d)) {
          a = std::min(a, j);
          b = std::max(b, j);
        }
      if (a <= b) sc.push_back(lfd_chunk{chunks[c].s0, chunks[c].s1, a - j0, b + 1 - j0});
    }
    lfd_lowpass_plan *sub = nullptr;
    const int rc = plan_create_uniform(&sub, sos, n_sec, padlen, n_ch, n_t, sl.data(), sw.data(),
                                       (int64_t)sl.size(), sc.data(), (int64_t)sc.size());
    if (rc != LFD_OK) {
      // (a phase the block plan cannot take: the caller's per-chunk general
      // path reports any real error of the grid)
      const std::string m = g_err;
      bad(rc);
      return fail(rc == LFD_EHIP ? rc : LFD_EUNSUPPORTED, "phase " + std::to_string(d) + ": " + m);
    }
    p->subs.push_back(sub);
    p->sub_toff.push_back(p->comp_T);
    jfirst.push_back(j0);
    p->comp_T += (int64_t)sl.size();
    ws_max = std::max(ws_max, sub->ws_bytes);
  }
  p->padlen = p->subs[0]->padlen;
  p->bg = p->subs[0]->bg;
  // blend map over the chunks' output points
  auto slot = [&](int64_t d, int64_t j) -> int64_t {
    for (size_t i = 0; i < ph.size(); ++i)
      if (ph[i].first == d) return p->sub_toff[i] + (j - jfirst[i]);
    return -1;
  };
  std::vector<int64_t> bj, bi;
  std::vector<double> bw;
  for (int64_t c = 0; c < n_chunks; ++c)
    for (int64_t j = chunks[c].g0; j < chunks[c].g1; ++j) {
      bj.push_back(j);
      bi.push_back(slot(phase(j), j));
      bi.push_back(w[j] != 0.0 ? slot(phase(j) + 1, j) : -1);
      bw.push_back(w[j]);
    }
  p->n_blend = (int64_t)bj.size();
  // one-pass alternative: every phase from one K1 pass (MFMA rows 8 + d are
  // the outputs at offset d from the lowest phase's lattice point, d < 8);
  // when it does not apply (more than 8 phases, points at chunk edges,
  // another cascade order) the per-phase sub-plans above run
  std::vector<int64_t> bi_lat;
  const int64_t dmin = ph.front().first, n_off = ph.back().first - dmin + 1;
  if (n_off <= lfd::LAT_MAX_OFF && n_sec == 2 && !lfd::option(LFD_OPT_LATTICE_PHASES)) {
    std::vector<int64_t> pos((size_t)n);
    for (int64_t j = 0; j < n; ++j) pos[j] = lo[0] + j * R + dmin;
    std::vector<double> zw((size_t)n, 0.0);
    lfd_lowpass_plan *lat = nullptr;
    const std::string err_keep = g_err;
    if (plan_create_uniform(&lat, sos, n_sec, padlen, n_ch, n_t, pos.data(), zw.data(), n, chunks, n_chunks,
                            (int)n_off) == LFD_OK) {
      lat->chunks_off.resize((size_t)(n_off * n_chunks));
      for (int64_t o = 0; o < n_off; ++o)
        for (int64_t c = 0; c < n_chunks; ++c) {
          const lfd::ChunkGeom &B = lat->chunks[c];
          lfd::ChunkGeom G = B;
          G.tail_out_j = -1;
          G.tail_out_pos = -1;
          int64_t a = INT64_MAX, b = INT64_MIN;
          for (int64_t j = chunks[c].g0; j < chunks[c].g1; ++j)
            if (phase(j) == dmin + o || (w[j] != 0.0 && phase(j) + 1 == dmin + o)) {
              a = std::min(a, j);
              b = std::max(b, j);
            }
          if (a <= b) {
            G.kout0 = B.kout0 + (a - B.jout0) * B.kstep;
            G.kout1 = B.kout0 + (b - B.jout0) * B.kstep + 1;
            G.jout0 = a;
          } else {
            G.kout0 = G.kout1 = G.kb;
            G.jout0 = 0;
          }
          lat->chunks_off[o * n_chunks + c] = G;
        }
      for (int64_t c = 0; c < n_chunks; ++c)
        for (int64_t j = chunks[c].g0; j < chunks[c].g1; ++j) {
          bi_lat.push_back((phase(j) - dmin) * n + j);
          bi_lat.push_back(w[j] != 0.0 ? (phase(j) + 1 - dmin) * n + j : -1);
        }
      p->lat = lat;
      ws_max = std::max(ws_max, lat->ws_bytes);
    }
    g_err = err_keep;
  }
  p->off_tmp = align256(ws_max);
  p->ws_bytes = align256(p->off_tmp + sizeof(double) * (size_t)n_ch *
                                          (size_t)std::max(p->comp_T, p->lat ? n_off * n : (int64_t)0));
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    (void)hipGetLastError();
    p->device = -1;
    *out = p;
    return LFD_OK;
  }
  hipError_t e = hipGetDevice(&p->device);
  if (e == hipSuccess) e = hipMalloc(&p->d_bj, sizeof(int64_t) * std::max<size_t>(1, bj.size()));
  if (e == hipSuccess) e = hipMalloc(&p->d_bi, sizeof(int64_t) * std::max<size_t>(1, bi.size()));
  if (e == hipSuccess) e = hipMalloc(&p->d_bw, sizeof(double) * std::max<size_t>(1, bw.size()));
  if (e == hipSuccess && !bj.empty()) e = hipMemcpy(p->d_bj, bj.data(), sizeof(int64_t) * bj.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess && !bi.empty()) e = hipMemcpy(p->d_bi, bi.data(), sizeof(int64_t) * bi.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess && !bw.empty()) e = hipMemcpy(p->d_bw, bw.data(), sizeof(double) * bw.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess && p->lat) {
    lfd_lowpass_plan *lat = p->lat;
    e = hipMalloc(&p->d_bi_lat, sizeof(int64_t) * std::max<size_t>(1, bi_lat.size()));
    if (e == hipSuccess && !bi_lat.empty())
      e = hipMemcpy(p->d_bi_lat, bi_lat.data(), sizeof(int64_t) * bi_lat.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&lat->d_chunks_off, sizeof(lfd::ChunkGeom) * lat->chunks_off.size());
    if (e == hipSuccess)
      e = hipMemcpy(lat->d_chunks_off, lat->chunks_off.data(), sizeof(lfd::ChunkGeom) * lat->chunks_off.size(),
                    hipMemcpyHostToDevice);
  }
  for (int i = 0; i < 3 && e == hipSuccess; ++i) e = hipEventCreate(&p->ev[i]);
  // (the sub-plans hold the chunk tables; d_chunks marks the plan executable)
  if (e == hipSuccess) e = hipMalloc(&p->d_chunks, sizeof(lfd::ChunkGeom));
  if (e != hipSuccess) {
    bad(LFD_EHIP);
    return fail(LFD_EHIP, std::string("plan allocation: ") + hipGetErrorString(e));
  }
  *out = p;
  return LFD_OK;
}

int lfd_lowpass_plan_info(const lfd_lowpass_plan *p, size_t *ws, int64_t *nb, int64_t *L) {
  if (!p) return fail(LFD_EINVAL, "plan is NULL");
  if (ws) *ws = p->ws_bytes;
  if (nb) *nb = p->bg.nb;
  if (L) *L = p->bg.L;
  return LFD_OK;
}

int lfd_lowpass_execute(const lfd_lowpass_plan *p, const float *x, int64_t s_ch,
                        int64_t s_t, double *y, int64_t ys_ch, int64_t ys_t,
                        void *workspace, void *stream) {
  return lfd::lowpass_execute_gen(p, x, s_ch, s_t, y, ys_ch, ys_t, workspace, stream, lfd::GridGen{});
}

int lfd_lowpass_execute_split(const lfd_lowpass_plan *p, const float *x, int64_t s_ch, int64_t s_t, double *y,
                              int64_t ys_ch, int64_t ys_t, void *workspace, void *block_stream, void *scan_stream) {
  if (!scan_stream) return fail(LFD_EINVAL, "scan_stream is NULL");
  return lfd::lowpass_execute_gen(p, x, s_ch, s_t, y, ys_ch, ys_t, workspace, block_stream, lfd::GridGen{},
                                  scan_stream == block_stream ? nullptr : scan_stream);
}
}  // extern "C"

namespace {
// `to` waits for the work enqueued so far on `from` (one of the plan's split
// events; a stream wait binds to the record made before it, so the event can
// be recorded again by a later execute)
hipError_t stream_after(const lfd_lowpass_plan *p, hipStream_t to, hipStream_t from) {
  constexpr size_t N_SPLIT_EV = 8;
  std::lock_guard<std::mutex> lk(p->split_mu);
  if (p->split_ev.size() < N_SPLIT_EV) {
    hipEvent_t e = nullptr;
    const hipError_t rc = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (rc != hipSuccess) return rc;
    p->split_ev.push_back(e);
  }
  hipEvent_t e = p->split_ev[p->split_i++ % p->split_ev.size()];
  hipError_t rc = hipEventRecord(e, from);
  if (rc == hipSuccess) rc = hipStreamWaitEvent(to, e, 0);
  return rc;
}
}  // namespace

int lfd::lowpass_execute_gen(const lfd_lowpass_plan *p, const float *x, int64_t s_ch, int64_t s_t, double *y,
                             int64_t ys_ch, int64_t ys_t, void *workspace, void *stream, const lfd::GridGen &gen,
                             void *scan_stream) {
  if (!p) return fail(LFD_EINVAL, "plan is NULL");
  if (!x || !y || !workspace) return fail(LFD_EINVAL, "x, y and workspace must be device pointers");
  if (s_t == 0 || (p->n_ch > 1 && s_ch == 0)) return fail(LFD_EINVAL, "zero stride");
  if (p->device < 0 || !p->d_chunks) return fail(LFD_EINVAL, "plan has no device state (created without a GPU)");
  int dev = -1;
  LFD_HIP(hipGetDevice(&dev));
  if (dev != p->device) return fail(LFD_EINVAL, "plan was created on another device");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // the scan's stream: `st`, or (split execute) scan_stream after the block pass
  hipStream_t st2 = scan_stream ? reinterpret_cast<hipStream_t>(scan_stream) : st;
  char *ws = static_cast<char *>(workspace);
  int scan_used = -1;
  double *F = reinterpret_cast<double *>(ws + p->off_F);
  double *SF = reinterpret_cast<double *>(ws + p->off_SF);
  double *TP = reinterpret_cast<double *>(ws + p->off_TP);
  const int ring_n = g_timing.load();
  const bool timed = ring_n != 0;
  p->timed = timed;
  hipEvent_t *ev = const_cast<hipEvent_t *>(p->ev);
  if (timed) {
    if (ring_n > 1) {
      if ((int)p->ring.size() < 3 * ring_n) {
        for (int i = (int)p->ring.size(); i < 3 * ring_n; ++i) {
          hipEvent_t e = nullptr;
          LFD_HIP(hipEventCreate(&e));
          p->ring.push_back(e);
        }
      }
      ev = p->ring.data() + 3 * (p->n_exec % ring_n);
    }
    ++p->n_exec;
    p->last_ring = ring_n > 1 ? ring_n : 0;
    LFD_HIP(hipEventRecord(ev[0], st));
  }
  if (!p->subs.empty()) {
    double *tmp = reinterpret_cast<double *>(ws + p->off_tmp);
    const lfd_lowpass_plan *L = p->lat;
    p->last_onepass = L && s_t == 1 && (reinterpret_cast<uintptr_t>(x) & 3) == 0 &&
                      !lfd::option(LFD_OPT_LATTICE_PHASES);
    if (p->last_onepass) {
      // one pass: K1 with every phase's outputs (ev[0] .. ev[1]), then the
      // state scan, the outputs per offset and the blend (ev[1] .. ev[2])
      const lfd::RunGeom rg{(int64_t)L->run_ks.size(), (int64_t)L->group_r0.size() - 1, L->n_sr,
                            L->d_run_ks, L->d_run_len, L->d_group_r0, L->d_rc};
      double *Y0 = reinterpret_cast<double *>(ws + L->off_Y0);
      double *AG = reinterpret_cast<double *>(ws + L->off_AG);
      LFD_HIP(lfd::launch_block_runs_mfma_lat(x, s_ch, L->n_t, L->bg, L->d_taps, L->tg, rg, Y0, AG, st));
      if (timed) LFD_HIP(hipEventRecord(ev[1], st));
      const int64_t n_g = p->n_grid;
      LFD_HIP(lfd::launch_lattice_scan(x, s_ch, s_t, L->bg, L->padlen, L->sc, rg, L->d_chunks, L->n_chunks, Y0, AG,
                                       reinterpret_cast<double *>(ws + L->off_SR),
                                       reinterpret_cast<double *>(ws + L->off_TP), L->tp_len,
                                       reinterpret_cast<double *>(ws + L->off_TR),
                                       reinterpret_cast<double *>(ws + L->off_CR), L->d_slot_chunk, L->n_off,
                                       L->d_rc_off, L->d_chunks_off, tmp, L->n_off * n_g, n_g, st, L->d_segs,
                                       L->seg_max, reinterpret_cast<double *>(ws + L->off_SC), &scan_used));
      p->last_scan = scan_used;
      LFD_HIP(lfd::launch_blend_grid_sm(tmp, p->n_ch, p->d_bj, p->d_bi_lat, p->d_bw, p->n_blend, y, ys_ch, ys_t, st,
                                        gen));
      if (timed) LFD_HIP(hipEventRecord(ev[2], st));
      if (st2 != st) LFD_HIP(stream_after(p, st2, st));
      p->last_k1 = LFD_K1_MFMA_RUNS;
      return LFD_OK;
    }
    // per-phase sub-plans into the scratch (ev[0] .. ev[1]), then the blend
    // (ev[1] .. ev[2])
    for (size_t i = 0; i < p->subs.size(); ++i) {
      const int rc = lfd_lowpass_execute(p->subs[i], x, s_ch, s_t, tmp + p->sub_toff[i], p->comp_T, 1, workspace,
                                         stream);
      if (rc != LFD_OK) return rc;
    }
    if (timed) LFD_HIP(hipEventRecord(ev[1], st));
    LFD_HIP(lfd::launch_blend_grid(tmp, p->comp_T, p->n_ch, p->d_bj, p->d_bi, p->d_bw, p->n_blend, y, ys_ch,
                                   ys_t, st, gen));
    if (timed) LFD_HIP(hipEventRecord(ev[2], st));
    if (st2 != st) LFD_HIP(stream_after(p, st2, st));
    p->last_k1 = p->subs[0]->last_k1.load();
    p->last_scan = p->subs[0]->last_scan.load();
    return LFD_OK;
  }
  // K1: fp64-MFMA block taps when the layout allows, else the recurrence
  const bool rec = lfd::option(LFD_OPT_K1_RECURRENCE) != 0;
  // (any row stride: the MFMA kernels load 4-B aligned 16-B pieces)
  const bool mfma = p->d_taps && s_t == 1 && (reinterpret_cast<uintptr_t>(x) & 3) == 0 && !rec;
  const bool runs = p->run_ok && !lfd::option(LFD_OPT_NO_RUNS);
  const bool mfma_runs = runs && mfma && p->run_mfma_ok;
  // (time, channel) rows (the real files' layout): the time-major MFMA kernel
  const bool mfma_tm = runs && !mfma && p->d_taps_tm && (s_ch == 1 || p->n_ch == 1) && s_t > 1 &&
                       s_t >= p->n_ch && !rec;
  p->last_k1 = mfma_runs ? LFD_K1_MFMA_RUNS
               : mfma_tm ? LFD_K1_MFMA_RUNS_TM
               : runs    ? (mfma ? LFD_K1_MFMA_FOLD : LFD_K1_RECURRENCE_FOLD)
                         : (mfma ? LFD_K1_MFMA : LFD_K1_RECURRENCE);
  if (runs) {
    const lfd::RunGeom rg{(int64_t)p->run_ks.size(), (int64_t)p->group_r0.size() - 1, p->n_sr,
                          p->d_run_ks, p->d_run_len, p->d_group_r0, p->d_rc};
    double *Y0 = reinterpret_cast<double *>(ws + p->off_Y0);
    double *AG = reinterpret_cast<double *>(ws + p->off_AG);
    double *SR = reinterpret_cast<double *>(ws + p->off_SR);
    if (mfma_runs) {
      LFD_HIP(lfd::launch_block_runs_mfma(x, s_ch, p->n_t, p->bg, p->d_taps, p->tg, rg, Y0, AG, st));
    } else if (mfma_tm) {
      LFD_HIP(lfd::launch_block_runs_mfma_tm(x, s_t, p->n_t, p->bg, p->d_taps_tm, p->tg_tm, rg, Y0, AG, st));
    } else {
      if (mfma)
        LFD_HIP(lfd::launch_block_functionals_mfma(x, s_ch, p->n_t, p->bg, p->d_taps, p->tg, F, st));
      else
        LFD_HIP(lfd::launch_block_functionals(p->n_sec, p->fir32, x, s_ch, s_t, p->bg, p->kc, F, st));
      LFD_HIP(lfd::launch_fold_runs(F, p->bg, rg, Y0, AG, st));
    }
    if (timed) LFD_HIP(hipEventRecord(ev[1], st));
    if (st2 != st) LFD_HIP(stream_after(p, st2, st));
    LFD_HIP(lfd::launch_chunk_scan_runs(x, s_ch, s_t, p->bg, p->padlen, p->sc, rg, p->d_chunks, p->n_chunks, Y0,
                                        AG, SR, TP, p->tp_len, y, ys_ch, ys_t, st2,
                                        reinterpret_cast<double *>(ws + p->off_TR),
                                        reinterpret_cast<double *>(ws + p->off_CR), p->d_slot_chunk, p->d_segs,
                                        p->seg_max, reinterpret_cast<double *>(ws + p->off_SC), p->d_segs_fu,
                                        p->nw_fu, &scan_used));
    p->last_scan = scan_used;
    if (timed) LFD_HIP(hipEventRecord(ev[2], st2));
    return LFD_OK;
  }
  if (mfma)
    LFD_HIP(lfd::launch_block_functionals_mfma(x, s_ch, p->n_t, p->bg, p->d_taps, p->tg, F, st));
  else
    LFD_HIP(lfd::launch_block_functionals(p->n_sec, p->fir32, x, s_ch, s_t, p->bg, p->kc, F, st));
  if (timed) LFD_HIP(hipEventRecord(ev[1], st));
  if (st2 != st) LFD_HIP(stream_after(p, st2, st));
  LFD_HIP(lfd::launch_chunk_scan(p->n_sec, p->fir32, x, s_ch, s_t, p->bg, p->padlen, p->sc, p->d_chunks,
                                 p->n_chunks, F, SF, TP, p->tp_len, y, ys_ch, ys_t, st2));
  p->last_scan = LFD_SCAN_BLOCKS;
  if (timed) LFD_HIP(hipEventRecord(ev[2], st2));
  return LFD_OK;
}

extern "C" {
int lfd_lowpass_last_timing(const lfd_lowpass_plan *p, float *ms_blocks, float *ms_scan) {
  if (!p) return fail(LFD_EINVAL, "plan is NULL");
  if (!p->timed) return fail(LFD_EINVAL, "timing was not enabled for the last execute");
  hipEvent_t *ev = p->last_ring > 1 ? p->ring.data() + 3 * ((p->n_exec - 1) % p->last_ring)
                                    : const_cast<hipEvent_t *>(p->ev);
  LFD_HIP(hipEventSynchronize(ev[2]));
  float a = 0, b = 0;
  LFD_HIP(hipEventElapsedTime(&a, ev[0], ev[1]));
  LFD_HIP(hipEventElapsedTime(&b, ev[1], ev[2]));
  if (ms_blocks) *ms_blocks = a;
  if (ms_scan) *ms_scan = b;
  return LFD_OK;
}

int lfd_lowpass_timings(const lfd_lowpass_plan *p, float *ms_blocks, float *ms_scan, int64_t n) {
  if (!p) return fail(LFD_EINVAL, "plan is NULL");
  if (!p->timed || p->last_ring < 2) return fail(LFD_EINVAL, "the last execute was not timed with a ring (lfd_set_timing(n > 1))");
  if (n < 1 || n > p->last_ring || n > p->n_exec) return fail(LFD_EINVAL, "n must be in [1, ring size] and <= timed executes");
  LFD_HIP(hipEventSynchronize(p->ring[3 * ((p->n_exec - 1) % p->last_ring) + 2]));
  for (int64_t i = 0; i < n; ++i) {
    const hipEvent_t *ev = p->ring.data() + 3 * ((p->n_exec - n + i) % p->last_ring);
    float a = 0, b = 0;
    LFD_HIP(hipEventElapsedTime(&a, ev[0], ev[1]));
    LFD_HIP(hipEventElapsedTime(&b, ev[1], ev[2]));
    if (ms_blocks) ms_blocks[i] = a;
    if (ms_scan) ms_scan[i] = b;
  }
  return LFD_OK;
}

int lfd_debug_plan_constants(const lfd_lowpass_plan *p, void *block_const, size_t bc_bytes,
                             void *scan_const, size_t sc_bytes, void *chunk_geom,
                             size_t cg_bytes) {
  if (!p) return fail(LFD_EINVAL, "plan is NULL");
  if (!p->subs.empty()) return fail(LFD_EUNSUPPORTED, "lattice (composite) plan: see its sub-plans");
  if (bc_bytes != sizeof(lfd::BlockConst) || sc_bytes != sizeof(lfd::ScanConst) ||
      cg_bytes != sizeof(lfd::ChunkGeom) * p->chunks.size())
    return fail(LFD_EINVAL, "size mismatch: BlockConst " + std::to_string(sizeof(lfd::BlockConst)) +
                                " ScanConst " + std::to_string(sizeof(lfd::ScanConst)) +
                                " ChunkGeom " + std::to_string(sizeof(lfd::ChunkGeom)));
  std::memcpy(block_const, &p->kc, bc_bytes);
  std::memcpy(scan_const, &p->sc, sc_bytes);
  std::memcpy(chunk_geom, p->chunks.data(), cg_bytes);
  return LFD_OK;
}

int lfd_debug_block_taps(const lfd_lowpass_plan *p, double *taps, size_t n_taps, int *n_comp,
                         int64_t *row_len) {
  if (!p) return fail(LFD_EINVAL, "plan is NULL");
  if (p->taps.empty()) return fail(LFD_EUNSUPPORTED, "plan has no block taps (recurrence kernel only)");
  const int64_t row = (int64_t)(p->taps.size() / p->tg.nc);
  if (n_comp) *n_comp = p->tg.nc;
  if (row_len) *row_len = row;
  if (taps) {
    if (n_taps != p->taps.size())
      return fail(LFD_EINVAL, "taps buffer must hold n_comp * row_len doubles");
    std::memcpy(taps, p->taps.data(), n_taps * sizeof(double));
  }
  return LFD_OK;
}

int lfd_debug_lattice(const lfd_lowpass_plan *p, int64_t *n_offsets, int *last_onepass,
                      const lfd_lowpass_plan **one_pass) {
  if (!p) return fail(LFD_EINVAL, "plan is NULL");
  if (n_offsets) *n_offsets = p->lat ? p->lat->n_off : 0;
  if (last_onepass) *last_onepass = p->last_onepass ? 1 : 0;
  if (one_pass) *one_pass = p->lat;
  return LFD_OK;
}

int lfd_debug_runs(const lfd_lowpass_plan *p, int64_t *run_ks, int *run_len, int64_t max_runs,
                   int64_t *n_runs, void *run_const, size_t rc_bytes) {
  if (!p) return fail(LFD_EINVAL, "plan is NULL");
  if (!p->run_ok) return fail(LFD_EUNSUPPORTED, "plan has no run mode");
  const int64_t nr = (int64_t)p->run_ks.size();
  if (n_runs) *n_runs = nr;
  if (run_ks || run_len) {
    if (max_runs < nr) return fail(LFD_EINVAL, "run arrays too small");
    if (run_ks) std::memcpy(run_ks, p->run_ks.data(), sizeof(int64_t) * nr);
    if (run_len) std::memcpy(run_len, p->run_len.data(), sizeof(int) * nr);
  }
  if (run_const) {
    if (rc_bytes != sizeof(lfd::RunConst))
      return fail(LFD_EINVAL, "RunConst is " + std::to_string(sizeof(lfd::RunConst)) + " bytes");
    std::memcpy(run_const, &p->rc, rc_bytes);
  }
  return LFD_OK;
}

int lfd_lowpass_last_scan(const lfd_lowpass_plan *p) {
  if (!p) return fail(LFD_EINVAL, "plan is NULL");
  return p->last_scan;
}

int lfd_lowpass_last_kernel(const lfd_lowpass_plan *p) {
  if (!p) return fail(LFD_EINVAL, "plan is NULL");
  return p->last_k1;
}

void lfd_lowpass_plan_destroy(lfd_lowpass_plan *p) {
  if (!p) return;
  for (auto *sp : p->subs) lfd_lowpass_plan_destroy(sp);
  if (p->lat) lfd_lowpass_plan_destroy(p->lat);
  for (void *d : {(void *)p->d_bj, (void *)p->d_bi, (void *)p->d_bw, (void *)p->d_bi_lat, (void *)p->d_rc_off,
                  (void *)p->d_chunks_off, (void *)p->d_segs, (void *)p->d_segs_fu})
    if (d) (void)hipFree(d);
  if (p->d_chunks) (void)hipFree(p->d_chunks);
  if (p->d_taps) (void)hipFree(p->d_taps);
  if (p->d_taps_tm) (void)hipFree(p->d_taps_tm);
  for (void *d : {(void *)p->d_run_ks, (void *)p->d_run_len, (void *)p->d_group_r0, (void *)p->d_rc,
                  (void *)p->d_slot_chunk})
    if (d) (void)hipFree(d);
  for (auto &e : p->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto &e : p->split_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto &e : p->ring)
    if (e) (void)hipEventDestroy(e);
  delete p;
}

}  // extern "C"

namespace {
// ---------------------------------------------------------------------------
// Full-rate path (lfd_sosfiltfilt_f32): k_fullrate_wave functionals over big
// blocks of FR_L samples -> k_fullrate_scan per channel (edges, states at
// every block start, the tail's outputs) -> k_fullrate_wave outputs.  The
// tail [nb * FR_L, n_t) keeps at least one sample (the reverse pass starts
// from y_f[-1], which the scan computes).
// ---------------------------------------------------------------------------
int64_t fullrate_blocks(int64_t n_t) {  // the tail keeps >= 1 sample
  return n_t > 1 ? (n_t - 1) / lfd::FR_L : 0;
}

struct FrLayout {
  size_t off_F, off_SF, off_ST, off_TP, bytes;
  size_t off_SFm = 0;  // (medium-block path) S_f at every medium block
};
FrLayout fullrate_layout(int64_t n_ch, int64_t n_t, int padlen, int n_sec, int64_t nb) {
  const size_t n = 2 * n_sec;
  FrLayout l{};
  l.off_F = 0;
  l.off_SF = align256(sizeof(double) * 2 * n * nb * n_ch);
  l.off_ST = l.off_SF + align256(sizeof(double) * n * (nb + 1) * n_ch);
  l.off_TP = l.off_ST + align256(sizeof(double) * n * (nb + 1) * n_ch);
  l.bytes = l.off_TP + align256(sizeof(double) * (size_t)(n_t - nb * lfd::FR_L + padlen) * n_ch);
  return l;
}
// Medium-block path: F2 [ch/16][M][2N][16], SF = SFm [M][N][ch], ST = STm
// [M + 1][N][ch] (M = (n_t - 1) / FR_LB medium blocks), TP.
int64_t fullrate_medium_blocks(int64_t n_t) { return (n_t - 1) / lfd::FR_LB; }  // the tail keeps >= 1 sample
FrLayout fullrate_layout_mb(int64_t n_ch, int64_t n_t, int padlen, int n_sec) {
  const size_t n = 2 * n_sec, ch16 = (size_t)((n_ch + 15) / 16) * 16;
  const int64_t M = fullrate_medium_blocks(n_t);
  FrLayout l{};
  l.off_F = 0;
  l.off_SF = align256(sizeof(double) * 2 * n * M * ch16);
  l.off_SFm = l.off_SF;
  l.off_ST = l.off_SF + align256(sizeof(double) * n * M * n_ch);
  l.off_TP = l.off_ST + align256(sizeof(double) * n * (M + 1) * n_ch);
  l.bytes = l.off_TP + align256(sizeof(double) * (size_t)(n_t - M * lfd::FR_LB + padlen) * n_ch);
  return l;
}

// Per-(device, cascade) device constants, built on first use (the per-call
// path then allocates nothing and never synchronises).
// Entries are shared: a caller holds its entry while it launches, so an
// eviction by another thread never frees a table under a running call (the
// destructor's hipFree also waits for queued kernels to finish).
struct FrEntry {
  int dev = -1, n_sec = 0;
  double sos[6 * MAX_SEC] = {0};
  lfd::FRConst *d_fc = nullptr;
  double *d_ktaps = nullptr;  // medium-block functional taps (fullrate_medium_taps)
  ~FrEntry() {
    if (d_fc) (void)hipFree(d_fc);
    if (d_ktaps) (void)hipFree(d_ktaps);
  }
};
std::mutex g_fr_mu;
std::vector<std::shared_ptr<FrEntry>> g_fr;
// lfd_set_timing(1): events around the three launches of the last blocked call
hipEvent_t g_fr_ev[4] = {nullptr, nullptr, nullptr, nullptr};
int g_fr_ev_dev = -1;
bool g_fr_timed = false;

int fullrate_entry(const double *sos, int n_sec, const Cascade &c, std::shared_ptr<const FrEntry> *out) {
  int dev = 0;
  LFD_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_fr_mu);
  for (const auto &e : g_fr)
    if (e->dev == dev && e->n_sec == n_sec && std::memcmp(e->sos, sos, sizeof(double) * 6 * n_sec) == 0) {
      *out = e;
      return LFD_OK;
    }
  auto e = std::make_shared<FrEntry>();
  e->dev = dev;
  e->n_sec = n_sec;
  std::memcpy(e->sos, sos, sizeof(double) * 6 * n_sec);
  auto fc = std::make_unique<lfd::FRConst>();
  fullrate_constants(c, *fc);
  LFD_HIP(hipMalloc(&e->d_fc, sizeof(lfd::FRConst)));
  hipError_t he = hipMemcpy(e->d_fc, fc.get(), sizeof(lfd::FRConst), hipMemcpyHostToDevice);
  if (he != hipSuccess) return fail(LFD_EHIP, std::string("full-rate constants: ") + hipGetErrorString(he));
  const std::vector<double> kt = fullrate_medium_taps(c);
  LFD_HIP(hipMalloc(&e->d_ktaps, sizeof(double) * kt.size()));
  he = hipMemcpy(e->d_ktaps, kt.data(), sizeof(double) * kt.size(), hipMemcpyHostToDevice);
  if (he != hipSuccess) return fail(LFD_EHIP, std::string("full-rate taps: ") + hipGetErrorString(he));
  // bounded: drop the oldest from the cache (freed when its last user returns)
  if (g_fr.size() >= 16) g_fr.erase(g_fr.begin());
  g_fr.push_back(e);
  *out = std::move(e);
  return LFD_OK;
}
}  // namespace

extern "C" {

size_t lfd_sosfiltfilt_workspace_bytes(int64_t n_ch, int64_t n_t, int padlen, int n_sec) {
  if (padlen < 0) padlen = 3 * (2 * n_sec + 1);
  size_t b = align256(sizeof(double) * (size_t)(n_t + 2 * (int64_t)padlen) * (size_t)n_ch);
  if (n_sec >= 1 && n_sec <= MAX_SEC && n_ch >= 1) {
    const int64_t nb = fullrate_blocks(n_t);
    if (nb > 0)
      b = std::max({b, fullrate_layout(n_ch, n_t, padlen, n_sec, nb).bytes,
                    fullrate_layout_mb(n_ch, n_t, padlen, n_sec).bytes});
  }
  return b;
}

int lfd_sosfiltfilt_f32(const float *x, int64_t n_ch, int64_t n_t, int64_t s_ch,
                        int64_t s_t, const double *sos, int n_sec, int padlen,
                        double *y, int64_t ys_ch, int64_t ys_t, void *workspace,
                        void *stream) {
  Cascade c;
  if (int e = load_sos(sos, n_sec, c)) return e;
  if (padlen < 0) padlen = default_padlen(c);
  if (n_ch < 1 || n_t < 1) return fail(LFD_EINVAL, "n_ch and n_t must be >= 1");
  if (n_t <= padlen)
    return fail(LFD_EINVAL, "The length of the input vector x must be greater than padlen, which is " +
                                std::to_string(padlen) + ".");
  if (!x || !y || !workspace) return fail(LFD_EINVAL, "x, y and workspace must be device pointers");
  lfd::SosCoef cf{};
  for (int s = 0; s < n_sec; ++s) {
    cf.b0[s] = c.b0[s];
    cf.b1[s] = c.b1[s];
    cf.b2[s] = c.b2[s];
    cf.a1[s] = c.a1[s];
    cf.a2[s] = c.a2[s];
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // blocked path (k_fullrate_wave -> k_fullrate_scan -> k_fullrate_wave) when
  // the array holds a big block; LFD_FULLRATE_SERIAL=1 (A/B knob) keeps the
  // one-thread-per-channel kernel
  const int64_t nb = fullrate_blocks(n_t);
  if (nb > 0 && !lfd::option(LFD_OPT_FULLRATE_SERIAL)) {
    std::shared_ptr<const FrEntry> fe;
    if (int e = fullrate_entry(sos, n_sec, c, &fe)) return e;
    // medium-block path (time-contiguous rows, any stride): the functionals
    // on the fp64 matrix cores and the segmented scan
    const bool mb = s_t == 1 && (reinterpret_cast<uintptr_t>(x) & 3) == 0 && !lfd::option(LFD_OPT_FULLRATE_BIGBLOCK);
    const FrLayout lo = mb ? fullrate_layout_mb(n_ch, n_t, padlen, n_sec)
                           : fullrate_layout(n_ch, n_t, padlen, n_sec, nb);
    char *ws = static_cast<char *>(workspace);
    double *F = reinterpret_cast<double *>(ws + lo.off_F);
    double *SF = reinterpret_cast<double *>(ws + lo.off_SF);
    double *ST = reinterpret_cast<double *>(ws + lo.off_ST);
    double *TP = reinterpret_cast<double *>(ws + lo.off_TP);
    const bool timed = lfd::timing_enabled();
    if (timed) {
      std::lock_guard<std::mutex> lk(g_fr_mu);
      int dev = 0;
      LFD_HIP(hipGetDevice(&dev));
      if (g_fr_ev_dev != dev) {
        for (auto &ev : g_fr_ev)
          if (ev) (void)hipEventDestroy(ev);
        for (auto &ev : g_fr_ev) LFD_HIP(hipEventCreate(&ev));
        g_fr_ev_dev = dev;
      }
      g_fr_timed = true;
    } else {
      std::lock_guard<std::mutex> lk(g_fr_mu);
      g_fr_timed = false;
    }
    if (timed) LFD_HIP(hipEventRecord(g_fr_ev[0], st));
    if (mb) {
      const int n = 2 * n_sec;
      const int64_t M = fullrate_medium_blocks(n_t);
      const lfd::BlockGeom g{n_ch, M, 0, lfd::FR_LB, 2 * n, 0};
      const lfd::TapGeom tg{lfd::FR_LB, 0, 2 * n, 1, 0};
      LFD_HIP(lfd::launch_block_functionals_mfma(x, s_ch, n_t, g, fe->d_ktaps, tg, F, st));
      if (timed) LFD_HIP(hipEventRecord(g_fr_ev[1], st));
      const lfd::FRSeg sg = fullrate_segments(c, M, n_ch);
      LFD_HIP(lfd::launch_fullrate_scan_seg(n_sec, x, s_ch, s_t, n_ch, n_t, M, padlen, fe->d_fc, F, SF, ST, TP, y,
                                            ys_ch, ys_t, sg, st));
    } else {
      LFD_HIP(lfd::launch_fullrate_blocks(n_sec, false, x, s_ch, s_t, n_ch, nb, fe->d_fc, nullptr, nullptr, F,
                                          nullptr, 0, 0, st));
      if (timed) LFD_HIP(hipEventRecord(g_fr_ev[1], st));
      LFD_HIP(lfd::launch_fullrate_scan(n_sec, x, s_ch, s_t, n_ch, n_t, nb, padlen, fe->d_fc, F, SF, ST, TP, y,
                                        ys_ch, ys_t, st));
    }
    if (timed) LFD_HIP(hipEventRecord(g_fr_ev[2], st));
    const int64_t n_mb = mb ? fullrate_medium_blocks(n_t) : 0;
    LFD_HIP(lfd::launch_fullrate_blocks(n_sec, true, x, s_ch, s_t, n_ch, mb ? (n_mb + 3) / 4 : nb, fe->d_fc, SF, ST,
                                        nullptr, y, ys_ch, ys_t, st, mb, n_mb));
    if (timed) LFD_HIP(hipEventRecord(g_fr_ev[3], st));
    return LFD_OK;
  }
  lfd::ZiVec zi{};
  sosfilt_zi(c, zi.v);
  LFD_HIP(lfd::launch_sosfiltfilt(n_sec, x, n_ch, n_t, s_ch, s_t, cf, zi, padlen,
                                  static_cast<double *>(workspace), y, ys_ch, ys_t, st));
  return LFD_OK;
}

int lfd_sosfiltfilt_last_timing(float *ms_functionals, float *ms_scan, float *ms_output) {
  std::lock_guard<std::mutex> lk(g_fr_mu);
  if (!g_fr_timed) return fail(LFD_EINVAL, "timing was not enabled for the last blocked full-rate call");
  LFD_HIP(hipEventSynchronize(g_fr_ev[3]));
  float a = 0, b = 0, c = 0;
  LFD_HIP(hipEventElapsedTime(&a, g_fr_ev[0], g_fr_ev[1]));
  LFD_HIP(hipEventElapsedTime(&b, g_fr_ev[1], g_fr_ev[2]));
  LFD_HIP(hipEventElapsedTime(&c, g_fr_ev[2], g_fr_ev[3]));
  if (ms_functionals) *ms_functionals = a;
  if (ms_scan) *ms_scan = b;
  if (ms_output) *ms_output = c;
  return LFD_OK;
}

int lfd_interp_linear_f64(const double *x, int64_t n_ch, int64_t n_t, int64_t s_ch,
                          int64_t s_t, const int64_t *lo_dev, const double *w_dev,
                          int64_t n_out, double *y, int64_t ys_ch, int64_t ys_t,
                          void *stream) {
  if (n_ch < 1 || n_out < 0) return fail(LFD_EINVAL, "bad sizes");
  if (n_out == 0) return LFD_OK;
  LFD_HIP(lfd::launch_interp_linear(x, n_ch, n_t, s_ch, s_t, lo_dev, w_dev, n_out, y, ys_ch,
                                    ys_t, reinterpret_cast<hipStream_t>(stream)));
  return LFD_OK;
}

int lfd_sos_filtfilt_resample_f32(const float *x, int64_t n_ch, int64_t n_t, int64_t s_ch,
                                  int64_t s_t, const double *sos, int n_sec, int padlen,
                                  const int64_t *lo, const double *w, int64_t n_out, double *y,
                                  int64_t ys_ch, int64_t ys_t, void *stream) {
  if (n_out < 1) return LFD_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  lfd_chunk ck{0, n_t - 1, 0, n_out};
  lfd_lowpass_plan *plan = nullptr;
  int rc = lfd_lowpass_plan_create(&plan, sos, n_sec, padlen, n_ch, n_t, lo, w, n_out, &ck, 1);
  if (rc == LFD_OK) {
    void *ws = nullptr;
    hipError_t e = hipMalloc(&ws, std::max<size_t>(plan->ws_bytes, 256));
    if (e == hipSuccess) rc = lfd_lowpass_execute(plan, x, s_ch, s_t, y, ys_ch, ys_t, ws, st);
    else rc = fail(LFD_EHIP, std::string("workspace: ") + hipGetErrorString(e));
    if (e == hipSuccess) {
      hipError_t e2 = hipStreamSynchronize(st);
      (void)hipFree(ws);
      if (rc == LFD_OK && e2 != hipSuccess) rc = fail(LFD_EHIP, hipGetErrorString(e2));
    }
    lfd_lowpass_plan_destroy(plan);
    return rc;
  }
  if (rc != LFD_EUNSUPPORTED) return rc;
  // general path: full-rate zero-phase filter, then a device gather
  Cascade c;
  if (int e = load_sos(sos, n_sec, c)) return e;
  const int pl = padlen < 0 ? default_padlen(c) : padlen;
  for (int64_t j = 0; j < n_out; ++j)
    if (lo[j] < 0 || lo[j] >= n_t || (w[j] != 0.0 && lo[j] + 1 >= n_t))
      return fail(LFD_EINVAL, "interpolation position outside the array");
  // channel slabs bound the float64 intermediate (<= 16 GB per slab)
  const int64_t slab = std::max<int64_t>(1, std::min<int64_t>(n_ch, ((int64_t)1 << 31) / std::max<int64_t>(1, n_t)));
  const size_t wsb = lfd_sosfiltfilt_workspace_bytes(slab, n_t, pl, n_sec);
  const size_t yb = align256(sizeof(double) * (size_t)slab * n_t);
  const size_t tb = align256((sizeof(int64_t) + sizeof(double)) * (size_t)n_out);
  char *buf = nullptr;
  LFD_HIP(hipMalloc(&buf, wsb + yb + tb));
  double *yf = reinterpret_cast<double *>(buf + wsb);
  int64_t *dlo = reinterpret_cast<int64_t *>(buf + wsb + yb);
  double *dw = reinterpret_cast<double *>(buf + wsb + yb + sizeof(int64_t) * n_out);
  hipError_t e = hipMemcpy(dlo, lo, sizeof(int64_t) * n_out, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dw, w, sizeof(double) * n_out, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(buf);
    return fail(LFD_EHIP, hipGetErrorString(e));
  }
  rc = LFD_OK;
  for (int64_t c0 = 0; c0 < n_ch && rc == LFD_OK; c0 += slab) {
    const int64_t nc = std::min(slab, n_ch - c0);
    rc = lfd_sosfiltfilt_f32(x + c0 * s_ch, nc, n_t, s_ch, s_t, sos, n_sec, pl, yf, n_t, 1, buf, stream);
    if (rc == LFD_OK)
      rc = lfd_interp_linear_f64(yf, nc, n_t, n_t, 1, dlo, dw, n_out, y + c0 * ys_ch, ys_ch, ys_t, stream);
  }
  e = hipStreamSynchronize(st);
  (void)hipFree(buf);
  if (rc == LFD_OK && e != hipSuccess) rc = fail(LFD_EHIP, hipGetErrorString(e));
  return rc;
}

int lfd_rolling_mean_f32(const float *x, int64_t n_ch, int64_t n_t, int64_t s_ch, int64_t s_t,
                         int64_t window, int64_t step, float *y, int64_t ys_ch, int64_t ys_t,
                         void *stream) {
  if (window < 1 || step < 1) return fail(LFD_EINVAL, "window and step must be >= 1 samples");
  if (n_ch < 1 || n_t < 1) return LFD_OK;
  if (!x || !y) return fail(LFD_EINVAL, "x and y must be device pointers");
  LFD_HIP(lfd::launch_rolling_mean(x, n_ch, n_t, s_ch, s_t, window, step, y, ys_ch, ys_t,
                                   reinterpret_cast<hipStream_t>(stream)));
  return LFD_OK;
}

static thread_local int g_fir_kernel = -1;

int lfd_fir_decimate_f32(const float *x, int64_t n_ch, int64_t n_t, int64_t s_ch, int64_t s_t,
                         const double *taps, int64_t n_taps, int64_t q, int64_t delay, double *y, int64_t ys_ch,
                         int64_t ys_t, void *stream) {
  if (q < 1) return fail(LFD_EINVAL, "decimation factor must be >= 1");
  if (n_taps < 1 || q > (1 << 20) || (n_taps + q - 1) / q + 3 > 16 * 1024 / q)
    return fail(LFD_EINVAL, "FIR too long for the staged tile (q * (ceil(n_taps / q) + 3) must be <= 16384)");
  if (n_ch < 1 || n_t < 1) return LFD_OK;
  if (!x || !y || !taps) return fail(LFD_EINVAL, "x, taps and y must be device pointers");
  LFD_HIP(lfd::launch_fir_decimate(x, n_ch, n_t, s_ch, s_t, taps, (int)n_taps, q, delay, y, ys_ch, ys_t,
                                   reinterpret_cast<hipStream_t>(stream), &g_fir_kernel));
  return LFD_OK;
}

int lfd_fir_decimate_last_kernel(void) { return g_fir_kernel; }

int lfd_demean_scale_f64(const double *x, int64_t n_rows, int64_t n_cols, int64_t s_r, int64_t s_c,
                         int64_t c0, int64_t c1, double scale, double *y, int64_t ys_r, int64_t ys_c,
                         void *stream) {
  if (n_rows < 0 || n_cols < 0) return fail(LFD_EINVAL, "negative size");
  if (c0 < 0 || c1 > n_cols || c1 <= c0) return fail(LFD_EINVAL, "demean channel range must be inside [0, n_cols) and non-empty");
  if (n_rows == 0) return LFD_OK;
  if (!x || !y) return fail(LFD_EINVAL, "x and y must be device pointers");
  LFD_HIP(lfd::launch_demean_scale(x, n_rows, n_cols, s_r, s_c, c0, c1, scale, y, ys_r, ys_c,
                                   reinterpret_cast<hipStream_t>(stream)));
  return LFD_OK;
}

int lfd_median_filter_f64(const double *x, int64_t n0, int64_t n1, int64_t s0, int64_t s1, int k0, int k1,
                          double *y, int64_t ys0, int64_t ys1, void *stream) {
  if (n0 < 0 || n1 < 0) return fail(LFD_EINVAL, "negative size");
  if (k0 < 1 || k1 < 1) return fail(LFD_EINVAL, "median window sizes must be >= 1");
  if ((size_t)(16 + k0 - 1) * (size_t)(16 + k1 - 1) * sizeof(double) > 64 * 1024)
    return fail(LFD_EUNSUPPORTED, "median window too large for one LDS tile");
  if (n0 == 0 || n1 == 0) return LFD_OK;
  if (!x || !y) return fail(LFD_EINVAL, "x and y must be device pointers");
  if (x == y) return fail(LFD_EINVAL, "median filter cannot run in place");
  LFD_HIP(lfd::launch_median2d(x, n0, n1, s0, s1, k0, k1, y, ys0, ys1, reinterpret_cast<hipStream_t>(stream)));
  return LFD_OK;
}

}  // extern "C"
