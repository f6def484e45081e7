// Host-side sanitizer driver (ASan + UBSan, SURVEY §5 "race detection /
// sanitizers"): drives the host code of liblfdas — plan geometry and
// constants (lfd_capi.cpp), the stream's arena / schedule bookkeeping
// (lfd_stream.cpp, LFD_STREAM_DRY_RUN) and the LFProc schedule — through
// include/lfdas.h alone, with no device visible, so every plan is host-only.
// Built and run by tests/test_sanitize.py (tools/sanitize.sh): any ASan or
// UBSan report aborts with a non-zero status.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "../../include/lfdas.h"

#define CHECK(x)                                                                                   \
  do {                                                                                             \
    int rc_ = (x);                                                                                 \
    if (rc_ != LFD_OK) {                                                                           \
      std::fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_, lfd_last_error()); \
      std::exit(1);                                                                                \
    }                                                                                              \
  } while (0)
#define EXPECT_FAIL(x)                                                         \
  do {                                                                         \
    if ((x) == LFD_OK) {                                                       \
      std::fprintf(stderr, "%s:%d %s unexpectedly ok\n", __FILE__, __LINE__, #x); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

namespace {

constexpr int64_t T0 = 1505692800000000000LL;  // 2017-09-18T00:00:00 (DASCore random_das)

// scipy zpk2sos(iirfilter(4, Wn, 'lowpass', 'butter', 'zpk')) of cfg3 (fs
// 500 Hz, fc 0.45 Hz) and cfg1 (250 Hz, 0.9 Hz), as lfdas.design.lowpass_sos
const double SOS_CFG3[12] = {6.344032428057516e-11, 1.2688064856115032e-10, 6.344032428057516e-11, 1.0,
                             -1.9895737178486945,   0.9896055290874918,     1.0,
                             2.0,                   1.0,                    1.0,
                             -1.9956494127028517,   0.9956813210857649};
const double SOS_CFG1[12] = {1.588723095420894e-08, 3.177446190841788e-08, 1.588723095420894e-08, 1.0,
                             -1.958562493267189,    0.9590636398459286,    1.0,
                             2.0,                   1.0,                   1.0,
                             -1.9823306020831202,   0.9828378303194311};
// scipy.signal.butter(8, 0.01, output='sos'): an 8th-order cascade (4
// sections: the recurrence-kernel plans, no run mode)
const double SOS_8[24] = {3.4219614165936484e-15, 6.843922833187297e-15, 3.4219614165936484e-15, 1.0,
                          -1.939269633591658,     0.9402270185020654,    1.0,
                          2.0,                    1.0,                   1.0,
                          -1.9481335385151675,    0.9490952993868512,    1.0,
                          2.0,                    1.0,                   1.0,
                          -1.9647269019487286,    0.9656968546857874,    1.0,
                          2.0,                    1.0,                   1.0,
                          -1.9868379069766875,    0.987818775546285};

// lf_das.py:252-256 time grid (int(dt*1000) ms step) over [t1, t2)
std::vector<int64_t> time_grid(int64_t t1, int64_t t2, double dt) {
  const int64_t step = (int64_t)(dt * 1000.0) * 1000000LL;
  std::vector<int64_t> tg;
  for (int64_t t = t1; t < t2; t += step) tg.push_back(t);
  return tg;
}

// one LFProc plan over n samples of sample_ns starting at t0: grid positions,
// inclusive select ranges, lfd_lfproc_schedule chunks; host-only create plus
// every debug accessor
void plan_case(const double *sos, int n_sec, int64_t n_ch, int64_t n, int64_t sample_ns, int64_t t0,
               int64_t t_grid0, double dt, int64_t P, int64_t B) {
  const std::vector<int64_t> tg = time_grid(t_grid0, t0 + n * sample_ns, dt);
  const int64_t L = (int64_t)tg.size();
  std::vector<int64_t> lo(L);
  std::vector<double> w(L);
  for (int64_t j = 0; j < L; ++j) {
    const int64_t rel = tg[j] - t0;
    lo[j] = rel >= 0 ? rel / sample_ns : -1;
    w[j] = rel >= 0 ? (double)(rel % sample_ns) / (double)sample_ns : 0.0;
  }
  std::vector<int64_t> rows(4 * (L + 4));
  int64_t nr = 0;
  CHECK(lfd_lfproc_schedule(L, P, B, rows.data(), L + 4, &nr));
  std::vector<lfd_chunk> ck(nr);
  for (int64_t i = 0; i < nr; ++i) {
    const int64_t a = tg[rows[4 * i]] - t0, b = tg[rows[4 * i + 1]] - t0;
    ck[i].s0 = a <= 0 ? 0 : (a + sample_ns - 1) / sample_ns;  // inclusive select
    ck[i].s1 = std::min<int64_t>(n - 1, b / sample_ns);
    ck[i].g0 = rows[4 * i + 2];
    ck[i].g1 = rows[4 * i + 3];
  }
  lfd_lowpass_plan *p = nullptr;
  CHECK(lfd_lowpass_plan_create(&p, sos, n_sec, 15, n_ch, n, lo.data(), w.data(), L, ck.data(), nr));
  size_t ws = 0;
  int64_t nb = 0, bl = 0;
  CHECK(lfd_lowpass_plan_info(p, &ws, &nb, &bl));
  int nc = 0;
  int64_t row = 0;
  if (lfd_debug_block_taps(p, nullptr, 0, &nc, &row) == LFD_OK) {
    std::vector<double> taps((size_t)nc * row);
    CHECK(lfd_debug_block_taps(p, taps.data(), taps.size(), &nc, &row));
  }
  int64_t n_runs = 0;
  if (lfd_debug_runs(p, nullptr, nullptr, 0, &n_runs, nullptr, 0) == LFD_OK) {
    std::vector<int64_t> ks(n_runs);
    std::vector<int> ln(n_runs);
    CHECK(lfd_debug_runs(p, ks.data(), ln.data(), n_runs, &n_runs, nullptr, 0));
    int64_t tmp = 0;
    if (n_runs > 1) EXPECT_FAIL(lfd_debug_runs(p, ks.data(), ln.data(), n_runs - 1, &tmp, nullptr, 0));
  }
  int64_t n_off = 0;
  int onepass = 0;
  const lfd_lowpass_plan *inner = nullptr;
  CHECK(lfd_debug_lattice(p, &n_off, &onepass, &inner));
  if (inner) {
    int64_t nb2 = 0, bl2 = 0;
    size_t ws2 = 0;
    CHECK(lfd_lowpass_plan_info(inner, &ws2, &nb2, &bl2));
  }
  // execute without a device fails cleanly
  float dummy = 0.f;
  double ydummy = 0.0;
  EXPECT_FAIL(lfd_lowpass_execute(p, &dummy, n, 1, &ydummy, L, 1, &dummy, nullptr));
  lfd_lowpass_plan_destroy(p);
}

void plan_errors() {
  lfd_lowpass_plan *p = nullptr;
  const int64_t lo[3] = {0, 10, 20};
  const double w[3] = {0, 0, 0};
  lfd_chunk ck = {0, 25, 0, 3};
  double bad[6] = {1, 2, 1, 2.0, -1.9, 0.9};  // a0 != 1
  EXPECT_FAIL(lfd_lowpass_plan_create(&p, bad, 1, 15, 4, 30, lo, w, 3, &ck, 1));
  EXPECT_FAIL(lfd_lowpass_plan_create(&p, SOS_CFG3, 0, 15, 4, 30, lo, w, 3, &ck, 1));
  EXPECT_FAIL(lfd_lowpass_plan_create(&p, SOS_CFG3, 2, 15, 4, 30, lo, w, 3, nullptr, 1));
  lfd_chunk past = {0, 40, 0, 3};  // beyond n_t
  EXPECT_FAIL(lfd_lowpass_plan_create(&p, SOS_CFG3, 2, 15, 4, 30, lo, w, 3, &past, 1));
  lfd_chunk shortc = {0, 10, 0, 2};  // <= padlen samples
  EXPECT_FAIL(lfd_lowpass_plan_create(&p, SOS_CFG3, 2, 15, 4, 30, lo, w, 3, &shortc, 1));
  EXPECT_FAIL(lfd_set_option(99, 1));
  EXPECT_FAIL(lfd_set_option(LFD_OPT_SCAN_DEFER, 9));
  int64_t rows[16], nr = 0;
  EXPECT_FAIL(lfd_lfproc_schedule(100, 12, 6, rows, 4, &nr));  // P <= 2B: the reference loops forever
  EXPECT_FAIL(lfd_lfproc_schedule(1, 40, 6, rows, 4, &nr));
}

void schedules() {
  for (int64_t L : {2, 3, 5, 14, 15, 16, 17, 40, 41, 100, 120, 601, 3600, 8640})
    for (const auto &pb : {std::pair<int64_t, int64_t>{40, 6}, {600, 7}, {100, 10}, {15, 7}, {30, 3}}) {
      std::vector<int64_t> rows(4 * (L + 4));
      int64_t nr = 0;
      (void)lfd_lfproc_schedule(L, pb.first, pb.second, rows.data(), L + 4, &nr);
      int64_t small[4];
      (void)lfd_lfproc_schedule(L, pb.first, pb.second, small, 1, &nr);  // too small: error, no overrun
    }
}

// DASCore random_das-like stream: n_push pushes of push samples
void stream_case(int mode, int64_t n_ch, int64_t sample_ns, double dt, int64_t P, int64_t B, int64_t push,
                 int n_push, int64_t t_start_off) {
  lfd_stream_config cfg{};
  cfg.n_ch = n_ch;
  cfg.sample_ns = sample_ns;
  cfg.output_sample_interval = dt;
  cfg.process_patch_size = P;
  cfg.edge_buff_size = B;
  cfg.mode = mode;
  cfg.flags = LFD_STREAM_DRY_RUN;
  cfg.t_start_ns = T0 + t_start_off;
  cfg.t_end_ns = T0 + (int64_t)n_push * push * sample_ns - sample_ns;
  cfg.resume_back_ns = (int64_t)((B - 1) * dt) * 1000000000LL;
  lfd_stream *s = nullptr;
  CHECK(lfd_stream_open(&s, &cfg, SOS_CFG1, 2, 15));
  CHECK(lfd_stream_reserve(s, push));
  for (int k = 0; k < n_push; ++k) {
    CHECK(lfd_stream_push(s, nullptr, push, push, 1, T0 + (int64_t)k * push * sample_ns));
    lfd_stream_output o{};
    CHECK(lfd_stream_last_output(s, &o));
    int64_t counts[64], nck = 0;
    CHECK(lfd_stream_last_chunks(s, counts, 64, &nck));
    int64_t cap = 0, held = 0, th = 0;
    CHECK(lfd_stream_info(s, &cap, &held, &th));
  }
  CHECK(lfd_stream_flush(s));
  // a gap: "patch merge failed! Gap in data exists"
  EXPECT_FAIL(lfd_stream_push(s, nullptr, push, push, 1, T0 + (int64_t)(n_push + 3) * push * sample_ns));
  int64_t created = 0, hits = 0;
  CHECK(lfd_debug_stream_plans(s, &created, &hits));
  lfd_stream_close(s);
}

}  // namespace

int main() {
  // host-only by construction: with a device visible the plans would get
  // device state and the dummy-pointer execute below would launch
  int ndev = 0;
  if (lfd_device_count(&ndev) == LFD_OK && ndev > 0) {
    std::printf("host sanitize driver: skipped (a device is visible)\n");
    return 0;
  }
  schedules();
  plan_errors();
  // cfg1 geometry (250 Hz, dt 0.2 s, P 40, B 6)
  plan_case(SOS_CFG1, 2, 24, 6000, 4000000, T0, T0, 0.2, 40, 6);
  // cfg3 parameters on a 20-minute slice (R = 500, P = 600, B = 7)
  plan_case(SOS_CFG3, 2, 70, 600000, 2000000, T0, T0, 1.0, 600, 7);
  // off-sample grid (samples start 1.9 ms after the grid's second: head skip)
  plan_case(SOS_CFG3, 2, 33, 750000, 2000000, T0 + 1900000, T0 + 1000000000, 1.0, 600, 7);
  // dt = 10 s at 200 Hz: sub-blocks (R = 2000)
  plan_case(SOS_CFG3, 2, 8, 600000, 5000000, T0, T0, 10.0, 100, 7);
  // 3 kHz on integer-ns times: lattice (composite + one-pass) plan
  plan_case(SOS_CFG3, 2, 16, 3000 * 600, 333333, T0, T0, 1.0, 120, 7);
  // 8th-order cascade: recurrence plans, no run mode
  plan_case(SOS_8, 4, 5, 100000, 1000000, T0, T0, 1.0, 30, 3);
  // streams (dry run): edge mode at cfg1 / cfg4-like cadence / lattice, continuous
  stream_case(LFD_STREAM_EDGE, 2, 4000000, 1.0, 125, 7, 30 * 250, 6, 0);
  stream_case(LFD_STREAM_EDGE, 2, 4000000, 0.2, 40, 6, 8 * 250, 6, 0);
  stream_case(LFD_STREAM_EDGE, 2, 333333, 1.0, 60, 6, 30 * 3000, 5, 0);
  stream_case(LFD_STREAM_CONTINUOUS, 3, 10000000, 1.0, 40, 5, 3000, 20, 0);
  std::printf("host sanitize driver: ok\n");
  return 0;
}
