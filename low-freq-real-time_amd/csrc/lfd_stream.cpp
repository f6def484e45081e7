// Streaming low-pass + decimate (include/lfdas.h, lfd_stream_*): the
// device-resident form of the real-time loop of low_pass_dascore_edge.ipynb
// (cell 11, :199-235) and of LFProc.process_time_range (lf_das.py:219-290)
// over spools larger than HBM.
//
// The reference re-reads the 2*edge overlap of every run from the archive
// and re-runs sosfiltfilt on it.  Here the samples stay in HBM: pushes append
// to a per-channel arena [n_ch][cap] (float32 rows, 16-B aligned, so the MFMA
// block-functional kernel applies), host->HBM copies run on their own HIP
// stream, and compaction copies only the columns a later run still reads into
// the second arena buffer (ping-pong), ordered on the compute stream.  Every
// run is one lfd_lowpass_plan execute over all of its chunks; plans are
// cached by geometry, so a steady stream of equal pushes creates no plans and
// allocates nothing.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/lfdas.h"
#include "lfd_internal.h"

using lfd::fail;

#define LFD_HIP(call)                                                           \
  do {                                                                          \
    hipError_t e_ = (call);                                                     \
    if (e_ != hipSuccess)                                                       \
      return fail(LFD_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define LFD_TRY(call)          \
  do {                         \
    int rc_ = (call);          \
    if (rc_ != LFD_OK) return rc_; \
  } while (0)

namespace {

using Row = std::array<int64_t, 4>;

inline int64_t floor_div(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}
inline int64_t ceil_div(int64_t a, int64_t b) { return -floor_div(-a, b); }
inline int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// lf_das.py:258-290 (first chunk, body loop, tail) as index arithmetic.
int lfproc_schedule(int64_t L, int64_t P, int64_t B, std::vector<Row> &out) {
  out.clear();
  if (L < 2) return fail(LFD_EINVAL, "time range holds fewer than 2 output samples");
  if (L <= P) P = L - 1;
  out.push_back({0, P, B, P - B});
  int64_t de = P, nde = de + P - 2 * B;
  if (nde <= de && nde < L)
    return fail(LFD_EINVAL, "process_patch_size must be larger than 2*edge_buff_size");
  while (nde < L) {
    out.push_back({de - 2 * B, nde, de - B, nde - B});
    de = nde;
    nde = de + P - 2 * B;
  }
  if (L - de > 1) {
    nde = L - 1;
    out.push_back({de - 2 * B, nde, de - B, nde - B});
  }
  return LFD_OK;
}

// Keeps the stream's device current for the duration of a call.
struct DeviceGuard {
  int prev = -1;
  bool active = false;
  explicit DeviceGuard(int dev) {
    if (dev < 0) return;
    if (hipGetDevice(&prev) == hipSuccess && prev != dev && hipSetDevice(dev) == hipSuccess)
      active = true;
  }
  ~DeviceGuard() {
    if (active) (void)hipSetDevice(prev);
  }
};

bool is_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

constexpr size_t PIN_BYTES = (size_t)32 << 20;  // each of the two staging buffers
constexpr size_t PLAN_CACHE_MAX = 32;

}  // namespace

struct lfd_stream {
  lfd_stream_config cfg{};
  std::vector<double> sos;
  int n_sec = 0, padlen = -1;
  int64_t out_ns = 0;
  bool dry = false;
  bool direct2d = false;  // LFD_STREAM_DIRECT2D=1: pitched DMA into the arena (A/B switch)
  int device = -1;
  hipStream_t s_copy = nullptr, s_comp = nullptr;
  hipEvent_t ev_h2d = nullptr, ev_compact = nullptr, ev_pin[2] = {}, ev_out[2] = {};
  hipEvent_t tm[4] = {};
  bool timed = false, timed_run = false;
  // arena: columns [a_lo, a_hi) of buffer `cur` are valid; column c holds
  // the sample at time t_col0 + c * sample_ns
  float *arena[2] = {};
  int cur = 0;
  int64_t cap = 0, a_lo = 0, a_hi = 0, t_col0 = 0;
  bool have = false;
  float *pin[2] = {};
  int pin_i = 0;
  float *stage = nullptr;
  size_t stage_bytes = 0;
  double *out[2] = {};
  size_t out_bytes[2] = {0, 0};
  int out_i = 0;
  lfd_stream_output last{};
  std::vector<int64_t> last_counts;
  std::map<std::vector<int64_t>, lfd_lowpass_plan *> plans;
  int64_t plans_created = 0, plan_hits = 0;  // lfd_debug_stream_plans
  void *ws = nullptr;
  size_t ws_bytes = 0;
  int64_t n_runs = 0;
  // edge mode
  bool produced = false;
  int64_t last_out_ns = 0;
  // continuous mode: the whole process_time_range schedule, next chunk
  std::vector<Row> sched;
  size_t next = 0;
  int64_t n_grid = 0;

  int64_t sample_ns() const { return cfg.sample_ns; }
  int64_t col_ceil(int64_t t) const { return ceil_div(t - t_col0, cfg.sample_ns); }
  int64_t col_floor(int64_t t) const { return floor_div(t - t_col0, cfg.sample_ns); }

  void drop_plans() {
    for (auto &kv : plans)
      if (kv.second) lfd_lowpass_plan_destroy(kv.second);
    plans.clear();
  }
};

namespace {

int alloc_arena(lfd_stream *s, int64_t new_cap) {
  // called with the streams idle (sync below); keeps [a_lo, a_hi)
  const int64_t keep = s->a_hi - s->a_lo;
  float *na[2] = {nullptr, nullptr};
  if (!s->dry) {
    LFD_HIP(hipStreamSynchronize(s->s_copy));
    LFD_HIP(hipStreamSynchronize(s->s_comp));
    const size_t bytes = sizeof(float) * (size_t)s->cfg.n_ch * (size_t)new_cap;
    for (auto &p : na) {
      hipError_t e = hipMalloc(&p, bytes);
      if (e != hipSuccess) {
        for (auto q : na)
          if (q) (void)hipFree(q);
        return fail(LFD_ENOMEM, "stream arena of " + std::to_string(bytes >> 20) + " MiB x 2: " +
                                    hipGetErrorString(e));
      }
    }
    if (keep > 0)
      LFD_HIP(hipMemcpy2DAsync(na[0], sizeof(float) * new_cap, s->arena[s->cur] + s->a_lo,
                               sizeof(float) * s->cap, sizeof(float) * keep, s->cfg.n_ch,
                               hipMemcpyDeviceToDevice, s->s_comp));
    LFD_HIP(hipStreamSynchronize(s->s_comp));
    for (auto &p : s->arena)
      if (p) (void)hipFree(p), p = nullptr;
    s->arena[0] = na[0];
    s->arena[1] = na[1];
  }
  s->cur = 0;
  s->cap = new_cap;
  s->t_col0 += s->a_lo * s->cfg.sample_ns;
  s->a_hi = keep;
  s->a_lo = 0;
  return LFD_OK;
}

// Make room for n_t more columns: compact [a_lo, a_hi) to column 0 of the
// other buffer (ordered after every run that still reads the current one),
// growing both buffers when the retained columns plus the push do not fit.
int make_room(lfd_stream *s, int64_t n_t) {
  const int64_t keep = s->a_hi - s->a_lo;
  if (keep + n_t > s->cap) return alloc_arena(s, round_up(std::max(2 * (keep + n_t), 2 * s->cap), 64));
  if (!s->dry) {
    const int other = s->cur ^ 1;
    if (keep > 0)
      LFD_HIP(hipMemcpy2DAsync(s->arena[other], sizeof(float) * s->cap, s->arena[s->cur] + s->a_lo,
                               sizeof(float) * s->cap, sizeof(float) * keep, s->cfg.n_ch,
                               hipMemcpyDeviceToDevice, s->s_comp));
    LFD_HIP(hipEventRecord(s->ev_compact, s->s_comp));
    LFD_HIP(hipStreamWaitEvent(s->s_copy, s->ev_compact, 0));
    s->cur = other;
  }
  s->t_col0 += s->a_lo * s->cfg.sample_ns;
  s->a_hi = keep;
  s->a_lo = 0;
  return LFD_OK;
}

// Host rectangle (rows x cols floats, row stride `sp` elements) -> device
// (pitch `dp` elements), through the pinned double buffer when `src` is
// pageable.  Row/column slabs keep every staging copy below PIN_BYTES.
int h2d_rect(lfd_stream *s, float *dst, int64_t dp, const float *src, int64_t sp, int64_t rows,
             int64_t cols) {
  if (rows <= 0 || cols <= 0) return LFD_OK;
  if (rows == 1) sp = cols;
  if (is_pinned(src)) {
    if (rows == 1) {
      LFD_HIP(hipMemcpyAsync(dst, src, sizeof(float) * cols, hipMemcpyHostToDevice, s->s_copy));
      return LFD_OK;
    }
    LFD_HIP(hipMemcpy2DAsync(dst, sizeof(float) * dp, src, sizeof(float) * sp, sizeof(float) * cols,
                             rows, hipMemcpyHostToDevice, s->s_copy));
    return LFD_OK;
  }
  const int64_t pin_f = (int64_t)(PIN_BYTES / sizeof(float));
  if (!s->pin[0])
    for (auto &p : s->pin) LFD_HIP(hipHostMalloc(reinterpret_cast<void **>(&p), PIN_BYTES, hipHostMallocDefault));
  const int64_t cw = std::min(cols, pin_f);
  const int64_t rh = std::max<int64_t>(1, pin_f / cw);
  for (int64_t c0 = 0; c0 < cols; c0 += cw) {
    const int64_t w = std::min(cw, cols - c0);
    for (int64_t r0 = 0; r0 < rows; r0 += rh) {
      const int64_t h = std::min(rh, rows - r0);
      const int i = s->pin_i;
      LFD_HIP(hipEventSynchronize(s->ev_pin[i]));  // previous DMA out of this buffer done
      float *p = s->pin[i];
      for (int64_t r = 0; r < h; ++r)
        std::memcpy(p + r * w, src + (r0 + r) * sp + c0, sizeof(float) * w);
      LFD_HIP(hipMemcpy2DAsync(dst + r0 * dp + c0, sizeof(float) * dp, p, sizeof(float) * w,
                               sizeof(float) * w, h, hipMemcpyHostToDevice, s->s_copy));
      LFD_HIP(hipEventRecord(s->ev_pin[i], s->s_copy));
      s->pin_i ^= 1;
    }
  }
  return LFD_OK;
}

int ensure_stage(lfd_stream *s, size_t need) {
  if (s->stage_bytes >= need) return LFD_OK;
  LFD_HIP(hipStreamSynchronize(s->s_copy));
  if (s->stage) (void)hipFree(s->stage), s->stage = nullptr;
  s->stage_bytes = 0;
  LFD_HIP(hipMalloc(&s->stage, need));
  s->stage_bytes = need;
  return LFD_OK;
}

// Copy a push into arena columns [a_hi, a_hi + n_t).
int copy_in(lfd_stream *s, const float *x, int64_t n_t, int64_t s_ch, int64_t s_t) {
  const int64_t n_ch = s->cfg.n_ch;
  float *dst = s->arena[s->cur] + s->a_hi;
  if (s->timed) LFD_HIP(hipEventRecord(s->tm[0], s->s_copy));
  if (s_t == 1 && (n_ch == 1 || s_ch == n_t) && !s->direct2d) {
    // dense (channel, time) block: one linear DMA into staging (a pitched
    // host->device copy pays per-row overhead: 50,000 rows of 48 KB run at
    // half the PCIe rate), then a device-side pitched copy into the arena
    LFD_TRY(ensure_stage(s, sizeof(float) * (size_t)n_t * (size_t)n_ch));
    LFD_TRY(h2d_rect(s, s->stage, (int64_t)n_t * n_ch, x, (int64_t)n_t * n_ch, 1, (int64_t)n_t * n_ch));
    LFD_HIP(hipMemcpy2DAsync(dst, sizeof(float) * s->cap, s->stage, sizeof(float) * n_t, sizeof(float) * n_t,
                             n_ch, hipMemcpyDeviceToDevice, s->s_copy));
  } else if (s_t == 1) {  // strided (channel, time) rows: pitched DMA straight into the arena
    LFD_TRY(h2d_rect(s, dst, s->cap, x, n_ch == 1 ? n_t : s_ch, n_ch, n_t));
  } else {  // (time, channel) rows: DMA to a staging array, transpose on device
    LFD_TRY(ensure_stage(s, sizeof(float) * (size_t)n_t * (size_t)n_ch));
    LFD_TRY(h2d_rect(s, s->stage, n_ch, x, s_t, n_t, n_ch));
    LFD_HIP(lfd::launch_transpose(s->stage, n_t, n_ch, n_ch, dst, s->cap, s->s_copy));
  }
  if (s->timed) LFD_HIP(hipEventRecord(s->tm[1], s->s_copy));
  LFD_HIP(hipEventRecord(s->ev_h2d, s->s_copy));
  LFD_HIP(hipStreamWaitEvent(s->s_comp, s->ev_h2d, 0));
  return LFD_OK;
}

int ensure_dev(void **p, size_t *have, size_t need, hipStream_t st) {
  if (*have >= need) return LFD_OK;
  LFD_HIP(hipStreamSynchronize(st));
  if (*p) (void)hipFree(*p), *p = nullptr;
  *have = 0;
  LFD_HIP(hipMalloc(p, need));
  *have = need;
  return LFD_OK;
}

// Run schedule rows `rows` (grid indices relative to t_grid0) on the arena.
int run_chunks(lfd_stream *s, int64_t t_grid0, const Row *rows, size_t n_rows) {
  const int64_t dts = s->cfg.sample_ns, n_ch = s->cfg.n_ch;
  std::vector<Row> cs(n_rows);  // arena columns s0, s1 and grid range
  for (size_t i = 0; i < n_rows; ++i) {
    const Row &r = rows[i];
    int64_t s0 = std::max(s->a_lo, s->col_ceil(t_grid0 + r[0] * s->out_ns));
    int64_t s1 = std::min(s->a_hi - 1, s->col_floor(t_grid0 + r[1] * s->out_ns));
    if (s1 < s0) return fail(LFD_EINVAL, "no samples in the chunk's time range (patch merge failed)");
    cs[i] = {s0, s1, r[2], std::max(r[2], r[3])};
  }
  const int64_t j0 = cs.front()[2], j1 = cs.back()[3];
  s->last_counts.clear();
  for (auto &c : cs) s->last_counts.push_back(c[3] - c[2]);
  s->last.n_chunks = (int64_t)n_rows;
  s->last.t_first_ns = t_grid0 + j0 * s->out_ns;
  s->last.t_step_ns = s->out_ns;
  const int64_t n_out = j1 - j0;
  s->last.n_out = std::max<int64_t>(n_out, 0);
  s->n_runs++;
  s->last.n_runs = s->n_runs;
  if (n_out <= 0) return LFD_OK;
  // output grid positions in arena columns
  std::vector<int64_t> lo(n_out);
  std::vector<double> w(n_out);
  bool aligned = true;
  for (int64_t j = 0; j < n_out; ++j) {
    const int64_t rel = t_grid0 + (j0 + j) * s->out_ns - s->t_col0;
    lo[j] = floor_div(rel, dts);
    w[j] = (double)(rel - lo[j] * dts) / (double)dts;
    // uniform grid, one fractional position for every point (the block plan's
    // domain; w != 0 when the archive's samples start off the output grid)
    aligned = aligned && w[j] == w[0] && (j == 0 || lo[j] - lo[j - 1] == lo[1] - lo[0]);
  }
  int64_t w0 = INT64_MAX, w1 = INT64_MIN;
  for (auto &c : cs) w0 = std::min(w0, c[0]), w1 = std::max(w1, c[1]);
  const int64_t x0 = w0 & ~(int64_t)3;  // 16-B aligned row start for the MFMA kernel
  const int64_t nt = w1 + 1 - x0;
  const int oi = s->out_i ^ 1;
  s->last.ys_ch = n_out;
  if (s->dry) {
    s->last.y = nullptr;
    s->out_i = oi;
    return LFD_OK;
  }
  LFD_TRY(ensure_dev(reinterpret_cast<void **>(&s->out[oi]), &s->out_bytes[oi],
                     sizeof(double) * (size_t)n_ch * (size_t)n_out, s->s_comp));
  double *y = s->out[oi];
  const float *x = s->arena[s->cur] + x0;
  lfd_lowpass_plan *plan = nullptr;
  // grid weights from the grid's integer times on device (lattice plans):
  // the same formula as w[] above, relative to the run's first output
  const lfd::GridGen gen{t_grid0 + j0 * s->out_ns - s->t_col0, s->out_ns, dts};
  if (n_out >= 2) {
    // uniform grids: keyed by (first point, spacing, fraction): the fraction
    // is part of the block plan's output functional.  Other grids (varying
    // fraction or spacing: lattice plans) are keyed by their STRUCTURE only —
    // every point's sample lo relative to the row start and whether it
    // blends (w != 0) — and take the fractions from `gen` at execute time, so
    // a steady 3 kHz stream reuses its few lattice plans instead of building
    // one per push
    int64_t wbits = 0;
    std::memcpy(&wbits, &w[0], sizeof(wbits));
    std::vector<int64_t> key = {nt, aligned ? 1 : 0, lo[0] - x0, lo[1] - lo[0], n_out, aligned ? wbits : 0};
    if (!aligned)
      for (int64_t j = 0; j < n_out; ++j) key.insert(key.end(), {lo[j] - x0, w[j] != 0.0 ? 1 : 0});
    for (auto &c : cs) key.insert(key.end(), {c[0] - x0, c[1] - x0, c[2] - j0, c[3] - j0});
    auto it = s->plans.find(key);
    if (it != s->plans.end()) {
      plan = it->second;
      s->plan_hits++;
    } else {
      if (s->plans.size() >= PLAN_CACHE_MAX) {
        LFD_HIP(hipStreamSynchronize(s->s_comp));  // in-flight runs use plan constants
        s->drop_plans();
      }
      std::vector<int64_t> llo(n_out);
      for (int64_t j = 0; j < n_out; ++j) llo[j] = lo[j] - x0;
      std::vector<lfd_chunk> lc(n_rows);
      for (size_t i = 0; i < n_rows; ++i)
        lc[i] = lfd_chunk{cs[i][0] - x0, cs[i][1] - x0, cs[i][2] - j0, cs[i][3] - j0};
      int rc = lfd_lowpass_plan_create(&plan, s->sos.data(), s->n_sec, s->padlen, n_ch, nt, llo.data(),
                                       w.data(), n_out, lc.data(), (int64_t)n_rows);
      if (rc != LFD_OK && rc != LFD_EUNSUPPORTED) return rc;
      if (rc != LFD_OK) plan = nullptr;
      s->plans[key] = plan;
      s->plans_created++;
    }
  }
  if (s->timed) LFD_HIP(hipEventRecord(s->tm[2], s->s_comp));
  if (plan) {
    size_t need = 0;
    LFD_TRY(lfd_lowpass_plan_info(plan, &need, nullptr, nullptr));
    LFD_TRY(ensure_dev(&s->ws, &s->ws_bytes, std::max<size_t>(need, 256), s->s_comp));
    LFD_TRY(lfd::lowpass_execute_gen(plan, x, s->cap, 1, y, n_out, 1, s->ws, s->s_comp,
                                     aligned ? lfd::GridGen{} : gen));
  } else {
    // single-point output, or a grid no block plan takes (more than 32
    // lattice phases): per-chunk general path (still on device)
    for (auto &c : cs) {
      const int64_t m = c[3] - c[2];
      if (m <= 0) continue;
      std::vector<int64_t> clo(m);
      std::vector<double> cw(w.begin() + (c[2] - j0), w.begin() + (c[3] - j0));
      for (int64_t j = 0; j < m; ++j) clo[j] = lo[c[2] - j0 + j] - c[0];
      LFD_TRY(lfd_sos_filtfilt_resample_f32(s->arena[s->cur] + c[0], n_ch, c[1] - c[0] + 1, s->cap, 1,
                                            s->sos.data(), s->n_sec, s->padlen, clo.data(), cw.data(),
                                            m, y + (c[2] - j0), n_out, 1, s->s_comp));
    }
  }
  if (s->timed) LFD_HIP(hipEventRecord(s->tm[3], s->s_comp));
  s->timed_run = s->timed;
  LFD_HIP(hipEventRecord(s->ev_out[oi], s->s_comp));
  s->out_i = oi;
  s->last.y = y;
  return LFD_OK;
}

// low_pass_dascore_edge.ipynb cell 11: process_time_range(t_1, t_2) with
// t_2 = newest sample time, t_1 = start (first run) or last output - buffer.
int run_edge(lfd_stream *s) {
  const int64_t t_hi = s->t_col0 + (s->a_hi - 1) * s->cfg.sample_ns;
  const int64_t t1 = s->produced ? s->last_out_ns - s->cfg.resume_back_ns : s->cfg.t_start_ns;
  const int64_t L = t_hi > t1 ? ceil_div(t_hi - t1, s->out_ns) : 0;
  std::vector<Row> sched;
  if (L < 2 || lfproc_schedule(L, s->cfg.process_patch_size, s->cfg.edge_buff_size, sched) != LFD_OK) {
    fail(LFD_OK, "");  // deferred: no output is possible on this range yet
    return LFD_OK;
  }
  LFD_TRY(run_chunks(s, t1, sched.data(), sched.size()));
  if (s->last.n_out > 0) {
    s->produced = true;
    s->last_out_ns = s->last.t_first_ns + (s->last.n_out - 1) * s->out_ns;
  }
  // keep what the next run selects: time >= its t_1
  const int64_t t_keep = s->produced ? s->last_out_ns - s->cfg.resume_back_ns : s->cfg.t_start_ns;
  s->a_lo = std::min(s->a_hi, std::max(s->a_lo, s->col_ceil(t_keep)));
  return LFD_OK;
}

// One process_time_range(t_start, t_end) over streamed data: run every chunk
// whose selection end has arrived (all remaining ones when flushing).
int run_continuous(lfd_stream *s, bool flush) {
  if (s->next >= s->sched.size() || s->a_hi <= s->a_lo) return LFD_OK;
  const int64_t t_hi = s->t_col0 + (s->a_hi - 1) * s->cfg.sample_ns;
  size_t e = s->next;
  while (e < s->sched.size() && (flush || s->cfg.t_start_ns + s->sched[e][1] * s->out_ns <= t_hi)) ++e;
  if (e == s->next) return LFD_OK;
  LFD_TRY(run_chunks(s, s->cfg.t_start_ns, s->sched.data() + s->next, e - s->next));
  s->next = e;
  if (s->next < s->sched.size())
    s->a_lo = std::min(s->a_hi, std::max(s->a_lo, s->col_ceil(s->cfg.t_start_ns +
                                                              s->sched[s->next][0] * s->out_ns)));
  else
    s->a_lo = s->a_hi;
  return LFD_OK;
}

}  // namespace

extern "C" {

int lfd_lfproc_schedule(int64_t n_grid, int64_t patch_size, int64_t buff_size, int64_t *rows,
                        int64_t max_rows, int64_t *n_rows) {
  std::vector<Row> sched;
  LFD_TRY(lfproc_schedule(n_grid, patch_size, buff_size, sched));
  if (n_rows) *n_rows = (int64_t)sched.size();
  if (rows) {
    if (max_rows < (int64_t)sched.size()) return fail(LFD_EINVAL, "rows buffer too small");
    for (size_t i = 0; i < sched.size(); ++i)
      for (int k = 0; k < 4; ++k) rows[4 * i + k] = sched[i][k];
  }
  return LFD_OK;
}

int lfd_stream_open(lfd_stream **out, const lfd_stream_config *cfg, const double *sos, int n_sec,
                    int padlen) {
  if (!out || !cfg) return fail(LFD_EINVAL, "stream and config must not be NULL");
  *out = nullptr;
  if (!sos || n_sec < 1 || n_sec > lfd::MAX_SEC) return fail(LFD_EINVAL, "sos must hold 1..4 sections");
  if (cfg->n_ch < 1 || cfg->sample_ns < 1) return fail(LFD_EINVAL, "n_ch and sample_ns must be >= 1");
  const int64_t out_ns = (int64_t)(cfg->output_sample_interval * 1000) * 1000000;  // lf_das.py:255
  if (out_ns <= 0) return fail(LFD_EINVAL, "output_sample_interval must be >= 1 ms");
  if (cfg->process_patch_size < 1 || cfg->edge_buff_size < 0)
    return fail(LFD_EINVAL, "process_patch_size must be >= 1 and edge_buff_size >= 0");
  if (cfg->process_patch_size <= 2 * cfg->edge_buff_size)
    return fail(LFD_EINVAL, "process_patch_size must be larger than 2*edge_buff_size");
  if (cfg->mode != LFD_STREAM_EDGE && cfg->mode != LFD_STREAM_CONTINUOUS)
    return fail(LFD_EINVAL, "unknown stream mode");
  auto *s = new lfd_stream();
  s->cfg = *cfg;
  s->sos.assign(sos, sos + 6 * n_sec);
  s->n_sec = n_sec;
  s->padlen = padlen;
  s->out_ns = out_ns;
  s->dry = (cfg->flags & LFD_STREAM_DRY_RUN) != 0;
  {
    const char *v = lfd::knob("LFD_STREAM_DIRECT2D");
    s->direct2d = v && v[0] && v[0] != '0';
  }
  if (cfg->mode == LFD_STREAM_CONTINUOUS) {
    if (cfg->t_end_ns <= cfg->t_start_ns) {
      delete s;
      return fail(LFD_EINVAL, "continuous mode needs t_end_ns > t_start_ns");
    }
    s->n_grid = ceil_div(cfg->t_end_ns - cfg->t_start_ns, out_ns);
    if (int rc = lfproc_schedule(s->n_grid, cfg->process_patch_size, cfg->edge_buff_size, s->sched)) {
      delete s;
      return rc;
    }
  }
  if (!s->dry) {
    hipError_t e = hipGetDevice(&s->device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->s_copy, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->s_comp, hipStreamNonBlocking);
    for (hipEvent_t *ev : {&s->ev_h2d, &s->ev_compact, &s->ev_pin[0], &s->ev_pin[1], &s->ev_out[0], &s->ev_out[1]})
      if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    for (auto &ev : s->tm)
      if (e == hipSuccess) e = hipEventCreate(&ev);
    if (e != hipSuccess) {
      lfd_stream_close(s);
      return fail(LFD_EHIP, std::string("stream setup: ") + hipGetErrorString(e));
    }
  }
  *out = s;
  return LFD_OK;
}

int lfd_stream_reserve(lfd_stream *s, int64_t max_push) {
  if (!s) return fail(LFD_EINVAL, "stream is NULL");
  if (max_push < 1) return fail(LFD_EINVAL, "max_push must be >= 1");
  DeviceGuard g(s->device);
  const int64_t want = round_up(std::max<int64_t>(s->cfg.capacity, 4 * max_push), 64);
  if (want > s->cap) LFD_TRY(alloc_arena(s, want));
  if (!s->dry) LFD_TRY(ensure_stage(s, sizeof(float) * (size_t)max_push * (size_t)s->cfg.n_ch));
  return LFD_OK;
}

int lfd_stream_push(lfd_stream *s, const float *x, int64_t n_t, int64_t s_ch, int64_t s_t, int64_t t0_ns) {
  if (!s) return fail(LFD_EINVAL, "stream is NULL");
  if (n_t < 1) return fail(LFD_EINVAL, "push needs n_t >= 1");
  if (!s->dry && !x) return fail(LFD_EINVAL, "x is NULL");
  if (s_t != 1 && s_ch != 1 && s->cfg.n_ch > 1)
    return fail(LFD_EINVAL, "push needs (channel, time) rows (s_t == 1) or (time, channel) rows (s_ch == 1)");
  if (s_t == 1 && s->cfg.n_ch > 1 && s_ch < n_t) return fail(LFD_EINVAL, "channel stride < n_t");
  if (s_t != 1 && s_t < s->cfg.n_ch) return fail(LFD_EINVAL, "time stride < n_ch");
  DeviceGuard g(s->device);
  s->last = lfd_stream_output{};
  s->last.n_runs = s->n_runs;
  s->last.t_step_ns = s->out_ns;
  s->last_counts.clear();
  s->timed = !s->dry && lfd::timing_enabled();
  s->timed_run = false;
  if (s->have) {
    // the merge rule of Spool.chunk(time=None) (lfdas/core.py _contiguous,
    // tolerance 1.5 samples): a push whose first sample lies within
    // (0, 1.5] sample intervals after the last held sample continues the
    // arena's sample grid (its t0 snaps to the next column, as the resident
    // path's merged patch indexes it); a first sample AT the last held time
    // is a duplicated boundary sample and is dropped; anything else is a gap
    const int64_t dts = s->cfg.sample_ns;
    const int64_t last = s->t_col0 + (s->a_hi - 1) * dts;
    const int64_t gap = t0_ns - last;
    if (gap == 0 && n_t > 0) {
      x += s_t;
      --n_t;
    } else if (!(gap > 0 && 2 * gap <= 3 * dts)) {
      return fail(LFD_EINVAL, "patch merge failed! Gap in data exists");
    }
    t0_ns = last + dts;
  } else {
    s->t_col0 = t0_ns;
    s->a_lo = s->a_hi = 0;
  }
  if (s->cap == 0) {
    const int64_t want = std::max<int64_t>(s->cfg.capacity, 4 * n_t);
    LFD_TRY(alloc_arena(s, round_up(want, 64)));
  } else if (s->a_hi + n_t > s->cap) {
    LFD_TRY(make_room(s, n_t));
  }
  if (!s->dry && n_t > 0) LFD_TRY(copy_in(s, x, n_t, s_ch, s_t));
  s->have = true;
  s->a_hi += n_t;
  return s->cfg.mode == LFD_STREAM_EDGE ? run_edge(s) : run_continuous(s, false);
}

int lfd_stream_flush(lfd_stream *s) {
  if (!s) return fail(LFD_EINVAL, "stream is NULL");
  if (s->cfg.mode != LFD_STREAM_CONTINUOUS) return LFD_OK;
  DeviceGuard g(s->device);
  s->last = lfd_stream_output{};
  s->last.n_runs = s->n_runs;
  s->last.t_step_ns = s->out_ns;
  s->last_counts.clear();
  return run_continuous(s, true);
}

int lfd_stream_last_output(const lfd_stream *s, lfd_stream_output *out) {
  if (!s || !out) return fail(LFD_EINVAL, "NULL argument");
  *out = s->last;
  return LFD_OK;
}

int lfd_stream_last_chunks(const lfd_stream *s, int64_t *counts, int64_t max_chunks, int64_t *n_chunks) {
  if (!s) return fail(LFD_EINVAL, "stream is NULL");
  if (n_chunks) *n_chunks = (int64_t)s->last_counts.size();
  if (counts) {
    if (max_chunks < (int64_t)s->last_counts.size()) return fail(LFD_EINVAL, "counts buffer too small");
    std::copy(s->last_counts.begin(), s->last_counts.end(), counts);
  }
  return LFD_OK;
}

int lfd_stream_fetch(lfd_stream *s, double *y, int64_t ys_ch, int64_t ys_t) {
  if (!s) return fail(LFD_EINVAL, "stream is NULL");
  if (s->dry) return LFD_OK;
  DeviceGuard g(s->device);
  if (s->have) LFD_HIP(hipEventSynchronize(s->ev_h2d));  // the push's host buffer is free again
  if (s->last.n_out == 0) return LFD_OK;
  if (!y) return fail(LFD_EINVAL, "y is NULL");
  const int64_t n_ch = s->cfg.n_ch, n = s->last.n_out;
  LFD_HIP(hipEventSynchronize(s->ev_out[s->out_i]));
  if (ys_t == 1 && (n_ch == 1 || ys_ch >= n)) {
    LFD_HIP(hipMemcpy2DAsync(y, sizeof(double) * (n_ch == 1 ? n : ys_ch), s->last.y, sizeof(double) * n,
                             sizeof(double) * n, n_ch, hipMemcpyDeviceToHost, s->s_comp));
    LFD_HIP(hipStreamSynchronize(s->s_comp));
    return LFD_OK;
  }
  std::vector<double> tmp((size_t)n_ch * n);
  LFD_HIP(hipMemcpyAsync(tmp.data(), s->last.y, sizeof(double) * tmp.size(), hipMemcpyDeviceToHost, s->s_comp));
  LFD_HIP(hipStreamSynchronize(s->s_comp));
  for (int64_t c = 0; c < n_ch; ++c)
    for (int64_t j = 0; j < n; ++j) y[c * ys_ch + j * ys_t] = tmp[c * n + j];
  return LFD_OK;
}

int lfd_stream_wait_copy(lfd_stream *s) {
  if (!s) return fail(LFD_EINVAL, "stream is NULL");
  if (s->dry || !s->have) return LFD_OK;
  DeviceGuard g(s->device);
  LFD_HIP(hipEventSynchronize(s->ev_h2d));
  return LFD_OK;
}

int lfd_stream_synchronize(lfd_stream *s) {
  if (!s) return fail(LFD_EINVAL, "stream is NULL");
  if (s->dry) return LFD_OK;
  DeviceGuard g(s->device);
  LFD_HIP(hipStreamSynchronize(s->s_copy));
  LFD_HIP(hipStreamSynchronize(s->s_comp));
  return LFD_OK;
}

int lfd_stream_last_timing(const lfd_stream *s, float *ms_copy, float *ms_run) {
  if (!s) return fail(LFD_EINVAL, "stream is NULL");
  if (!s->timed) return fail(LFD_EINVAL, "timing was not enabled for the last push");
  DeviceGuard g(s->device);
  float a = 0.f, b = 0.f;
  LFD_HIP(hipEventSynchronize(s->tm[1]));
  LFD_HIP(hipEventElapsedTime(&a, s->tm[0], s->tm[1]));
  if (s->timed_run) {
    LFD_HIP(hipEventSynchronize(s->tm[3]));
    LFD_HIP(hipEventElapsedTime(&b, s->tm[2], s->tm[3]));
  }
  if (ms_copy) *ms_copy = a;
  if (ms_run) *ms_run = b;
  return LFD_OK;
}

int lfd_stream_info(const lfd_stream *s, int64_t *capacity, int64_t *held, int64_t *t_first_held_ns) {
  if (!s) return fail(LFD_EINVAL, "stream is NULL");
  if (capacity) *capacity = s->cap;
  if (held) *held = s->a_hi - s->a_lo;
  if (t_first_held_ns) *t_first_held_ns = s->t_col0 + s->a_lo * s->cfg.sample_ns;
  return LFD_OK;
}

int lfd_debug_stream_plans(const lfd_stream *s, int64_t *created, int64_t *hits) {
  if (!s) return fail(LFD_EINVAL, "stream is NULL");
  if (created) *created = s->plans_created;
  if (hits) *hits = s->plan_hits;
  return LFD_OK;
}

void lfd_stream_close(lfd_stream *s) {
  if (!s) return;
  DeviceGuard g(s->device);
  if (s->s_copy) (void)hipStreamSynchronize(s->s_copy);
  if (s->s_comp) (void)hipStreamSynchronize(s->s_comp);
  s->drop_plans();
  for (void *p : {(void *)s->arena[0], (void *)s->arena[1], (void *)s->stage, (void *)s->out[0],
                  (void *)s->out[1], s->ws})
    if (p) (void)hipFree(p);
  for (auto p : s->pin)
    if (p) (void)hipHostFree(p);
  for (hipEvent_t e : {s->ev_h2d, s->ev_compact, s->ev_pin[0], s->ev_pin[1], s->ev_out[0], s->ev_out[1],
                       s->tm[0], s->tm[1], s->tm[2], s->tm[3]})
    if (e) (void)hipEventDestroy(e);
  for (hipStream_t st : {s->s_copy, s->s_comp})
    if (st) (void)hipStreamDestroy(st);
  delete s;
}

int lfd_host_alloc(void **p, size_t bytes) {
  if (!p) return fail(LFD_EINVAL, "p is NULL");
  *p = nullptr;
  LFD_HIP(hipHostMalloc(p, std::max<size_t>(bytes, 1), hipHostMallocDefault));
  return LFD_OK;
}

void lfd_host_free(void *p) {
  if (p) (void)hipHostFree(p);
}

int lfd_host_register(void *p, size_t bytes) {
  if (!p || !bytes) return fail(LFD_EINVAL, "lfd_host_register: empty range");
  LFD_HIP(hipHostRegister(p, bytes, hipHostRegisterDefault));
  return LFD_OK;
}

int lfd_host_unregister(void *p) {
  if (!p) return fail(LFD_EINVAL, "lfd_host_unregister: p is NULL");
  LFD_HIP(hipHostUnregister(p));
  return LFD_OK;
}

}  // extern "C"
