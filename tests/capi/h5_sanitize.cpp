// Host-side sanitizer driver for lfd_h5.cpp (ASan + UBSan): the
// DASDAE-layout round trip of lf_das.py:230-232 / :214-217 through
// include/lfdas_h5.h — write a patch with every coordinate and attribute
// kind, read it back (data, dims, coords, attrs, including too-small name /
// string buffers), and the error paths (missing file, bad arguments).
// Built and run by tests/test_sanitize.py (tools/sanitize.sh).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lfdas_h5.h"

#define CHECK(x)                                                                                      \
  do {                                                                                                \
    int rc_ = (x);                                                                                    \
    if (rc_ != 0) {                                                                                   \
      std::fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_, lfdh5_last_error()); \
      std::exit(1);                                                                                   \
    }                                                                                                 \
  } while (0)

int main(int argc, char **argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const std::string path = dir + "/lfd_h5_sanitize.h5";
  const int64_t n0 = 7, n1 = 33;
  std::vector<double> data((size_t)(n0 * n1));
  for (size_t i = 0; i < data.size(); ++i) data[i] = std::sin(0.1 * (double)i) + (i % 5 == 0 ? NAN : 0.0);
  std::vector<double> dist(n0);
  std::vector<int64_t> tm(n1), td(n1);
  for (int64_t i = 0; i < n0; ++i) dist[i] = 10.0 * (double)i;
  for (int64_t j = 0; j < n1; ++j) {
    tm[j] = 1505692800000000000LL + j * 1000000000LL;
    td[j] = j * 1000000000LL;
  }
  const lfdh5_coord coords[3] = {{"distance", LFDH5_F64, n0, dist.data()},
                                 {"time", LFDH5_DT64, n1, tm.data()},
                                 {"lag", LFDH5_TD64, n1, td.data()}};
  const lfdh5_attr attrs[5] = {{"station", LFDH5_STR, "LFDAS_test_station_name", 0.0, 0},
                               {"d_time", LFDH5_F64, nullptr, 1.0, 0},
                               {"n_samples", LFDH5_I64, nullptr, 0.0, 42},
                               {"flag", LFDH5_BOOL, nullptr, 0.0, 1},
                               {"time_min", LFDH5_DT64, nullptr, 0.0, tm[0]}};
  CHECK(lfdh5_write_patch(path.c_str(), "DAS__LF__2017-09-18T00_00_00", data.data(), n0, n1, "distance,time",
                          coords, 3, attrs, 5));
  lfdh5_file *f = nullptr;
  int64_t r0 = 0, r1 = 0;
  int nc = 0, na = 0;
  CHECK(lfdh5_open(path.c_str(), &f, &r0, &r1, &nc, &na));
  if (r0 != n0 || r1 != n1 || nc != 3 || na < 5) {
    std::fprintf(stderr, "shape/count mismatch %lld %lld %d %d\n", (long long)r0, (long long)r1, nc, na);
    return 1;
  }
  std::vector<double> back((size_t)(n0 * n1));
  CHECK(lfdh5_read_data(f, back.data()));
  for (size_t i = 0; i < back.size(); ++i)
    if (!(back[i] == data[i] || (std::isnan(back[i]) && std::isnan(data[i])))) {
      std::fprintf(stderr, "data mismatch at %zu\n", i);
      return 1;
    }
  char dims[64], tiny[4];
  CHECK(lfdh5_dims(f, dims, sizeof dims));
  (void)lfdh5_dims(f, tiny, sizeof tiny);  // truncated or an error, never an overrun
  for (int i = 0; i < nc; ++i) {
    char name[64];
    int kind = -1;
    int64_t len = 0;
    CHECK(lfdh5_coord_info(f, i, name, sizeof name, &kind, &len));
    (void)lfdh5_coord_info(f, i, tiny, sizeof tiny, &kind, &len);
    std::vector<int64_t> buf((size_t)len + 1);
    CHECK(lfdh5_coord_read(f, i, buf.data()));
  }
  for (int i = 0; i < na; ++i) {
    char name[64], sbuf[64];
    int kind = -1;
    double fv = 0.0;
    int64_t iv = 0;
    CHECK(lfdh5_attr_info(f, i, name, sizeof name, &kind, sbuf, sizeof sbuf, &fv, &iv));
    (void)lfdh5_attr_info(f, i, tiny, sizeof tiny, &kind, tiny, sizeof tiny, &fv, &iv);
  }
  if (lfdh5_coord_info(f, nc + 3, dims, sizeof dims, nullptr, nullptr) == 0) return 1;
  lfdh5_close(f);
  if (lfdh5_open((dir + "/no_such_file.h5").c_str(), &f, &r0, &r1, &nc, &na) == 0) return 1;
  if (lfdh5_write_patch(path.c_str(), "g", nullptr, n0, n1, "distance,time", coords, 3, attrs, 5) == 0) return 1;
  std::remove(path.c_str());
  std::printf("h5 sanitize driver: ok\n");
  return 0;
}
