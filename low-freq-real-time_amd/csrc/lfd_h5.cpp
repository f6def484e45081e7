// DASDAE-layout HDF5 patch files (include/lfdas_h5.h) on the image's libhdf5
// 1.10: the format step of lp_process (lf_das.py:230-232, DASCore's
// io.write(..., "dasdae")) and of get_last_processed_time (lf_das.py:214-217).
// Host-only I/O (no HIP); pytables-style CLASS/VERSION/TITLE attributes are
// written so the file looks like a pytables file to readers that check.
#include <hdf5.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lfdas_h5.h"

namespace {

thread_local std::string g_err;

int fail(const std::string &m) {
  g_err = m;
  return -1;
}

struct Quiet {  // HDF5 prints its error stack to stderr by default
  Quiet() { H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr); }
};

// RAII for hid_t handles
struct H {
  hid_t id = -1;
  herr_t (*close)(hid_t) = nullptr;
  H(hid_t i, herr_t (*c)(hid_t)) : id(i), close(c) {}
  ~H() {
    if (id >= 0 && close) close(id);
  }
  H(const H &) = delete;
  H &operator=(const H &) = delete;
  operator hid_t() const { return id; }
  bool ok() const { return id >= 0; }
};

bool put_str_attr(hid_t obj, const char *name, const char *value) {
  const size_t n = std::max<size_t>(1, std::strlen(value));
  H t(H5Tcopy(H5T_C_S1), H5Tclose);
  if (!t.ok() || H5Tset_size(t, n) < 0 || H5Tset_strpad(t, H5T_STR_NULLPAD) < 0) return false;
  H sp(H5Screate(H5S_SCALAR), H5Sclose);
  H a(H5Acreate2(obj, name, t, sp, H5P_DEFAULT, H5P_DEFAULT), H5Aclose);
  std::string buf(value);
  buf.resize(n, '\0');
  return a.ok() && H5Awrite(a, t, buf.data()) >= 0;
}

template <class T>
bool put_num_attr(hid_t obj, const char *name, hid_t type, T v) {
  H sp(H5Screate(H5S_SCALAR), H5Sclose);
  H a(H5Acreate2(obj, name, type, sp, H5P_DEFAULT, H5P_DEFAULT), H5Aclose);
  return a.ok() && H5Awrite(a, type, &v) >= 0;
}

hid_t bool_type() {  // pytables stores numpy bool as a 1-byte enum {FALSE, TRUE}
  hid_t t = H5Tenum_create(H5T_NATIVE_INT8);
  int8_t v = 0;
  H5Tenum_insert(t, "FALSE", &v);
  v = 1;
  H5Tenum_insert(t, "TRUE", &v);
  return t;
}

bool put_bool_attr(hid_t obj, const char *name, bool v) {
  H t(bool_type(), H5Tclose);
  const int8_t b = v ? 1 : 0;
  return put_num_attr(obj, name, t, b);
}

bool pytables_group(hid_t g) {
  return put_str_attr(g, "CLASS", "GROUP") && put_str_attr(g, "TITLE", "") && put_str_attr(g, "VERSION", "1.0");
}

bool pytables_array(hid_t d) {
  return put_str_attr(d, "CLASS", "ARRAY") && put_str_attr(d, "FLAVOR", "numpy") &&
         put_str_attr(d, "TITLE", "") && put_str_attr(d, "VERSION", "2.4");
}

bool write_array(hid_t g, const char *name, hid_t mem_type, hid_t file_type, int rank, const hsize_t *dims,
                 const void *data, int kind) {
  H sp(H5Screate_simple(rank, dims, nullptr), H5Sclose);
  H d(H5Dcreate2(g, name, file_type, sp, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT), H5Dclose);
  if (!d.ok()) return false;
  if (H5Dwrite(d, mem_type, H5S_ALL, H5S_ALL, H5P_DEFAULT, data) < 0) return false;
  return pytables_array(d) && put_bool_attr(d, "is_datetime64", kind == LFDH5_DT64) &&
         put_bool_attr(d, "is_timedelta64", kind == LFDH5_TD64);
}

std::string read_str_attr(hid_t a) {
  H t(H5Aget_type(a), H5Tclose);
  std::string out;
  if (H5Tis_variable_str(t) > 0) {
    char *p = nullptr;
    H mt(H5Tcopy(H5T_C_S1), H5Tclose);
    H5Tset_size(mt, H5T_VARIABLE);
    if (H5Aread(a, mt, &p) >= 0 && p) {
      out = p;
      H5free_memory(p);
    }
    return out;
  }
  const size_t n = H5Tget_size(t);
  std::vector<char> buf(n + 1, '\0');
  if (H5Aread(a, t, buf.data()) < 0) return out;
  return std::string(buf.data());
}

bool read_bool_attr(hid_t obj, const char *name) {
  if (H5Aexists(obj, name) <= 0) return false;
  H a(H5Aopen(obj, name, H5P_DEFAULT), H5Aclose);
  int8_t v = 0;
  H t(H5Aget_type(a), H5Tclose);
  if (H5Tget_size(t) != 1) return false;
  H mt(bool_type(), H5Tclose);
  return H5Aread(a, H5Tget_class(t) == H5T_ENUM ? (hid_t)mt : H5T_NATIVE_INT8, &v) >= 0 && v != 0;
}

herr_t collect_link(hid_t, const char *name, const H5L_info_t *, void *op) {
  static_cast<std::vector<std::string> *>(op)->push_back(name);
  return 0;
}

herr_t collect_attr(hid_t, const char *name, const H5A_info_t *, void *op) {
  static_cast<std::vector<std::string> *>(op)->push_back(name);
  return 0;
}

}  // namespace

struct lfdh5_file {
  hid_t file = -1, group = -1;
  int64_t n0 = 0, n1 = 0;
  std::string dims;
  std::vector<std::string> coords;  // dataset names without the _coord_ prefix
  std::vector<std::string> attrs;   // attribute keys without the _attrs_ prefix
};

extern "C" {

const char *lfdh5_last_error(void) { return g_err.c_str(); }

int lfdh5_write_patch(const char *path, const char *group, const double *data, int64_t n0, int64_t n1,
                      const char *dims_csv, const lfdh5_coord *coords, int n_coords,
                      const lfdh5_attr *attrs, int n_attrs) {
  Quiet q;
  if (!path || !group || !data || !dims_csv || n0 < 0 || n1 < 0) return fail("bad arguments");
  H f(H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT), H5Fclose);
  if (!f.ok()) return fail(std::string("cannot create ") + path);
  H root(H5Gopen2(f, "/", H5P_DEFAULT), H5Gclose);
  if (!pytables_group(root) || !put_str_attr(root, "PYTABLES_FORMAT_VERSION", "2.1") ||
      !put_str_attr(root, "__format__", "DASDAE") || !put_str_attr(root, "__DASDAE_version__", "1"))
    return fail("root attributes");
  H wf(H5Gcreate2(f, "/waveforms", H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT), H5Gclose);
  if (!wf.ok() || !pytables_group(wf)) return fail("/waveforms group");
  H g(H5Gcreate2(wf, group, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT), H5Gclose);
  if (!g.ok() || !pytables_group(g)) return fail(std::string("patch group ") + group);
  if (!put_str_attr(g, "_dims", dims_csv)) return fail("_dims attribute");
  for (int i = 0; i < n_attrs; ++i) {
    const lfdh5_attr &a = attrs[i];
    const std::string key = std::string("_attrs_") + a.name;
    bool ok = false;
    switch (a.kind) {
      case LFDH5_STR: ok = put_str_attr(g, key.c_str(), a.s ? a.s : ""); break;
      case LFDH5_F64: ok = put_num_attr(g, key.c_str(), H5T_NATIVE_DOUBLE, a.f); break;
      case LFDH5_I64: ok = put_num_attr(g, key.c_str(), H5T_NATIVE_INT64, a.i); break;
      case LFDH5_BOOL: ok = put_bool_attr(g, key.c_str(), a.i != 0); break;
      case LFDH5_DT64:
      case LFDH5_TD64:
        ok = put_num_attr(g, key.c_str(), H5T_NATIVE_INT64, a.i) &&
             put_str_attr(g, (std::string("_dtypes_") + a.name).c_str(),
                          a.kind == LFDH5_DT64 ? "datetime64[ns]" : "timedelta64[ns]");
        break;
      default: return fail(std::string("attribute kind of ") + a.name);
    }
    if (!ok) return fail(std::string("attribute ") + a.name);
  }
  const hsize_t dshape[2] = {(hsize_t)n0, (hsize_t)n1};
  if (!write_array(g, "data", H5T_NATIVE_DOUBLE, H5T_IEEE_F64LE, 2, dshape, data, LFDH5_F64))
    return fail("data array");
  for (int i = 0; i < n_coords; ++i) {
    const lfdh5_coord &c = coords[i];
    const hsize_t n = (hsize_t)c.len;
    const std::string name = std::string("_coord_") + c.name;
    const bool f64 = c.kind == LFDH5_F64;
    if (!write_array(g, name.c_str(), f64 ? H5T_NATIVE_DOUBLE : H5T_NATIVE_INT64,
                     f64 ? H5T_IEEE_F64LE : H5T_STD_I64LE, 1, &n, c.data, c.kind))
      return fail("coordinate " + name);
  }
  if (H5Fflush(f, H5F_SCOPE_GLOBAL) < 0) return fail("flush");
  return 0;
}

int lfdh5_open(const char *path, lfdh5_file **out, int64_t *n0, int64_t *n1, int *n_coords, int *n_attrs) {
  Quiet q;
  if (!out) return fail("out is NULL");
  *out = nullptr;
  hid_t f = H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT);
  if (f < 0) return fail(std::string("cannot open ") + path);
  auto *h = new lfdh5_file();
  h->file = f;
  auto bad = [&](const std::string &m) {
    lfdh5_close(h);
    return fail(m);
  };
  if (H5Lexists(f, "/waveforms", H5P_DEFAULT) <= 0) return bad("no /waveforms group (not a DASDAE file)");
  std::vector<std::string> names;
  {
    H wf(H5Gopen2(f, "/waveforms", H5P_DEFAULT), H5Gclose);
    hsize_t idx = 0;
    H5Literate(wf, H5_INDEX_NAME, H5_ITER_INC, &idx, collect_link, &names);
    if (names.empty()) return bad("/waveforms holds no patch");
    h->group = H5Gopen2(wf, names[0].c_str(), H5P_DEFAULT);
  }
  if (h->group < 0) return bad("cannot open the patch group");
  {
    H d(H5Dopen2(h->group, "data", H5P_DEFAULT), H5Dclose);
    if (!d.ok()) return bad("patch has no data array");
    H sp(H5Dget_space(d), H5Sclose);
    hsize_t dims[2] = {0, 0};
    if (H5Sget_simple_extent_ndims(sp) != 2) return bad("data is not 2-D");
    H5Sget_simple_extent_dims(sp, dims, nullptr);
    h->n0 = (int64_t)dims[0];
    h->n1 = (int64_t)dims[1];
  }
  if (H5Aexists(h->group, "_dims") > 0) {
    H a(H5Aopen(h->group, "_dims", H5P_DEFAULT), H5Aclose);
    h->dims = read_str_attr(a);
  }
  std::vector<std::string> links;
  hsize_t idx = 0;
  H5Literate(h->group, H5_INDEX_NAME, H5_ITER_INC, &idx, collect_link, &links);
  for (const auto &l : links)
    if (l.rfind("_coord_", 0) == 0) h->coords.push_back(l.substr(7));
  std::vector<std::string> anames;
  H5Aiterate2(h->group, H5_INDEX_NAME, H5_ITER_INC, nullptr, collect_attr, &anames);
  for (const auto &a : anames)
    if (a.rfind("_attrs_", 0) == 0) h->attrs.push_back(a.substr(7));
  if (n0) *n0 = h->n0;
  if (n1) *n1 = h->n1;
  if (n_coords) *n_coords = (int)h->coords.size();
  if (n_attrs) *n_attrs = (int)h->attrs.size();
  *out = h;
  return 0;
}

int lfdh5_read_data(lfdh5_file *h, double *out) {
  Quiet q;
  if (!h || !out) return fail("NULL argument");
  H d(H5Dopen2(h->group, "data", H5P_DEFAULT), H5Dclose);
  if (!d.ok() || H5Dread(d, H5T_NATIVE_DOUBLE, H5S_ALL, H5S_ALL, H5P_DEFAULT, out) < 0)
    return fail("reading data");
  return 0;
}

int lfdh5_dims(lfdh5_file *h, char *buf, int cap) {
  if (!h || !buf || cap < 1) return fail("NULL argument");
  std::snprintf(buf, (size_t)cap, "%s", h->dims.c_str());
  return 0;
}

int lfdh5_coord_info(lfdh5_file *h, int i, char *name, int cap, int *kind, int64_t *len) {
  Quiet q;
  if (!h || i < 0 || i >= (int)h->coords.size()) return fail("coordinate index");
  const std::string ds = "_coord_" + h->coords[i];
  H d(H5Dopen2(h->group, ds.c_str(), H5P_DEFAULT), H5Dclose);
  if (!d.ok()) return fail("open " + ds);
  H sp(H5Dget_space(d), H5Sclose);
  hsize_t n = 0;
  H5Sget_simple_extent_dims(sp, &n, nullptr);
  H t(H5Dget_type(d), H5Tclose);
  int k = H5Tget_class(t) == H5T_FLOAT ? LFDH5_F64 : LFDH5_I64;
  if (read_bool_attr(d, "is_datetime64")) k = LFDH5_DT64;
  if (read_bool_attr(d, "is_timedelta64")) k = LFDH5_TD64;
  if (name && cap > 0) std::snprintf(name, (size_t)cap, "%s", h->coords[i].c_str());
  if (kind) *kind = k;
  if (len) *len = (int64_t)n;
  return 0;
}

int lfdh5_coord_read(lfdh5_file *h, int i, void *out) {
  Quiet q;
  int kind = 0;
  if (lfdh5_coord_info(h, i, nullptr, 0, &kind, nullptr) < 0) return -1;
  const std::string ds = "_coord_" + h->coords[i];
  H d(H5Dopen2(h->group, ds.c_str(), H5P_DEFAULT), H5Dclose);
  if (H5Dread(d, kind == LFDH5_F64 ? H5T_NATIVE_DOUBLE : H5T_NATIVE_INT64, H5S_ALL, H5S_ALL, H5P_DEFAULT,
              out) < 0)
    return fail("read " + ds);
  return 0;
}

int lfdh5_attr_info(lfdh5_file *h, int i, char *name, int cap, int *kind, char *sbuf, int scap, double *fv,
                    int64_t *iv) {
  Quiet q;
  if (!h || i < 0 || i >= (int)h->attrs.size()) return fail("attribute index");
  const std::string key = h->attrs[i];
  const std::string an = "_attrs_" + key;
  H a(H5Aopen(h->group, an.c_str(), H5P_DEFAULT), H5Aclose);
  if (!a.ok()) return fail("open attribute " + an);
  H t(H5Aget_type(a), H5Tclose);
  const H5T_class_t cls = H5Tget_class(t);
  int k = LFDH5_STR;
  if (name && cap > 0) std::snprintf(name, (size_t)cap, "%s", key.c_str());
  if (cls == H5T_STRING) {
    const std::string v = read_str_attr(a);
    if (sbuf && scap > 0) std::snprintf(sbuf, (size_t)scap, "%s", v.c_str());
  } else if (cls == H5T_FLOAT) {
    k = LFDH5_F64;
    double v = 0;
    H5Aread(a, H5T_NATIVE_DOUBLE, &v);
    if (fv) *fv = v;
  } else if (cls == H5T_ENUM) {
    k = LFDH5_BOOL;
    if (iv) *iv = read_bool_attr(h->group, an.c_str()) ? 1 : 0;
  } else if (cls == H5T_INTEGER) {
    k = LFDH5_I64;
    int64_t v = 0;
    H5Aread(a, H5T_NATIVE_INT64, &v);
    if (iv) *iv = v;
    const std::string dn = "_dtypes_" + key;
    if (H5Aexists(h->group, dn.c_str()) > 0) {
      H da(H5Aopen(h->group, dn.c_str(), H5P_DEFAULT), H5Aclose);
      const std::string dt = read_str_attr(da);
      if (dt == "datetime64[ns]") k = LFDH5_DT64;
      if (dt == "timedelta64[ns]") k = LFDH5_TD64;
    }
  } else {
    return fail("unsupported attribute type of " + an);
  }
  if (kind) *kind = k;
  return 0;
}

void lfdh5_close(lfdh5_file *h) {
  if (!h) return;
  if (h->group >= 0) H5Gclose(h->group);
  if (h->file >= 0) H5Fclose(h->file);
  delete h;
}

}  // extern "C"
