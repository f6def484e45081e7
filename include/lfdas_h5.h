/*
 * lfdas_h5.h — DASDAE-layout HDF5 patch files (liblfdas_h5.so, built from
 * low-freq-real-time_amd/csrc/lfd_h5.cpp against the image's libhdf5 1.10).
 *
 * Replaces the reference's output/input format step:
 *   lf_das.py:230-232   lfDAS.io.write(filename, "dasdae")   (DASCore → pytables)
 *   lf_das.py:214-217   dc.spool(output_folder).update(); out_sp[-1].attrs["time_max"]
 *
 * Layout written (DASCore's DASDAE v1 writer, restated from its public
 * source — DASCore/pytables are not installed here, so byte-level
 * compatibility with DASCore's reader is unpinned):
 *   /                       attrs __format__ = "DASDAE", __DASDAE_version__ = "1"
 *   /waveforms/<group>/     attrs _dims = "distance,time", _attrs_<key> = value
 *   /waveforms/<group>/data             float64 array in dims order
 *   /waveforms/<group>/_coord_<name>    coordinate arrays (datetime64 /
 *                                       timedelta64 as int64 ns with attrs
 *                                       is_datetime64 / is_timedelta64)
 * All calls return 0 or a negative code; lfdh5_last_error() explains.
 */
#ifndef LFDAS_H5_H
#define LFDAS_H5_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LFDH5_STR 0  /* attribute string                         */
#define LFDH5_F64 1  /* float64                                  */
#define LFDH5_I64 2  /* int64                                    */
#define LFDH5_BOOL 3 /* bool                                     */
#define LFDH5_DT64 4 /* datetime64[ns] as int64 ns since epoch   */
#define LFDH5_TD64 5 /* timedelta64[ns] as int64 ns              */

typedef struct lfdh5_attr {
  const char *name;
  int kind;
  const char *s; /* LFDH5_STR */
  double f;      /* LFDH5_F64 */
  int64_t i;     /* LFDH5_I64 / BOOL / DT64 / TD64 */
} lfdh5_attr;

typedef struct lfdh5_coord {
  const char *name;
  int kind;       /* LFDH5_F64, LFDH5_I64, LFDH5_DT64 or LFDH5_TD64 */
  int64_t len;
  const void *data; /* double[len] or int64_t[len] */
} lfdh5_coord;

const char *lfdh5_last_error(void);

/* Create (truncate) `path` holding one patch: data (n0, n1) float64 in
 * row-major dims order, dims_csv "distance,time". */
int lfdh5_write_patch(const char *path, const char *group, const double *data, int64_t n0, int64_t n1,
                      const char *dims_csv, const lfdh5_coord *coords, int n_coords,
                      const lfdh5_attr *attrs, int n_attrs);

/* Reader of the first patch of a file written in this layout. */
typedef struct lfdh5_file lfdh5_file;
int lfdh5_open(const char *path, lfdh5_file **f, int64_t *n0, int64_t *n1, int *n_coords, int *n_attrs);
int lfdh5_read_data(lfdh5_file *f, double *out);
int lfdh5_dims(lfdh5_file *f, char *buf, int cap);
int lfdh5_coord_info(lfdh5_file *f, int i, char *name, int cap, int *kind, int64_t *len);
int lfdh5_coord_read(lfdh5_file *f, int i, void *out);
int lfdh5_attr_info(lfdh5_file *f, int i, char *name, int cap, int *kind, char *sbuf, int scap, double *fv,
                    int64_t *iv);
void lfdh5_close(lfdh5_file *f);

#ifdef __cplusplus
}
#endif
#endif /* LFDAS_H5_H */
