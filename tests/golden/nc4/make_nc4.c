/*
 * make_nc4.c -- writes the netCDF-4 (HDF5) fixtures of tests/test_nc4read.py with
 * the HDF5 library found in this image (/opt/conda/lib/libhdf5 1.10.6; there is
 * no netCDF library), following the netCDF-4 conventions the netCDF-C library
 * uses when it creates a file (libhdf5/hdf5create.c, hdf5var.c): libver bounds
 * (EARLIEST, V18), link and attribute creation order tracked + indexed, every
 * dimension a dataset marked as an HDF5 dimension scale (coordinate variables
 * are the scale itself), _Netcdf4Dimid on each scale, _NCProperties on the root.
 * Variants cover the storage the reader must decode:
 *   rfm_nc4.nc        netCDF-4 layout, 7 links (compact link messages):
 *                     contiguous f64 axes, chunked+shuffle+deflate f64 (CO2),
 *                     contiguous f32 (H2O), chunked big-endian f64 (O3)
 *   rfm_nc4_dense.nc  + 10 variables: dense links (fractal heap, v2 B-tree leaf)
 *   rfm_nc4_many.nc   + 60 variables: v2 B-tree of depth 1, heap with indirect rows
 *   rfm_latest.nc     libver LATEST: superblock v3, layout v4 (fixed-array,
 *                     single-chunk (filtered) and implicit chunk indexes)
 *   rfm_v0.nc         libver EARLIEST, no creation order: superblock v0, symbol-
 *                     table group, v1 object headers, B-tree v1 chunks, compact
 *   weights_nc4.nc    dimension + variable "weights" (read_weights.cpp:18-46)
 * Values: v(var, i) = sin(0.37 i + var) * 10^((i % 7) - 3) + var, i = C-order index;
 * Pressure (var 2): 10^(5 - 0.4 i) * (1 + 0.05 sin(0.37 i + 2)) (positive, decreasing).
 *
 *   gcc make_nc4.c -I/opt/conda/include -L/opt/conda/lib -lhdf5_hl -lhdf5 \
 *       -Wl,-rpath,/opt/conda/lib -lm -o make_nc4 && ./make_nc4 OUTDIR
 * (tests/golden/nc4/make.sh)
 */
#include <hdf5.h>
#include <hdf5_hl.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NW 37
#define NP 11
#define NT 5

/* Pressure (var 2) is a strictly positive, decreasing axis, as RFM.reset takes its log */
static double val(int var, long i) {
  if (var == 2) return pow(10.0, 5.0 - 0.4 * (double)i) * (1.0 + 0.05 * sin(0.37 * i + var));
  return sin(0.37 * i + var) * pow(10.0, (double)(i % 7) - 3.0) + var;
}

static void check(herr_t e, const char* what) {
  if (e < 0) {
    fprintf(stderr, "make_nc4: %s failed\n", what);
    exit(1);
  }
}

static hid_t new_file(const char* dir, const char* name, int mode) {
  /* mode 0: netCDF-4 conventions, 1: libver LATEST, 2: libver EARLIEST without creation order */
  char path[1024];
  snprintf(path, sizeof(path), "%s/%s", dir, name);
  hid_t fapl = H5Pcreate(H5P_FILE_ACCESS);
  hid_t fcpl = H5Pcreate(H5P_FILE_CREATE);
  if (mode == 0) {
    check(H5Pset_libver_bounds(fapl, H5F_LIBVER_EARLIEST, H5F_LIBVER_V18), "libver");
    check(H5Pset_link_creation_order(fcpl, H5P_CRT_ORDER_TRACKED | H5P_CRT_ORDER_INDEXED), "lco");
    check(H5Pset_attr_creation_order(fcpl, H5P_CRT_ORDER_TRACKED | H5P_CRT_ORDER_INDEXED), "aco");
  } else if (mode == 1) {
    check(H5Pset_libver_bounds(fapl, H5F_LIBVER_LATEST, H5F_LIBVER_LATEST), "libver");
    check(H5Pset_link_creation_order(fcpl, H5P_CRT_ORDER_TRACKED | H5P_CRT_ORDER_INDEXED), "lco");
  }
  hid_t f = H5Fcreate(path, H5F_ACC_TRUNC, fcpl, fapl);
  check(f, path);
  H5Pclose(fapl);
  H5Pclose(fcpl);
  if (mode == 0) {
    const char* props = "version=2,netcdf=4.7.4,hdf5=1.10.6";
    check(H5LTset_attribute_string(f, "/", "_NCProperties", props), "_NCProperties");
  }
  return f;
}

/* dataset `name` of the given file type and rank, values val(var, i) */
static hid_t put(hid_t f, const char* name, int var, hid_t ftype, int rank, const hsize_t* dims,
                 const hsize_t* chunk, int shuffle, int deflate, int layout_compact, int early,
                 int mode) {
  hid_t sp = H5Screate_simple(rank, dims, NULL);
  hid_t dcpl = H5Pcreate(H5P_DATASET_CREATE);
  if (mode == 0) H5Pset_attr_creation_order(dcpl, H5P_CRT_ORDER_TRACKED | H5P_CRT_ORDER_INDEXED);
  if (chunk) {
    check(H5Pset_chunk(dcpl, rank, chunk), "chunk");
    if (shuffle) check(H5Pset_shuffle(dcpl), "shuffle");
    if (deflate) check(H5Pset_deflate(dcpl, deflate), "deflate");
  }
  if (layout_compact) check(H5Pset_layout(dcpl, H5D_COMPACT), "compact");
  if (early) check(H5Pset_alloc_time(dcpl, H5D_ALLOC_TIME_EARLY), "alloc");
  hid_t d = H5Dcreate2(f, name, ftype, sp, H5P_DEFAULT, dcpl, H5P_DEFAULT);
  check(d, name);
  long n = 1;
  for (int k = 0; k < rank; ++k) n *= (long)dims[k];
  double* buf = (double*)malloc(sizeof(double) * n);
  for (long i = 0; i < n; ++i) buf[i] = val(var, i);
  check(H5Dwrite(d, H5T_NATIVE_DOUBLE, H5S_ALL, H5S_ALL, H5P_DEFAULT, buf), "write");
  free(buf);
  H5Pclose(dcpl);
  H5Sclose(sp);
  return d;
}

static void dimid(hid_t d, int id) {
  hid_t sp = H5Screate(H5S_SCALAR);
  hid_t a = H5Acreate2(d, "_Netcdf4Dimid", H5T_NATIVE_INT, sp, H5P_DEFAULT, H5P_DEFAULT);
  check(H5Awrite(a, H5T_NATIVE_INT, &id), "dimid");
  H5Aclose(a);
  H5Sclose(sp);
}

/* the RFM table (rfm.cpp:34-120): axes, reference temperature, species k tables */
static void rfm_file(const char* dir, const char* name, int mode, int extra) {
  hid_t f = new_file(dir, name, mode);
  hsize_t dw[1] = {NW}, dp[1] = {NP}, dt[1] = {NT}, d3[3] = {NW, NP, NT};
  hsize_t c3[3] = {8, 4, NT};
  hid_t w = put(f, "Wavenumber", 1, H5T_IEEE_F64LE, 1, dw, NULL, 0, 0, 0, 0, mode);
  hid_t p = put(f, "Pressure", 2, H5T_IEEE_F64LE, 1, dp, NULL, 0, 0, 0, 0, mode);
  hid_t t = put(f, "TempGrid", 3, H5T_IEEE_F64LE, 1, dt, NULL, 0, 0, 0, 0, mode);
  hid_t tr = put(f, "Temperature", 4, H5T_IEEE_F64LE, 1, dp, NULL, 0, 0, mode == 2, 0, mode);
  hid_t co2 = put(f, "CO2", 5, H5T_IEEE_F64LE, 3, d3, c3, 1, 4, 0, 0, mode);
  hid_t h2o = put(f, "H2O", 6, H5T_IEEE_F32LE, 3, d3, NULL, 0, 0, 0, 0, mode);
  hsize_t c3b[3] = {16, NP, 2};
  hid_t o3 = put(f, "O3", 7, H5T_IEEE_F64BE, 3, d3, c3b, 0, 0, 0, mode == 1, mode);
  if (mode == 1) {  /* one chunk covering the whole (filtered) dataset: single-chunk index */
    hsize_t c1[3] = {NW, NP, NT};
    H5Dclose(put(f, "N2O", 8, H5T_IEEE_F64LE, 3, d3, c1, 1, 6, 0, 0, mode));
  }
  if (mode == 0) {
    check(H5DSset_scale(w, "Wavenumber"), "scale");
    check(H5DSset_scale(p, "Pressure"), "scale");
    check(H5DSset_scale(t, "TempGrid"), "scale");
    dimid(w, 0);
    dimid(p, 1);
    dimid(t, 2);
    hid_t vars3[3] = {co2, h2o, o3};
    for (int v = 0; v < 3; ++v) {
      check(H5DSattach_scale(vars3[v], w, 0), "attach");
      check(H5DSattach_scale(vars3[v], p, 1), "attach");
      check(H5DSattach_scale(vars3[v], t, 2), "attach");
    }
    check(H5DSattach_scale(tr, p, 0), "attach");
  }
  for (int x = 0; x < extra; ++x) {
    char nm[32];
    snprintf(nm, sizeof(nm), "X%02d", x);
    hsize_t dx[1] = {(hsize_t)(3 + x % 5)};
    hid_t d = put(f, nm, 100 + x, x % 2 ? H5T_STD_I32LE : H5T_IEEE_F64LE, 1, dx, NULL, 0, 0, 0,
                  0, mode);
    H5Dclose(d);
  }
  H5Dclose(w);
  H5Dclose(p);
  H5Dclose(t);
  H5Dclose(tr);
  H5Dclose(co2);
  H5Dclose(h2o);
  H5Dclose(o3);
  H5Fclose(f);
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : ".";
  rfm_file(dir, "rfm_nc4.nc", 0, 0);
  rfm_file(dir, "rfm_nc4_dense.nc", 0, 10);
  rfm_file(dir, "rfm_nc4_many.nc", 0, 60);
  rfm_file(dir, "rfm_latest.nc", 1, 0);
  rfm_file(dir, "rfm_v0.nc", 2, 0);
  {
    hid_t f = new_file(dir, "weights_nc4.nc", 0);
    hsize_t dw[1] = {16};
    hid_t d = put(f, "weights", 9, H5T_IEEE_F64LE, 1, dw, NULL, 0, 0, 0, 0, 0);
    check(H5DSset_scale(d, "weights"), "scale");
    dimid(d, 0);
    H5Dclose(d);
    H5Fclose(f);
  }
  return 0;
}
