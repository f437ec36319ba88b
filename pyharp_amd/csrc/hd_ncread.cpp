// hd_ncread.cpp -- include/hdnc.h over the header-only readers of
// include/harp_amd/ncread.hpp (classic and netCDF-4 / HDF5 files).
#include <exception>
#include <memory>
#include <string>

#include "../../include/harp_amd/ncread.hpp"
#include "../../include/hdisort.h"
#include "../../include/hdnc.h"
#include "hd_kernels.hpp"

struct hd_ncfile {
  std::unique_ptr<harp_amd::NetCDFFile> nc;
};

namespace {
template <class F>
int guarded(const char* what, F&& f) {
  try {
    return f();
  } catch (std::exception const& e) {
    return hd::set_global_error(HD_EINVAL, "%s: %s", what, e.what());
  }
}
}  // namespace

extern "C" {

int hd_nc_open(const char* path, hd_ncfile** out, int* netcdf4) {
  if (!path || !out) return hd::set_global_error(HD_EINVAL, "hd_nc_open: null argument");
  *out = nullptr;
  return guarded("hd_nc_open", [&] {
    auto f = std::make_unique<hd_ncfile>();
    f->nc = std::make_unique<harp_amd::NetCDFFile>(path);
    if (netcdf4) *netcdf4 = f->nc->netcdf4() ? 1 : 0;
    *out = f.release();
    return HD_OK;
  });
}

int hd_nc_close(hd_ncfile* f) {
  delete f;
  return HD_OK;
}

int hd_nc_dim_len(const hd_ncfile* f, const char* name, long* len) {
  if (!f || !name || !len) return hd::set_global_error(HD_EINVAL, "hd_nc_dim_len: null argument");
  return guarded("hd_nc_dim_len", [&] {
    *len = (long)f->nc->dim_len(name);
    return HD_OK;
  });
}

int hd_nc_var_size(const hd_ncfile* f, const char* name, long* n) {
  if (!f || !name || !n) return hd::set_global_error(HD_EINVAL, "hd_nc_var_size: null argument");
  return guarded("hd_nc_var_size", [&] {
    *n = (long)f->nc->var(name).size();
    return HD_OK;
  });
}

int hd_nc_get_var_double(const hd_ncfile* f, const char* name, double* out, long n) {
  if (!f || !name || !out)
    return hd::set_global_error(HD_EINVAL, "hd_nc_get_var_double: null argument");
  return guarded("hd_nc_get_var_double", [&] {
    auto v = f->nc->var(name);
    if ((long)v.size() != n)
      return hd::set_global_error(HD_EINVAL, "hd_nc_get_var_double: %s has %zu values, not %ld",
                                  name, v.size(), n);
    std::copy(v.begin(), v.end(), out);
    return HD_OK;
  });
}

}  // extern "C"
