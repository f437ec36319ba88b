// harp_amd/ncread.hpp -- header-only readers of the netCDF files harp opens for
// the RFM opacity tables and ck weights with nc_open / nc_inq_dimid /
// nc_inq_dimlen / nc_inq_varid / nc_get_var_double (src/opacity/rfm.cpp:34-120,
// src/utils/read_weights.cpp:18-46):
//   NetCDFClassic  classic files (CDF-1, CDF-2 64-bit offset, CDF-5)
//   NetCDF4        netCDF-4 / HDF5 files, the format rfm.cpp:39 opens
//                  (nc_open(..., NC_NETCDF4, ...)) -- harp_amd/nc4read.hpp
//   NetCDFFile     either, chosen by the file's signature (what nc_open does)
// The netCDF library is not a dependency (NetCDF4 needs zlib: link -lz).
// Mirrors pyharp_amd/ncread.py.
#pragma once

#include "nc4read.hpp"

#include <memory>

#include <cstdint>
#include <cstring>
#include <fstream>
#include <iterator>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace harp_amd {

class NetCDFClassic {
 public:
  struct Var {
    std::vector<int> dimids;
    std::vector<size_t> shape;
    int type = 0;
    uint64_t vsize = 0, begin = 0;
    bool record = false;
  };

  explicit NetCDFClassic(std::string const& path) : path_(path) {
    std::ifstream f(path, std::ios::binary);
    if (!f.good()) throw std::runtime_error("ncread: cannot open " + path);
    buf_.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    if (buf_.size() >= 4 && (unsigned char)buf_[0] == 0x89 && buf_[1] == 'H' && buf_[2] == 'D' &&
        buf_[3] == 'F')
      throw std::runtime_error(path + ": netCDF-4/HDF5 file; NetCDFClassic takes classic netCDF "
                                      "only (NetCDFFile / NetCDF4 read it)");
    if (buf_.size() < 8 || buf_[0] != 'C' || buf_[1] != 'D' || buf_[2] != 'F' ||
        (buf_[3] != 1 && buf_[3] != 2 && buf_[3] != 5))
      throw std::runtime_error(path + ": not a netCDF classic file");
    version_ = buf_[3];
    pos_ = 4;
    numrecs_ = nonneg();
    // dimensions
    for (uint64_t n = tag_list(0x0A), i = 0; i < n; ++i) {
      std::string name = read_name();
      dims_.push_back({name, nonneg()});
    }
    skip_atts();
    // variables
    for (uint64_t n = tag_list(0x0B), i = 0; i < n; ++i) {
      std::string name = read_name();
      Var v;
      for (uint64_t nd = nonneg(), d = 0; d < nd; ++d) v.dimids.push_back((int)nonneg());
      skip_atts();
      v.type = (int)u32();
      v.vsize = nonneg();
      v.begin = version_ == 1 ? u32() : u64();
      for (int d : v.dimids) v.shape.push_back((size_t)dims_.at(d).second);
      v.record = !v.dimids.empty() && dims_.at(v.dimids[0]).second == 0;
      vars_[name] = v;
    }
    int nrec = 0;
    for (auto const& kv : vars_)
      if (kv.second.record) {
        recsize_ += kv.second.vsize;
        ++nrec;
      }
  }

  //! nc_inq_dimid + nc_inq_dimlen
  size_t dim_len(std::string const& name) const {
    for (auto const& d : dims_)
      if (d.first == name) return d.second == 0 ? (size_t)numrecs_ : (size_t)d.second;
    throw std::runtime_error(path_ + ": NetCDF: Invalid dimension ID or name (" + name + ")");
  }

  //! nc_inq_varid + nc_get_var_double (C order, converted to double)
  std::vector<double> var(std::string const& name) const {
    auto it = vars_.find(name);
    if (it == vars_.end())
      throw std::runtime_error(path_ + ": NetCDF: Variable not found (" + name + ")");
    Var const& v = it->second;
    size_t per = 1;
    for (size_t d = v.record ? 1 : 0; d < v.shape.size(); ++d) per *= v.shape[d];
    const size_t nrec = v.record ? (size_t)numrecs_ : 1;
    std::vector<double> out;
    out.reserve(per * nrec);
    for (size_t r = 0; r < nrec; ++r) {
      uint64_t off = v.begin + (v.record ? r * recsize_ : 0);
      for (size_t i = 0; i < per; ++i) out.push_back(value(v.type, off, i));
    }
    return out;
  }

 private:
  std::string path_;
  std::vector<char> buf_;
  size_t pos_ = 0;
  int version_ = 1;
  uint64_t numrecs_ = 0, recsize_ = 0;
  std::vector<std::pair<std::string, uint64_t>> dims_;
  std::map<std::string, Var> vars_;

  void need(size_t n) const {
    if (pos_ + n > buf_.size()) throw std::runtime_error(path_ + ": truncated netCDF header");
  }
  uint64_t be(size_t at, int n) const {
    uint64_t x = 0;
    for (int i = 0; i < n; ++i) x = (x << 8) | (unsigned char)buf_[at + i];
    return x;
  }
  uint32_t u32() {
    need(4);
    uint32_t x = (uint32_t)be(pos_, 4);
    pos_ += 4;
    return x;
  }
  uint64_t u64() {
    need(8);
    uint64_t x = be(pos_, 8);
    pos_ += 8;
    return x;
  }
  uint64_t nonneg() { return version_ == 5 ? u64() : u32(); }
  std::string read_name() {
    uint64_t n = nonneg();
    need((size_t)n);
    std::string s(buf_.data() + pos_, (size_t)n);
    pos_ += (size_t)((n + 3) & ~3ull);
    return s;
  }
  uint64_t tag_list(uint32_t tag) {
    uint32_t t = u32();
    uint64_t n = nonneg();
    if (t == 0 && n == 0) return 0;
    if (t != tag) throw std::runtime_error(path_ + ": corrupt netCDF header");
    return n;
  }
  static int type_size(int t) {
    switch (t) {
      case 1: case 2: case 7: return 1;
      case 3: case 8: return 2;
      case 4: case 5: case 9: return 4;
      case 6: case 10: case 11: return 8;
      default: throw std::runtime_error("ncread: unknown netCDF type");
    }
  }
  void skip_atts() {
    for (uint64_t n = tag_list(0x0C), i = 0; i < n; ++i) {
      read_name();
      int t = (int)u32();
      uint64_t ne = nonneg();
      pos_ += (size_t)((ne * type_size(t) + 3) & ~3ull);
    }
  }
  double value(int type, uint64_t off, size_t i) const {
    const size_t at = (size_t)off + i * type_size(type);
    if (at + type_size(type) > buf_.size()) throw std::runtime_error(path_ + ": truncated data");
    const uint64_t raw = be(at, type_size(type));
    switch (type) {
      case 1: return (double)(int8_t)raw;
      case 3: return (double)(int16_t)raw;
      case 4: return (double)(int32_t)raw;
      case 5: { uint32_t b = (uint32_t)raw; float f; std::memcpy(&f, &b, 4); return f; }
      case 6: { double d; std::memcpy(&d, &raw, 8); return d; }
      case 7: return (double)(uint8_t)raw;
      case 8: return (double)(uint16_t)raw;
      case 9: return (double)(uint32_t)raw;
      case 10: return (double)(int64_t)raw;
      case 11: return (double)raw;
      default: throw std::runtime_error("ncread: char variables are not numeric");
    }
  }
};

//! nc_open: a classic or a netCDF-4 (HDF5) file, by signature
class NetCDFFile {
 public:
  explicit NetCDFFile(std::string const& path) {
    if (NetCDF4::is_hdf5(path))
      h5_ = std::make_unique<NetCDF4>(path);
    else
      cl_ = std::make_unique<NetCDFClassic>(path);
  }
  bool netcdf4() const { return h5_ != nullptr; }
  size_t dim_len(std::string const& name) const {
    return h5_ ? h5_->dim_len(name) : cl_->dim_len(name);
  }
  std::vector<double> var(std::string const& name) const {
    return h5_ ? h5_->var(name) : cl_->var(name);
  }

 private:
  std::unique_ptr<NetCDF4> h5_;
  std::unique_ptr<NetCDFClassic> cl_;
};

}  // namespace harp_amd
