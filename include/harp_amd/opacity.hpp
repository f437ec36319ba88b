// harp_amd/opacity.hpp -- libtorch drop-ins for pyharp's table attenuators
// (harp::S8Fuller, harp::H2SO4Simple; src/opacity/s8_fuller.cpp,
// src/opacity/h2so4_simple.cpp), the RFM absorption tables (harp::RFM,
// src/opacity/rfm.cpp; tables read from netCDF-4 or classic files by ncread.hpp),
// read_weights_rfm (src/utils/read_weights.cpp) and the SW example's optics
// assembly (examples/amars_sw.cpp:261-271), backed by libhdisort.so (include/hdharp.h).
//
//     harp_amd::AttenuatorOptions op;
//     op.species_names({"S8", "H2SO4"}).species_weights({256.e-3, 98.e-3});
//     op.species_ids({0}).opacity_files({"s8_k_fuller.txt"});
//     harp_amd::S8Fuller s8(op);
//     auto prop1 = s8->forward(conc, kwargs);           // (nwave, ncol, nlyr, 2)
//     auto prop = harp_amd::band_optics_of(conc, dz, kwargs, /*nprop=*/2, s8, h2so4);
//
// Tables are read on the host as the reference does (decommented 3-column text,
// k_ext times the species weight); interpolation, mixing and the dz scaling
// run on the device.  There is no CPU compute path: tensors on the CPU are
// staged through the GPU.
#pragma once

#include <ATen/hip/HIPContext.h>
#include <torch/nn/cloneable.h>
#include <torch/nn/module.h>
#include <torch/torch.h>

#include <cmath>
#include <cstdlib>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../hdharp.h"
#include "ncread.hpp"
#include "../hdisort.h"

namespace harp_amd {

// ---- resources (src/utils/find_resource.cpp) ---------------------------------
inline std::vector<std::string>& resource_dirs() {
  static std::vector<std::string> dirs = {"."};
  return dirs;
}
inline void add_resource_directory(std::string const& d) {
  auto& v = resource_dirs();
  for (auto it = v.begin(); it != v.end(); ++it)
    if (*it == d) {
      v.erase(it);
      break;
    }
  v.insert(v.begin(), d);
}
inline std::string find_resource(std::string const& name) {
  auto exists = [](std::string const& p) { return std::ifstream(p).good(); };
  if (!name.empty() && name[0] == '/' && exists(name)) return name;
  std::vector<std::string> dirs = resource_dirs();
  if (const char* env = std::getenv("HARP_RESOURCE_PATH")) {
    std::stringstream ss(env);
    std::string d;
    while (std::getline(ss, d, ':'))
      if (!d.empty()) dirs.push_back(d);
  }
  for (auto const& d : dirs)
    if (exists(d + "/" + name)) return d + "/" + name;
  TORCH_CHECK(false, "find_resource: cannot find ", name);
  return "";
}

// decommented whitespace table (src/utils/fileio.cpp decomment_file)
inline std::vector<std::vector<double>> read_table(std::string const& path) {
  std::ifstream f(path);
  TORCH_CHECK(f.good(), "decomment_file: file not found: ", path);
  std::vector<std::vector<double>> rows;
  std::string line;
  while (std::getline(f, line)) {
    auto h = line.find('#');
    if (h != std::string::npos) line.resize(h);
    std::stringstream ss(line);
    std::vector<double> r;
    double v;
    while (ss >> v) r.push_back(v);
    if (!r.empty()) rows.push_back(r);
  }
  TORCH_CHECK(!rows.empty(), "Empty file: ", path);
  return rows;
}

#define HARP_AMD_ARG(T, name)                                      \
 public:                                                          \
  inline auto name(const T& v) -> decltype(*this) {               \
    this->name##_ = v;                                            \
    return *this;                                                 \
  }                                                               \
  inline const T& name() const noexcept { return this->name##_; } \
  inline T& name() noexcept { return this->name##_; }             \
                                                                  \
 private:                                                         \
  T name##_

// src/opacity/attenuator_options.hpp:8-19
struct AttenuatorOptions {
  HARP_AMD_ARG(std::string, type) = "";
  HARP_AMD_ARG(std::vector<std::string>, opacity_files) = {};
  HARP_AMD_ARG(std::vector<int>, species_ids) = {0};
  HARP_AMD_ARG(std::vector<std::string>, species_names) = {};
  HARP_AMD_ARG(std::vector<double>, species_weights) = {};
};
#undef HARP_AMD_ARG

namespace detail {
inline torch::Device device_of(std::initializer_list<torch::Tensor> ts) {
  for (auto const& t : ts)
    if (t.defined() && t.is_cuda()) return t.device();
  return torch::Device(torch::kCUDA, 0);
}
inline void* stream_of(torch::Device dev) {
  return reinterpret_cast<void*>(at::hip::getCurrentHIPStream(dev.index()).stream());
}
inline std::pair<torch::Tensor, int> coord_of(std::map<std::string, torch::Tensor> const& kw) {
  if (kw.count("wavelength")) return {kw.at("wavelength"), HD_COORD_WAVELENGTH};
  if (kw.count("wavenumber")) return {kw.at("wavenumber"), HD_COORD_WAVENUMBER};
  TORCH_CHECK(false, "wavelength or wavenumber is required in kwargs");
  return {};
}
}  // namespace detail

// Common body of S8FullerImpl / H2SO4SimpleImpl (they differ by type name only)
template <class Derived>
class TableAttenuatorImpl : public torch::nn::Cloneable<Derived> {
 public:
  AttenuatorOptions options;
  torch::Tensor kwave, kdata;  // (rows,), (rows, 2): wavelength [um], (k_ext [m^2/mol], ssa)

  TableAttenuatorImpl() = default;
  explicit TableAttenuatorImpl(AttenuatorOptions const& op) : options(op) {}

  void reset() override {
    TORCH_CHECK(options.opacity_files().size() == 1, "Only one opacity file is allowed");
    TORCH_CHECK(options.species_ids().size() == 1, "Only one species is allowed");
    TORCH_CHECK(options.species_ids()[0] >= 0, "Invalid species_id: ", options.species_ids()[0]);
    TORCH_CHECK(options.type().empty() || options.type() == Derived::kType,
                "Mismatch type: ", options.type());
    auto path = find_resource(options.opacity_files()[0]);
    auto rows = read_table(path);
    const int n = (int)rows.size();
    for (auto const& r : rows) TORCH_CHECK(r.size() == 3, "Invalid file: ", path);
    const int sid = options.species_ids()[0];
    TORCH_CHECK(sid < (int)options.species_weights().size(), "no species weight for ", sid);
    kwave = this->register_buffer("kwave", torch::zeros({n}, torch::kFloat64));
    kdata = this->register_buffer("kdata", torch::zeros({n, 2}, torch::kFloat64));
    auto wa = kwave.accessor<double, 1>();
    auto da = kdata.accessor<double, 2>();
    for (int i = 0; i < n; ++i) {
      wa[i] = rows[i][0];
      da[i][0] = rows[i][1] * options.species_weights()[sid];  // m^2/kg -> m^2/mol
      da[i][1] = rows[i][2];
    }
    dev_.clear();
  }

  //! table in the layout hdharp.h wants, on `dev` (kept alive by this module)
  hd_attenuator table(torch::Device dev) {
    auto key = dev.str();
    if (!dev_.count(key)) {
      auto o = torch::TensorOptions().dtype(torch::kFloat64).device(dev);
      dev_[key] = {kwave.to(o).contiguous(), kdata.select(1, 0).to(o).contiguous(),
                   kdata.select(1, 1).to(o).contiguous()};
    }
    auto& t = dev_[key];
    return hd_attenuator{(int)kwave.size(0), t[0].data_ptr<double>(), t[1].data_ptr<double>(),
                         t[2].data_ptr<double>(), options.species_ids()[0]};
  }

  //! (nwave, ncol, nlyr, 2): [0] = k c [1/m], [1] = ssa k c
  torch::Tensor forward(torch::Tensor conc, std::map<std::string, torch::Tensor> const& kwargs) {
    auto [coord, kind] = detail::coord_of(kwargs);
    auto dev = detail::device_of({conc, coord});
    auto o = torch::TensorOptions().dtype(torch::kFloat64).device(dev);
    auto c = conc.to(o).contiguous();
    auto x = coord.to(o).contiguous().view({-1});
    TORCH_CHECK(c.dim() == 3, "conc must be (ncol, nlyr, nspecies)");
    auto out = torch::empty({x.size(0), c.size(0), c.size(1), 2}, o);
    auto att = table(dev);
    int rc = hd_attenuate(&att, x.data_ptr<double>(), kind, (int)x.size(0),
                          c.data_ptr<double>(), (int)c.size(0), (int)c.size(1), (int)c.size(2),
                          out.data_ptr<double>(), detail::stream_of(dev));
    TORCH_CHECK(rc == HD_OK, "hd_attenuate: ", hd_last_error(nullptr));
    return conc.is_cuda() ? out : out.to(conc.device());
  }

 private:
  std::map<std::string, std::vector<torch::Tensor>> dev_;
};

class S8FullerImpl : public TableAttenuatorImpl<S8FullerImpl> {
 public:
  static constexpr const char* kType = "s8_fuller";
  S8FullerImpl() = default;
  explicit S8FullerImpl(AttenuatorOptions const& op) : TableAttenuatorImpl(op) { reset(); }
};
TORCH_MODULE(S8Fuller);

class H2SO4SimpleImpl : public TableAttenuatorImpl<H2SO4SimpleImpl> {
 public:
  static constexpr const char* kType = "h2so4_simple";
  H2SO4SimpleImpl() = default;
  explicit H2SO4SimpleImpl(AttenuatorOptions const& op) : TableAttenuatorImpl(op) { reset(); }
};
TORCH_MODULE(H2SO4Simple);

//! prop (nwave, ncol, nlyr, nprop) for Disort::forward: tau = dz sum_a k_a c_a,
//! ssa = sum_a ssa_a k_a c_a / sum_a k_a c_a (0 without extinction), moments 0.
//! tables: device tables of the attenuators (module->table(device)).
inline torch::Tensor band_optics(std::vector<hd_attenuator> const& tables, torch::Tensor conc,
                          torch::Tensor dz, std::map<std::string, torch::Tensor> const& kwargs,
                          int nprop = 2) {
  auto [coord, kind] = detail::coord_of(kwargs);
  auto dev = detail::device_of({conc, coord, dz});
  auto o = torch::TensorOptions().dtype(torch::kFloat64).device(dev);
  auto c = conc.to(o).contiguous();
  const int ncol = c.size(0), nlyr = c.size(1), nsp = c.size(2);
  auto d = dz.to(o).reshape({-1, nlyr}).expand({ncol, nlyr}).contiguous();
  auto x = coord.to(o).contiguous().view({-1});
  auto prop = torch::empty({x.size(0), ncol, nlyr, nprop}, o);
  int rc = hd_band_optics(tables.data(), (int)tables.size(), x.data_ptr<double>(), kind,
                          (int)x.size(0), c.data_ptr<double>(), ncol, nlyr, nsp,
                          d.data_ptr<double>(), nprop, prop.data_ptr<double>(),
                          detail::stream_of(dev));
  TORCH_CHECK(rc == HD_OK, "hd_band_optics: ", hd_last_error(nullptr));
  return prop;
}

//! band_optics over attenuator modules: band_optics_of(conc, dz, kwargs, 2, s8, h2so4)
template <class... M>
torch::Tensor band_optics_of(torch::Tensor conc, torch::Tensor dz,
                             std::map<std::string, torch::Tensor> const& kwargs, int nprop,
                             M&... mods) {
  auto dev = detail::device_of({conc, detail::coord_of(kwargs).first, dz});
  return band_optics({mods->table(dev)...}, conc, dz, kwargs, nprop);
}

//! prop (nwave, ncol, nlyr, 2 + nmom) by RadiationBandImpl::forward's mixing
//! (src/radiation/radiation_band.cpp:86-116): tau-weighted ssa, tau*ssa-weighted
//! Henyey-Greenstein moments, the +1e-10 regularisation, tau = ext dz (hdharp.h
//! hd_band_loop_optics).  atts: {module->table(device), gasym device pointer or
//! nullptr}; ext0: (nwave, ncol, nlyr[, 1]) extinction of attenuators without ssa
//! (an RFM forward), or undefined.
inline torch::Tensor band_loop_optics(std::vector<hd_band_attenuator> const& atts,
                                      torch::Tensor conc, torch::Tensor dz,
                                      std::map<std::string, torch::Tensor> const& kwargs,
                                      int nmom, torch::Tensor ext0 = {}) {
  auto [coord, kind] = detail::coord_of(kwargs);
  auto dev = detail::device_of({conc, coord, dz});
  auto o = torch::TensorOptions().dtype(torch::kFloat64).device(dev);
  auto c = conc.to(o).contiguous();
  const int ncol = c.size(0), nlyr = c.size(1), nsp = c.size(2);
  auto d = dz.to(o).reshape({-1, nlyr}).expand({ncol, nlyr}).contiguous();
  auto x = coord.to(o).contiguous().view({-1});
  torch::Tensor e0;
  if (ext0.defined()) {
    e0 = ext0.to(o).contiguous();
    TORCH_CHECK(e0.numel() == x.size(0) * ncol * nlyr, "band_loop_optics: ext0 size");
  }
  auto prop = torch::empty({x.size(0), ncol, nlyr, 2 + nmom}, o);
  int rc = hd_band_loop_optics(atts.data(), (int)atts.size(),
                               e0.defined() ? e0.data_ptr<double>() : nullptr,
                               x.data_ptr<double>(), kind, (int)x.size(0), c.data_ptr<double>(),
                               ncol, nlyr, nsp, d.data_ptr<double>(), nmom,
                               prop.data_ptr<double>(), detail::stream_of(dev));
  TORCH_CHECK(rc == HD_OK, "hd_band_loop_optics: ", hd_last_error(nullptr));
  return prop;
}

// ---- RFM (src/opacity/rfm.hpp, rfm.cpp) -------------------------------------
class RFMImpl : public torch::nn::Cloneable<RFMImpl> {
 public:
  constexpr static int IPR = 0;
  constexpr static int ITM = 1;
  size_t kshape[3] = {0, 0, 0};  //! (nwave, npres, ntemp)
  torch::Tensor kaxis;           //! (nwave + npres + ntemp,): wave, ln p, T anomaly
  torch::Tensor kdata;           //! (nwave, npres, ntemp) ln(m^2/kmol)
  torch::Tensor krefatm;         //! (2, npres): ln p, T_ref
  AttenuatorOptions options;

  RFMImpl() = default;
  explicit RFMImpl(AttenuatorOptions const& op) : options(op) {
    TORCH_CHECK(options.opacity_files().size() == 1, "Only one opacity file is allowed");
    TORCH_CHECK(options.species_ids().size() == 1, "Only one species is allowed");
    TORCH_CHECK(options.species_ids()[0] >= 0, "Invalid species_id: ", options.species_ids()[0]);
    TORCH_CHECK(options.type().empty() || options.type() == "rfm", "Mismatch type: ",
                options.type());
    reset();
  }

  void reset() override {
    NetCDFFile nc(find_resource(options.opacity_files()[0]));
    kshape[0] = nc.dim_len("Wavenumber");
    kshape[1] = nc.dim_len("Pressure");
    kshape[2] = nc.dim_len("TempGrid");
    const int nw = (int)kshape[0], np_ = (int)kshape[1], nt = (int)kshape[2];
    std::vector<double> ax = nc.var("Wavenumber");
    std::vector<double> pr = nc.var("Pressure");
    std::vector<double> tg = nc.var("TempGrid");
    std::vector<double> tr = nc.var("Temperature");
    TORCH_CHECK((int)ax.size() == nw && (int)pr.size() == np_ && (int)tg.size() == nt &&
                    (int)tr.size() == np_, "RFM: inconsistent table axes");
    for (auto& x : pr) x = std::log(x);  // pressure -> ln pressure
    ax.insert(ax.end(), pr.begin(), pr.end());
    ax.insert(ax.end(), tg.begin(), tg.end());
    auto name = options.species_names().at(options.species_ids()[0]);
    std::vector<double> kd = nc.var(name);
    TORCH_CHECK((int64_t)kd.size() == (int64_t)nw * np_ * nt, "RFM: table ", name, " size");
    auto o = torch::TensorOptions().dtype(torch::kFloat64);
    kaxis = register_buffer("kaxis", torch::tensor(ax, o));
    kdata = register_buffer("kdata", torch::tensor(kd, o).view({nw, np_, nt}));
    krefatm = register_buffer("krefatm", torch::stack({torch::tensor(pr, o), torch::tensor(tr, o)}));
    dev_.clear();
  }

  //! (nwave, ncol, nlyr, 1) = 1e-3 exp(k) conc; kwargs "pres" [Pa], "temp" [K]: (ncol, nlyr)
  torch::Tensor forward(torch::Tensor conc, std::map<std::string, torch::Tensor> const& kwargs) {
    TORCH_CHECK(kwargs.count("pres") > 0, "pres is required in kwargs");
    TORCH_CHECK(kwargs.count("temp") > 0, "temp is required in kwargs");
    auto dev = detail::device_of({conc, kwargs.at("pres"), kwargs.at("temp")});
    auto o = torch::TensorOptions().dtype(torch::kFloat64).device(dev);
    auto c = conc.to(o).contiguous();
    TORCH_CHECK(c.dim() == 3, "conc must be (ncol, nlyr, nspecies)");
    const int ncol = c.size(0), nlyr = c.size(1), nsp = c.size(2);
    auto p = kwargs.at("pres").to(o).expand({ncol, nlyr}).contiguous();
    auto t = kwargs.at("temp").to(o).expand({ncol, nlyr}).contiguous();
    auto out = torch::empty({(int64_t)kshape[0], ncol, nlyr, 1}, o);
    auto key = dev.str();
    if (!dev_.count(key))
      dev_[key] = {kaxis.to(o).contiguous(), krefatm.select(0, ITM).to(o).contiguous(),
                   kdata.to(o).contiguous()};
    auto& d = dev_[key];
    const double* ax = d[0].data_ptr<double>();
    hd_rfm_table tab{(int)kshape[0], (int)kshape[1], (int)kshape[2], ax, ax + kshape[0],
                     ax + kshape[0] + kshape[1], d[1].data_ptr<double>(), d[2].data_ptr<double>(),
                     options.species_ids()[0]};
    int rc = hd_rfm_attenuate(&tab, c.data_ptr<double>(), ncol, nlyr, nsp, p.data_ptr<double>(),
                              t.data_ptr<double>(), out.data_ptr<double>(), detail::stream_of(dev));
    TORCH_CHECK(rc == HD_OK, "hd_rfm_attenuate: ", hd_last_error(nullptr));
    return conc.is_cuda() ? out : out.to(conc.device());
  }

 private:
  std::map<std::string, std::vector<torch::Tensor>> dev_;
};
TORCH_MODULE(RFM);

//! src/utils/read_weights.cpp:18-46
inline torch::Tensor read_weights_rfm(std::string const& filename) {
  NetCDFFile nc(find_resource(filename));
  const size_t n = nc.dim_len("weights");
  auto w = nc.var("weights");
  TORCH_CHECK(w.size() == n, "read_weights_rfm: size mismatch");
  return torch::tensor(w, torch::TensorOptions().dtype(torch::kFloat64));
}

}  // namespace harp_amd
