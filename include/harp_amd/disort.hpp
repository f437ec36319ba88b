// harp_amd/disort.hpp -- libtorch drop-in for pydisort's `disort::Disort` module,
// backed by the MI355X kernels of libhdisort.so (C-ABI: include/hdisort.h).
//
// pyharp builds its solver as
//     rtsolver = torch::nn::AnyModule(disort::Disort(options.disort()));
// (src/radiation/radiation_band.cpp:57-69) and calls
//     rtsolver.forward(prop, &bc[, temf])      (radiation_band.cpp:123-128,
//     examples/amars_sw.cpp:280, examples/amars_lw.cpp:80)
// with the plugin contract of RTSolverImpl::forward (src/rtsolver/rtsolver.hpp:25-29).
// Swapping `disort::Disort` for `harp_amd::Disort` keeps that code unchanged:
//
//     harp_amd::DisortOptions op;
//     op.flags("lamber,quiet,onlyfl").nwave(nwave).ncol(ncol);
//     op.ds().nlyr = nlyr; op.ds().nstr = 16; op.ds().nmom = 16;
//     harp_amd::Disort disort(op);
//     auto flux = disort->forward(prop, &bc);          // (nwave, ncol, nlyr+1, 2)
//
// Without `onlyfl` the module also computes radiances (hd_solve_radiance; the
// configuration of tests/test_disort.cpp:13-55): at user_mu x user_phi with
// `usrang` (else the quadrature cosines), at user_tau with `usrtau` (else the
// levels); `disort->get_rad()` returns (nwave, ncol, nphi, ntau, numu).  With
// `usrtau` the fluxes are at the user depths, index 0 = the deepest.
//
// Tensors may live on the CPU (staged through the GPU, result returned on the
// CPU) or on a ROCm device (zero-copy, torch's current stream).  Errors are
// raised with TORCH_CHECK, like the reference (radiation_band.cpp:25,50,71).
#pragma once

#include <ATen/hip/HIPContext.h>
#include <torch/nn/cloneable.h>
#include <torch/nn/module.h>
#include <torch/nn/modules/container/any.h>
#include <torch/torch.h>

#include <cmath>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "../hdisort.h"

namespace harp_amd {

namespace index {
constexpr int IEX = 0;  // optical thickness
constexpr int ISS = 1;  // single-scattering albedo
constexpr int IPM = 2;  // phase moments chi_1..chi_nmom
constexpr int IUP = 0;  // upward flux
constexpr int IDN = 1;  // downward flux (rfldir + rfldn)
}  // namespace index

#define HARP_AMD_ARG(T, name)                                         \
 public:                                                             \
  inline auto name(const T& v) -> decltype(*this) {                  \
    this->name##_ = v;                                               \
    return *this;                                                    \
  }                                                                  \
  inline const T& name() const noexcept { return this->name##_; }    \
  inline T& name() noexcept { return this->name##_; }                \
                                                                     \
 private:                                                            \
  T name##_

struct DisortState {  // subset of cdisort's disort_state reachable via ds()
  int nlyr = 1, nstr = 4, nmom = 4, nphi = 0, ntau = 0, numu = 0;
  std::vector<double> utau;  // user optical depths (usrtau), filled by reset()
};

// pydisort's scattering_moments(nmom, PhaseMomentOptions) for the phase
// functions with closed-form moments (used at tests/test_disort.cpp:44-47):
// chi_1..chi_nmom of the isotropic, Rayleigh and Henyey-Greenstein functions
enum PhaseFunctionType { kIsotropic, kRayleigh, kHenyeyGreenstein };
struct PhaseMomentOptions {
  PhaseMomentOptions() = default;
  PhaseMomentOptions& type(PhaseFunctionType t) {
    type_ = t;
    return *this;
  }
  PhaseMomentOptions& gg(double g) {
    gg_ = g;
    return *this;
  }
  PhaseFunctionType type_ = kIsotropic;
  double gg_ = 0.0;
};
inline torch::Tensor scattering_moments(int nmom, PhaseMomentOptions const& op) {
  auto m = torch::zeros({nmom}, torch::kFloat64);
  auto a = m.accessor<double, 1>();
  for (int l = 1; l <= nmom; ++l) {
    if (op.type_ == kRayleigh) a[l - 1] = l == 2 ? 0.1 : 0.0;
    if (op.type_ == kHenyeyGreenstein) a[l - 1] = std::pow(op.gg_, l);
  }
  return m;
}

struct DisortOptions {
  DisortOptions() = default;
  DisortState& ds() { return ds_; }
  const DisortState& ds() const { return ds_; }
  HARP_AMD_ARG(std::string, header) = "";
  HARP_AMD_ARG(std::string, flags) = "";
  HARP_AMD_ARG(int, nwave) = 1;
  HARP_AMD_ARG(int, ncol) = 1;
  HARP_AMD_ARG(std::vector<double>, wave_lower) = {};
  HARP_AMD_ARG(std::vector<double>, wave_upper) = {};
  HARP_AMD_ARG(std::vector<double>, user_tau) = {};
  HARP_AMD_ARG(std::vector<double>, user_mu) = {};
  HARP_AMD_ARG(std::vector<double>, user_phi) = {};
  HARP_AMD_ARG(int, device) = 0;

 private:
  DisortState ds_;
};

// Converts pyharp's solver options (`options.disort()`, a pydisort
// disort::DisortOptions -- or any type with its accessors) into this module's
// options: the fields pyharp sets at src/radiation/radiation_band.cpp:58-66 plus
// the header, flags, user depths and ds().nstr/nmom.  This is the one line that
// changes at radiation_band.cpp:68:
//   rtsolver = torch::nn::AnyModule(harp_amd::Disort(harp_amd::to_harp_amd(options.disort())));
template <class PydisortOptions>
DisortOptions to_harp_amd(PydisortOptions&& src) {
  DisortOptions op;
  op.header(src.header()).flags(src.flags()).nwave(src.nwave()).ncol(src.ncol());
  op.wave_lower(std::vector<double>(src.wave_lower().begin(), src.wave_lower().end()));
  op.wave_upper(std::vector<double>(src.wave_upper().begin(), src.wave_upper().end()));
  op.user_tau(std::vector<double>(src.user_tau().begin(), src.user_tau().end()));
  op.user_mu(std::vector<double>(src.user_mu().begin(), src.user_mu().end()));
  op.user_phi(std::vector<double>(src.user_phi().begin(), src.user_phi().end()));
  op.ds().nlyr = src.ds().nlyr;
  op.ds().nstr = src.ds().nstr;
  op.ds().nmom = src.ds().nmom;
  return op;
}

inline std::set<std::string> parse_flags(const std::string& s) {
  std::set<std::string> out;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    tok.erase(0, tok.find_first_not_of(" \t"));
    tok.erase(tok.find_last_not_of(" \t") + 1);
    if (!tok.empty()) out.insert(tok);
  }
  return out;
}

class DisortImpl : public torch::nn::Cloneable<DisortImpl> {
 public:
  DisortOptions options;

  DisortImpl() = default;
  explicit DisortImpl(DisortOptions const& op) : options(op) { reset(); }

  void reset() override {
    // cdisort's disort_flag fields as pydisort's flag string names them
    // (examples/amarsw-ck.yaml:74-90); the semantics match pyharp_amd.disort.check_flags
    static const std::set<std::string> known = {
        "lamber", "quiet", "onlyfl", "planck", "usrtau", "usrang", "intensity_correction",
        "old_intensity_correction", "print-input", "print-fluxes", "print-intensity",
        "print-transmissivity", "print-phase-function", "ibcnd", "spher", "general_source",
        "output_uum"};
    auto flags = parse_flags(options.flags());
    for (auto const& f : flags) TORCH_CHECK(known.count(f), "Disort: unknown flag ", f);
    // harp's DISORT driver refuses ibcnd (src/rtsolver/rt_solver_disort.cpp_:67-68)
    TORCH_CHECK(!flags.count("ibcnd"), "RTSolverDisort::CalRadtranFlux: ibcnd = 1, expected 0 "
                "(the special-case albedo/transmissivity mode is not supported)");
    TORCH_CHECK(!flags.count("spher"), "Disort: flag 'spher': pseudo-spherical geometry is not "
                "implemented");
    TORCH_CHECK(!flags.count("general_source"), "Disort: flag 'general_source': general "
                "(user-supplied) sources are not implemented");
    TORCH_CHECK(!flags.count("output_uum"), "Disort: flag 'output_uum': per-mode intensities "
                "(uum) are not output");
    TORCH_CHECK(!(flags.count("intensity_correction") && !flags.count("old_intensity_correction") &&
                  !flags.count("onlyfl")),
                "Disort: intensity_correction without old_intensity_correction selects cdisort's "
                "new (Buras-Emde-Dowling) correction, which is not implemented; add "
                "old_intensity_correction for the Nakajima-Tanaka correction (TMS + IMS) or use "
                "onlyfl");
    TORCH_CHECK(flags.count("lamber"), "Disort: only Lambertian lower boundaries are supported");
    auto const& ds = options.ds();
    TORCH_CHECK(ds.nstr >= 2 && ds.nstr % 2 == 0 && ds.nstr <= 32,
                "Disort: nstr must be even and in [2, 32]");
    TORCH_CHECK(ds.nlyr >= 1, "Disort: nlyr must be >= 1");
    planck_ = flags.count("planck") > 0;
    if (planck_)
      TORCH_CHECK((int)options.wave_lower().size() == options.nwave() &&
                      (int)options.wave_upper().size() == options.nwave(),
                  "Disort: planck needs wave_lower/wave_upper of size nwave");
    onlyfl_ = flags.count("onlyfl") > 0;
    usrtau_ = flags.count("usrtau") > 0;
    // cdisort corrects with both flags; old_intensity_correction alone applies none
    corint_ = flags.count("intensity_correction") && flags.count("old_intensity_correction");
    radiance_ = !onlyfl_ || usrtau_;
    rad_ = torch::Tensor();
    auto& d = options.ds();
    if (radiance_) {
      if (usrtau_) {
        d.utau = options.user_tau();
        TORCH_CHECK(!d.utau.empty(), "Disort: usrtau set but user_tau is empty");
        for (size_t i = 0; i < d.utau.size(); ++i)
          TORCH_CHECK(d.utau[i] >= 0 && (i == 0 || d.utau[i] >= d.utau[i - 1]),
                      "Disort: user_tau must be >= 0 and ascending");
        d.ntau = (int)d.utau.size();
      } else {
        d.utau.clear();
        d.ntau = d.nlyr + 1;
      }
      if (flags.count("usrang")) {
        umu_ = options.user_mu();
        TORCH_CHECK(!umu_.empty(), "Disort: usrang needs user_mu");
        for (double x : umu_)
          TORCH_CHECK(x != 0.0 && std::fabs(x) <= 1.0, "Disort: user_mu must be in [-1,0)U(0,1]");
      } else {
        std::vector<double> mu(d.nstr / 2), w(d.nstr / 2);
        TORCH_CHECK(hd_quadrature(d.nstr, mu.data(), w.data()) == HD_OK, "Disort: quadrature");
        umu_.clear();
        for (int i = d.nstr / 2 - 1; i >= 0; --i) umu_.push_back(-mu[i]);
        for (double x : mu) umu_.push_back(x);
      }
      phi_ = options.user_phi();
      if (phi_.empty()) phi_ = {0.0};
      d.numu = onlyfl_ ? 0 : (int)umu_.size();
      d.nphi = onlyfl_ ? 0 : (int)phi_.size();
    }
  }

  DisortState& ds() { return options.ds(); }

  //! radiances of the last forward: (nwave, ncol, nphi, ntau, numu)
  torch::Tensor get_rad(torch::TensorOptions const& op = {}) const {
    TORCH_CHECK(!onlyfl_, "Disort.get_rad: radiances are off (onlyfl flag)");
    TORCH_CHECK(rad_.defined(), "Disort.get_rad: call forward first");
    return rad_.to(op.has_device() ? op.device() : rad_.device(),
                   op.has_dtype() ? op.dtype() : rad_.dtype());
  }

  //! flux (nwave, ncol, nlyr+1, 2); level 0 = surface; [..,0] up, [..,1] down.
  //! temf is a Tensor (undefined = none) with a registered default, so
  //! torch::nn::AnyModule takes both forward(prop, &bc) and
  //! forward(prop, &bc, layer2level(...)) as radiation_band.cpp:124-127 calls them.
  torch::Tensor forward(torch::Tensor prop, std::map<std::string, torch::Tensor>* bc,
                        torch::Tensor temf = torch::Tensor()) {
    Batch x = prepare(prop, bc, temf);
    const int nlev = radiance_ ? options.ds().ntau : x.nlyr + 1;
    auto flux = torch::empty({x.nwave, x.ncol, nlev, 2}, x.f64);
    auto stream = at::hip::getCurrentHIPStream(x.dev.index()).stream();
    int rc;
    if (radiance_) {
      auto const& d = options.ds();
      hd_radiance rad{usrtau_ ? d.ntau : 0, d.utau.data(), (int)umu_.size(), umu_.data(),
                      (int)phi_.size(), phi_.data(), x.bp("phi0"), onlyfl_ ? 1 : 0,
                      corint_ ? 1 : 0};
      torch::Tensor uu;
      if (!onlyfl_)
        uu = torch::empty({x.nwave, x.ncol, (int)phi_.size(), d.ntau, (int)umu_.size()}, x.f64);
      rc = hd_solve_radiance(context(x.dev.index()), &x.cfg, &x.in, &rad,
                             flux.data_ptr<double>(),
                             uu.defined() ? uu.data_ptr<double>() : nullptr, nullptr,
                             reinterpret_cast<void*>(stream));
      rad_ = uu.defined() ? (x.in_dev.is_cuda() ? uu : uu.to(x.in_dev)) : uu;
    } else if (x.host) {  // CPU tensors: hd_solve_host (pieces copied beside the solve)
      rc = hd_solve_host(context(x.dev.index()), &x.cfg, &x.in, flux.data_ptr<double>(), nullptr);
    } else {
      rc = hd_solve(context(x.dev.index()), &x.cfg, &x.in, flux.data_ptr<double>(), nullptr,
                    reinterpret_cast<void*>(stream));
    }
    TORCH_CHECK(rc == HD_OK, "DisortWrapper::Run failed: ", hd_last_error(context(x.dev.index())));
    return x.in_dev.is_cuda() ? flux : flux.to(x.in_dev);
  }

  //! band flux (ncol, nlyr+1, 2) = sum_w weights[w] flux[w] with the sum fused into
  //! the solve (hd_solve_band): what examples/amars_lw.cpp:84-88 forms from
  //! forward's result, without storing the per-point fluxes
  torch::Tensor forward_band(torch::Tensor prop, std::map<std::string, torch::Tensor>* bc,
                             torch::Tensor temf, torch::Tensor weights) {
    TORCH_CHECK(!radiance_, "Disort.forward_band: the fused band sum is a flux-only path");
    Batch x = prepare(prop, bc, temf);
    auto w = weights.to(x.f64).reshape({-1}).contiguous();
    TORCH_CHECK(w.size(0) == x.nwave, "Disort.forward_band: ", w.size(0), " weights for ",
                x.nwave, " waves");
    auto bflux = torch::empty({x.ncol, x.nlyr + 1, 2}, x.f64);
    hd_band band{w.data_ptr<double>(), bflux.data_ptr<double>()};
    auto stream = at::hip::getCurrentHIPStream(x.dev.index()).stream();
    const int rc =
        x.host ? hd_solve_band_host(context(x.dev.index()), &x.cfg, &x.in, w.data_ptr<double>(),
                                    bflux.data_ptr<double>(), nullptr, nullptr)
               : hd_solve_band(context(x.dev.index()), &x.cfg, &x.in, &band, nullptr, nullptr,
                               reinterpret_cast<void*>(stream));
    TORCH_CHECK(rc == HD_OK, "DisortWrapper::Run failed: ", hd_last_error(context(x.dev.index())));
    return x.in_dev.is_cuda() ? bflux : bflux.to(x.in_dev);
  }

 protected:
  FORWARD_HAS_DEFAULT_ARGS({2, torch::nn::AnyValue(torch::Tensor())})

 private:
  bool planck_ = false;
  bool onlyfl_ = true, usrtau_ = false, radiance_ = false, corint_ = false;
  std::vector<double> umu_, phi_;
  torch::Tensor rad_;

  // one batch on the device in the C-ABI's form (the tensors own the memory the
  // hd_inputs pointers refer to)
  struct Batch {
    torch::Device dev = torch::kCPU, in_dev = torch::kCPU;
    bool host = false;  // CPU tensors on the flux path: arrays stay on the host
    torch::TensorOptions f64;
    int nwave = 0, ncol = 0, nlyr = 0, nprop = 0;
    torch::Tensor p, tf, wl, wu;
    std::map<std::string, torch::Tensor> b;
    hd_config cfg{};
    hd_inputs in{};
    const double* bp(const char* k) const {
      auto it = b.find(k);
      return it == b.end() ? nullptr : it->second.data_ptr<double>();
    }
  };

  Batch prepare(torch::Tensor prop, std::map<std::string, torch::Tensor>* bc,
                torch::Tensor temf) {
    TORCH_CHECK(prop.dim() == 4, "Disort.forward: prop must be (nwave, ncol, nlyr, nprop)");
    Batch x;
    x.nwave = prop.size(0);
    x.ncol = prop.size(1);
    x.nlyr = prop.size(2);
    x.nprop = prop.size(3);
    const int nwave = x.nwave, ncol = x.ncol, nlyr = x.nlyr;
    TORCH_CHECK(nlyr == options.ds().nlyr, "Disort.forward: prop has ", nlyr,
                " layers, ds().nlyr = ", options.ds().nlyr);
    TORCH_CHECK(!planck_ || temf.defined(), "Disort.forward: planck flag set but temf missing");
    TORCH_CHECK(!planck_ || ((int)options.wave_lower().size() == nwave &&
                             (int)options.wave_upper().size() == nwave),
                "Disort.forward: planck: prop has ", nwave, " waves but wave_lower/wave_upper hold ",
                options.wave_lower().size(), "/", options.wave_upper().size());
    x.in_dev = prop.device();
    x.dev = x.in_dev.is_cuda() ? x.in_dev : torch::Device(torch::kCUDA, options.device());
    // pydisort's callers hand over CPU tensors (amars_sw.cpp:280, amars_lw.cpp:80,
    // radiation_band.cpp:124-127): on the flux path they go to the host-array entry
    // points, which copy them over in pieces beside the solve
    x.host = !x.in_dev.is_cuda() && !radiance_;
    x.f64 = torch::TensorOptions().dtype(torch::kFloat64).device(x.host ? x.in_dev : x.dev);
    auto to_dev = [&](torch::Tensor t) { return t.to(x.f64).contiguous(); };
    x.p = to_dev(prop);
    static const char* keys[] = {"fbeam", "umu0", "albedo", "btemp", "ttemp", "temis", "fisot"};
    if (bc) {
      for (auto const& [k, v] : *bc) {
        bool ok = k == "phi0";
        for (auto key : keys) ok = ok || k == key;
        TORCH_CHECK(ok, "Disort.forward: unknown boundary condition '", k, "'");
        x.b[k] = to_dev(v.expand({nwave, ncol}));
      }
    }
    if (planck_) {
      x.tf = to_dev(temf);
      TORCH_CHECK(x.tf.size(0) == ncol && x.tf.size(1) == nlyr + 1,
                  "Disort.forward: temf must be (ncol, nlyr+1)");
      x.wl = torch::tensor(options.wave_lower(), x.f64);
      x.wu = torch::tensor(options.wave_upper(), x.f64);
    }
    auto ptr = [](const torch::Tensor& t) -> const double* {
      return t.defined() ? t.data_ptr<double>() : nullptr;
    };
    x.cfg = hd_config{options.ds().nstr, options.ds().nmom, nlyr, x.nprop,
                      HD_FLAG_LAMBER | HD_FLAG_ONLYFL | (planck_ ? HD_FLAG_PLANCK : 0u)};
    x.in = hd_inputs{nwave,          ncol,          ptr(x.p),       x.bp("fbeam"),
                     x.bp("umu0"),   x.bp("albedo"), x.bp("btemp"), x.bp("ttemp"),
                     x.bp("temis"),  x.bp("fisot"),  ptr(x.tf),     ptr(x.wl),
                     ptr(x.wu)};
    return x;
  }

  // one hd_context per (device, host thread) (SURVEY 8(b) "Threading"); the
  // modules of a thread share it and libhdisort orders their solves, on any
  // streams, behind each other
  static hd_context* context(int device) {
    thread_local std::map<int, std::unique_ptr<hd_context, int (*)(hd_context*)>> ctxs;
    auto it = ctxs.find(device);
    if (it != ctxs.end()) return it->second.get();
    hd_context* c = nullptr;
    int rc = hd_context_create(&c, device);
    TORCH_CHECK(rc == HD_OK, "Disort: ", hd_last_error(nullptr));
    ctxs.emplace(device, std::unique_ptr<hd_context, int (*)(hd_context*)>(c, hd_context_destroy));
    return c;
  }
};
TORCH_MODULE(Disort);

#undef HARP_AMD_ARG

}  // namespace harp_amd
