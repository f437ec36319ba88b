// The INTEGRATION.md swap at src/radiation/radiation_band.cpp:57-69, compiled.
//
// `BandOptions::disort()` holds an options object with the accessors of
// pydisort's disort::DisortOptions that pyharp uses (header, flags, nwave,
// ncol, wave_lower/upper, user_tau/mu/phi, ds().nlyr/nstr/nmom).  `reset()`
// is RadiationBandImpl::reset's solver block with the one changed line
// (harp_amd::Disort(harp_amd::to_harp_amd(...)) in place of
// disort::Disort(...)); `forward()` is the call at radiation_band.cpp:123-128
// through torch::nn::AnyModule, with and without temf.
//
// Two bands run on two host threads at once (SURVEY 8(b) "Threading": one
// hd_context per (device, host thread)), each three times; the last result
// of each is printed as "band w c l up dn" and checked against the oracle by
// tests/test_gpu_concurrency.py::test_cpp_radiation_band_swap.
#include <harp_amd/disort.hpp>

#include <cmath>
#include <cstdio>
#include <thread>

namespace pyharp_side {

// accessors of pydisort's disort::DisortOptions reached from pyharp
struct DisortState {
  int nlyr = 1, nstr = 4, nmom = 4;
};
struct DisortOptions {
  std::string header_ = "", flags_ = "";
  int nwave_ = 1, ncol_ = 1;
  std::vector<double> wave_lower_, wave_upper_, user_tau_, user_mu_, user_phi_;
  DisortState ds_;
  DisortState& ds() { return ds_; }
  std::string const& header() const { return header_; }
  std::string const& flags() const { return flags_; }
  int nwave() const { return nwave_; }
  int ncol() const { return ncol_; }
  std::vector<double> const& wave_lower() const { return wave_lower_; }
  std::vector<double> const& wave_upper() const { return wave_upper_; }
  std::vector<double> const& user_tau() const { return user_tau_; }
  std::vector<double> const& user_mu() const { return user_mu_; }
  std::vector<double> const& user_phi() const { return user_phi_; }
  DisortOptions& flags(std::string const& v) { flags_ = v; return *this; }
  DisortOptions& nwave(int v) { nwave_ = v; return *this; }
  DisortOptions& ncol(int v) { ncol_ = v; return *this; }
  DisortOptions& wave_lower(std::vector<double> const& v) { wave_lower_ = v; return *this; }
  DisortOptions& wave_upper(std::vector<double> const& v) { wave_upper_ = v; return *this; }
  DisortOptions& user_mu(std::vector<double> const& v) { user_mu_ = v; return *this; }
  DisortOptions& user_phi(std::vector<double> const& v) { user_phi_ = v; return *this; }
};

// the RadiationBandOptions fields reset() reads (radiation_band.hpp:26-51)
struct BandOptions {
  DisortOptions disort_;
  DisortOptions& disort() { return disort_; }
  int nlyr_ = 1, ncol_ = 1;
  int nlyr() const { return nlyr_; }
  int ncol() const { return ncol_; }
  std::vector<double> wave_lower_, wave_upper_;
  std::vector<double> const& wave_lower() const { return wave_lower_; }
  std::vector<double> const& wave_upper() const { return wave_upper_; }
};

struct Band {
  BandOptions options;
  torch::nn::AnyModule rtsolver;

  void reset(int nwave, std::vector<double> const& uphi, std::vector<double> const& umu) {
    // radiation_band.cpp:58-69, the solver block
    options.disort().ds().nlyr = options.nlyr();

    options.disort().nwave(nwave);
    options.disort().ncol(options.ncol());

    options.disort().user_phi(uphi);
    options.disort().user_mu(umu);
    options.disort().wave_lower(options.wave_lower());
    options.disort().wave_upper(options.wave_upper());

    rtsolver = torch::nn::AnyModule(harp_amd::Disort(harp_amd::to_harp_amd(options.disort())));
  }

  // radiation_band.cpp:123-128
  torch::Tensor forward(torch::Tensor prop, std::map<std::string, torch::Tensor>& bc,
                        std::map<std::string, torch::Tensor> const& op) {
    if (op.count("temf") > 0) {
      return rtsolver.forward(prop, &bc, op.at("temf"));
    } else {
      return rtsolver.forward(prop, &bc);
    }
  }
};

}  // namespace pyharp_side

// band 0: SW beam, nstr 8, HG moments; band 1: LW planck, nstr 4, omega = 0
// (tests/test_gpu_concurrency.py::_swap_inputs restates these formulas)
static void inputs(int band, int nwave, int ncol, int nlyr, int nstr, torch::Tensor& prop,
                   std::map<std::string, torch::Tensor>& bc, torch::Tensor& temf) {
  const int nprop = 2 + nstr;
  prop = torch::zeros({nwave, ncol, nlyr, nprop}, torch::kFloat64);
  auto p = prop.accessor<double, 4>();
  for (int w = 0; w < nwave; ++w)
    for (int c = 0; c < ncol; ++c)
      for (int l = 0; l < nlyr; ++l) {
        p[w][c][l][0] = 0.02 * (1 + w) * (1 + (l * 7 + c) % 5);
        if (band == 0) {
          p[w][c][l][1] = 0.5 + 0.04 * ((w + 2 * l + c) % 12);
          const double g = 0.1 + 0.05 * ((l + w) % 10);
          for (int m = 1; m <= nstr; ++m) p[w][c][l][1 + m] = std::pow(g, m);
        }
      }
  auto ones = torch::ones({nwave, ncol}, torch::kFloat64);
  if (band == 0) {
    bc["fbeam"] = ones;
    bc["umu0"] = 0.3 + 0.1 * torch::arange(nwave * ncol, torch::kFloat64).remainder(7).view({nwave, ncol});
    bc["albedo"] = 0.2 * ones;
  } else {
    temf = torch::zeros({ncol, nlyr + 1}, torch::kFloat64);
    auto t = temf.accessor<double, 2>();
    for (int c = 0; c < ncol; ++c)
      for (int l = 0; l <= nlyr; ++l) t[c][l] = 260.0 - 100.0 * l / nlyr + 5.0 * c;
    bc["albedo"] = 0.1 * ones;
    bc["btemp"] = 265.0 * ones;
  }
}

int main() {
  const int nwave[2] = {7, 6}, ncol[2] = {3, 2}, nlyr[2] = {12, 9}, nstr[2] = {8, 4};
  torch::Tensor result[2];
  auto run = [&](int band) {
    pyharp_side::Band b;
    b.options.nlyr_ = nlyr[band];
    b.options.ncol_ = ncol[band];
    b.options.disort().flags(band == 0 ? "lamber,quiet,onlyfl" : "lamber,quiet,onlyfl,planck");
    b.options.disort().ds().nstr = nstr[band];
    b.options.disort().ds().nmom = nstr[band];
    for (int w = 0; w < nwave[band]; ++w) {
      b.options.wave_lower_.push_back(100.0 + 50.0 * w);
      b.options.wave_upper_.push_back(150.0 + 50.0 * w);
    }
    b.reset(nwave[band], {0.0}, {1.0});
    torch::Tensor prop, temf;
    std::map<std::string, torch::Tensor> bc;
    inputs(band, nwave[band], ncol[band], nlyr[band], nstr[band], prop, bc, temf);
    std::map<std::string, torch::Tensor> op;
    if (temf.defined()) op["temf"] = temf;
    for (int it = 0; it < 3; ++it) result[band] = b.forward(prop, bc, op);
  };
  std::thread t0(run, 0), t1(run, 1);
  t0.join();
  t1.join();
  for (int band = 0; band < 2; ++band) {
    auto a = result[band].accessor<double, 4>();
    for (int w = 0; w < nwave[band]; ++w)
      for (int c = 0; c < ncol[band]; ++c)
        for (int l = 0; l <= nlyr[band]; ++l)
          std::printf("%d %d %d %d %.17g %.17g\n", band, w, c, l, a[w][c][l][0], a[w][c][l][1]);
  }
  return 0;
}
