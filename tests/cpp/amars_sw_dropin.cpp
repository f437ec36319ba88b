// C++ drop-in check of the whole SW chain: the reference's examples/amars_sw.cpp
// main() (:198-302) with harp_amd:: types in place of harp:: / disort:: --
// attenuators, optics assembly, Disort, band integral, heating rates -- all on
// the device.  Host-side atmosphere setup (regrid_ptx, calc_dz) is the
// example's own code path, restated.  Prints "level F_up F_dn" and
// "layer dT/dt"; tests/test_gpu_harp.py::test_cpp_amars_sw compares with the
// oracle pipeline.  argv[1] = data directory.
#include <harp_amd/disort.hpp>
#include <harp_amd/opacity.hpp>
#include <harp_amd/spectral.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>

static double interp1(double x, std::vector<double> const& ax, std::vector<double> const& v) {
  // interpn.h/locate.h on a monotonic axis, clamped
  const int n = ax.size();
  const bool asc = ax[n - 1] >= ax[0];
  int jl = 0, ju = n + 1;
  while (ju - jl > 1) {
    int jm = (ju + jl) >> 1;
    if ((x >= ax[jm - 1]) == asc) jl = jm;
    else ju = jm;
  }
  int j = x == ax[0] ? 1 : (x == ax[n - 1] ? n : jl);
  int i1 = j - 1, i2;
  if (i1 == -1) i1 = i2 = 0;
  else if (i1 == n - 1) i2 = n - 1;
  else i2 = i1 + 1;
  double x1 = ax[i1], x2 = ax[i2];
  if (x2 != x1) return ((x - x1) * v[i2] + (x2 - x) * v[i1]) / (x2 - x1);
  return (v[i1] + v[i2]) / 2.;
}

int main(int argc, char** argv) {
  if (argc > 1) harp_amd::add_resource_directory(argv[1]);
  const int nwave = 500, ncol = 1, nlyr = 40, nspecies = 2, nstr = argc > 2 ? std::atoi(argv[2]) : 8;
  const double g = 3.711, mean_mol_weight = 0.044, R = 8.314472, cp = 844;
  torch::Device dev(torch::kCUDA, 0);
  auto f64 = torch::TensorOptions().dtype(torch::kFloat64);

  harp_amd::DisortOptions dop;
  dop.header("running amars RT").flags("lamber,quiet,onlyfl,intensity_correction,old_intensity_correction");
  dop.nwave(nwave).ncol(ncol);
  dop.ds().nlyr = nlyr;
  dop.ds().nstr = nstr;
  dop.ds().nmom = nstr;
  harp_amd::Disort disort(dop);

  harp_amd::AttenuatorOptions op;
  op.species_names({"S8", "H2SO4"}).species_weights({256.e-3, 98.e-3});
  op.species_ids({0}).opacity_files({"s8_k_fuller.txt"});
  harp_amd::S8Fuller s8(op);
  op.species_ids({1}).opacity_files({"h2so4.txt"});
  harp_amd::H2SO4Simple h2so4(op);

  auto wave = torch::linspace(2000, 50000, nwave, f64);
  // atmosphere (amars_sw.cpp:104-170, 228-258)
  auto rows = harp_amd::read_table(harp_amd::find_resource("aerosol_output_data.txt"));
  std::vector<double> p, T, mr0, mr1;
  for (auto const& r : rows) {
    p.push_back(r[0] * 1e5);
    T.push_back(r[1]);
    mr0.push_back(r[2]);
    mr1.push_back(r[3]);
  }
  double p_min = *std::min_element(p.begin(), p.end()), p_max = *std::max_element(p.begin(), p.end());
  double T_min = *std::min_element(T.begin(), T.end()), T_max = *std::max_element(T.begin(), T.end());
  std::vector<double> new_p(nlyr), new_T(nlyr), rho(nlyr);
  for (int i = 0; i < nlyr; ++i) {
    new_p[nlyr - 1 - i] = p_min + i * (p_max - p_min) / (nlyr - 1);
    new_T[nlyr - 1 - i] = T_min + i * (T_max - T_min) / (nlyr - 1);
  }
  auto conc = torch::ones({ncol, nlyr, nspecies}, f64);
  for (int k = 0; k < nlyr; ++k) {
    double m0 = interp1(new_p[k], p, mr0), m1 = interp1(new_p[k], p, mr1);
    conc[0][k][0] = (m1 * new_p[k]) / (R * new_T[k]);
    conc[0][k][1] = (m0 * new_p[k]) / (R * new_T[k]);
    rho[k] = (new_p[k] * mean_mol_weight) / (R * new_T[k]);
  }
  auto dz = torch::ones({nlyr}, f64);
  for (int i = 0; i < nlyr - 1; ++i) dz[i] = (new_p[i] - new_p[i + 1]) / (g * rho[i]);
  dz[nlyr - 1] = 2 * dz[nlyr - 2].item<double>();

  std::map<std::string, torch::Tensor> kwargs;
  kwargs["wavenumber"] = wave.to(dev);
  auto prop = harp_amd::band_optics_of(conc.to(dev), dz.to(dev), kwargs, 2, s8, h2so4);

  // bb_toa_flux (amars_sw.cpp:84-102)
  double c1 = 1.19144e-5 * 1e-3, c2 = 1.4388, sr_sun = 2.92842e-5;
  auto fb = 0.7 * sr_sun * c1 * wave.pow(3) / ((c2 * wave / 5772.0).exp() - 1);
  std::map<std::string, torch::Tensor> bc;
  bc["fbeam"] = fb.view({nwave, 1}).to(dev);
  bc["umu0"] = torch::ones({nwave, ncol}, f64.device(dev));
  bc["albedo"] = torch::ones({nwave, ncol}, f64.device(dev));
  auto flux = disort->forward(prop, &bc);

  double dnu = (wave[1] - wave[0]).item<double>();
  auto bflx = harp_amd::band_flux(flux, torch::full({nwave}, dnu, f64.device(dev)));
  auto dTdt = harp_amd::heating_rate(bflx, dz.to(dev), torch::tensor(rho, f64).to(dev), cp);
  auto b = bflx.cpu();
  auto h = dTdt.cpu();
  for (int k = 0; k <= nlyr; ++k)
    std::printf("level %d %.17g %.17g\n", k, b[0][k][0].item<double>(), b[0][k][1].item<double>());
  for (int k = 0; k < nlyr; ++k) std::printf("layer %d %.17g\n", k, h[0][k].item<double>());
  return 0;
}
