// The reference's examples/amars_lw.cpp main() with the harp_amd modules in place
// of harp::RFM / disort::Disort / harp::read_weights_rfm: RFM CO2 and H2O optics
// from a classic-netCDF ck table (argv[1] = its directory), the Planck solve at
// 10 bar / 300 K over an albedo-1 surface, the ck-weighted band flux.  Prints
// "prop", "flux" and "bflx" lines; tests/test_gpu_harp.py::test_cpp_amars_lw
// checks them against the oracles.
#include <harp_amd/disort.hpp>
#include <harp_amd/opacity.hpp>

#include <cstdio>

int main(int argc, char** argv) {
  if (argc > 1) harp_amd::add_resource_directory(argv[1]);
  harp_amd::AttenuatorOptions op;
  op.species_names({"CO2", "H2O"});
  op.species_weights({44.0e-3, 18.0e-3});
  op.species_ids({0}).opacity_files({"amarsw-ck-B1.nc"});
  harp_amd::RFM co2(op);
  op.species_ids({1}).opacity_files({"amarsw-ck-B1.nc"});
  harp_amd::RFM h2o(op);

  int nwave = co2->kdata.size(0), ncol = 1, nlyr = 40, nspecies = 2;
  auto dev = torch::Device(torch::kCUDA, 0);
  auto f64 = torch::TensorOptions().dtype(torch::kFloat64).device(dev);
  auto conc = torch::ones({ncol, nlyr, nspecies}, f64);

  harp_amd::DisortOptions dop;
  dop.header("running amars lw");
  dop.flags("lamber,quiet,onlyfl,planck,intensity_correction,old_intensity_correction,"
            "print-input,print-phase-function,print-fluxes");
  dop.nwave(nwave).ncol(ncol);
  dop.wave_lower(std::vector<double>(nwave, 1.)).wave_upper(std::vector<double>(nwave, 150.));
  dop.ds().nlyr = nlyr;
  dop.ds().nstr = 8;
  dop.ds().nmom = 8;
  harp_amd::Disort disort(dop);

  std::map<std::string, torch::Tensor> kwargs;
  kwargs["pres"] = torch::ones({ncol, nlyr}, f64) * 10.e5;
  kwargs["temp"] = torch::ones({ncol, nlyr}, f64) * 300.0;
  auto prop = co2->forward(conc, kwargs) + h2o->forward(conc, kwargs);

  std::map<std::string, torch::Tensor> bc;
  bc["albedo"] = torch::ones({nwave, ncol}, f64);
  bc["btemp"] = torch::ones({nwave, ncol}, f64) * 300.0;
  // layer2level of an isothermal profile is the same constant at every level
  auto temf = torch::ones({ncol, nlyr + 1}, f64) * 300.0;
  auto flux = disort->forward(prop, &bc, temf);
  auto weights = harp_amd::read_weights_rfm("amarsw-ck-B1.nc").to(dev);
  auto bflx = (flux * weights.view({-1, 1, 1, 1})).sum(0).cpu();
  auto pc = prop.cpu();
  for (int w = 0; w < nwave; ++w) std::printf("prop %d %.17e\n", w, pc[w][0][0][0].item<double>());
  for (int l = 0; l <= nlyr; ++l)
    std::printf("bflx %d %.17e %.17e\n", l, bflx[0][l][0].item<double>(),
                bflx[0][l][1].item<double>());
  return 0;
}
