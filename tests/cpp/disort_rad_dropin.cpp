// The reference's intensity test (tests/test_disort.cpp:13-55, DISOTEST
// problem 1a) with harp_amd::Disort in place of disort::Disort: usrtau/usrang,
// user_mu/phi/tau, isotropic moments from scattering_moments, forward(prop,
// &bc), get_rad().  Prints "flux <lu> <up> <dn>" and "rad <lu> <iu> <value>"
// lines; tests/test_gpu_radiance.py::test_cpp_disort_rad checks them against
// DISOTEST's published values.
#include <harp_amd/disort.hpp>

#include <cmath>
#include <cstdio>

int main() {
  harp_amd::DisortOptions op;
  op.header("running disort example");
  op.flags(
      "usrtau,usrang,lamber,quiet,intensity_correction,"
      "old_intensity_correction,print-input,print-phase-function");
  op.nwave(10);
  op.ds().nlyr = 1;
  op.ds().nstr = 16;
  op.ds().nmom = 16;
  op.user_mu({-1, -0.5, -0.1, 0.1, 0.5, 1});
  op.user_phi({0});
  op.user_tau({0, 0.03125});
  harp_amd::Disort disort(op);

  auto prop = torch::zeros({disort->options.nwave(), disort->options.ncol(),
                            disort->ds().nlyr, 2 + disort->ds().nstr},
                           torch::kDouble);
  prop.select(3, harp_amd::index::IEX) = disort->ds().utau[1];
  prop.select(3, harp_amd::index::ISS) = 0.2;
  prop.narrow(3, harp_amd::index::IPM, disort->ds().nstr) = harp_amd::scattering_moments(
      disort->ds().nstr, harp_amd::PhaseMomentOptions().type(harp_amd::kIsotropic));

  std::map<std::string, torch::Tensor> bc;
  bc["umu0"] = 0.1 * torch::ones({disort->options.nwave(), disort->options.ncol()}, torch::kDouble);
  bc["fbeam"] = M_PI / bc["umu0"];

  auto result = disort->forward(prop, &bc);
  auto rad = disort->get_rad(prop.options());
  for (int lu = 0; lu < 2; ++lu)
    std::printf("flux %d %.9e %.9e\n", lu, result[9][0][lu][0].item<double>(),
                result[9][0][lu][1].item<double>());
  for (int lu = 0; lu < 2; ++lu)
    for (int iu = 0; iu < 6; ++iu)
      std::printf("rad %d %d %.9e\n", lu, iu, rad[9][0][0][lu][iu].item<double>());
  return 0;
}
