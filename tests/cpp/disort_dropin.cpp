// Drop-in check at the C++ level: the reference's SW call pattern
// (examples/amars_sw.cpp:43-65,216,275-280) with harp_amd::Disort in place of
// disort::Disort.  Prints "flux" and the upward/downward TOA/surface values;
// tests/test_gpu_parity.py::test_cpp_dropin runs it on the GPU box and
// compares against the oracle.
#include <harp_amd/disort.hpp>

#include <cmath>
#include <cstdio>

int main(int argc, char** argv) {
  int nwave = 6, ncol = 2, nlyr = 12, nstr = 8;
  harp_amd::DisortOptions op;
  op.header("running amars RT").flags("lamber,quiet,onlyfl,intensity_correction,old_intensity_correction");
  op.nwave(nwave).ncol(ncol);
  op.ds().nlyr = nlyr;
  op.ds().nstr = nstr;
  op.ds().nmom = nstr;
  harp_amd::Disort disort(op);

  auto prop = torch::zeros({nwave, ncol, nlyr, 2}, torch::kFloat64);
  for (int w = 0; w < nwave; ++w)
    for (int c = 0; c < ncol; ++c)
      for (int l = 0; l < nlyr; ++l) {
        prop[w][c][l][0] = 0.01 * (1 + w) * (1 + l % 3) + 0.05 * c;
        prop[w][c][l][1] = 0.3 + 0.05 * w + 0.02 * (l % 4);
      }
  std::map<std::string, torch::Tensor> bc;
  bc["fbeam"] = torch::ones({nwave, ncol}, torch::kFloat64);
  bc["umu0"] = torch::ones({nwave, ncol}, torch::kFloat64);
  bc["albedo"] = torch::ones({nwave, ncol}, torch::kFloat64);
  auto result = disort->forward(prop, &bc);
  auto acc = result.accessor<double, 4>();
  for (int w = 0; w < nwave; ++w)
    for (int c = 0; c < ncol; ++c)
      for (int l = 0; l <= nlyr; ++l)
        std::printf("%d %d %d %.17g %.17g\n", w, c, l, acc[w][c][l][0], acc[w][c][l][1]);
  // the band sum amars_lw.cpp:84-88 forms next, fused into the solve
  auto wts = 1.0 + 0.1 * torch::arange(nwave, torch::kFloat64);
  auto band = disort->forward_band(prop, &bc, torch::Tensor(), wts).cpu();
  auto bacc = band.accessor<double, 3>();
  for (int c = 0; c < ncol; ++c)
    for (int l = 0; l <= nlyr; ++l)
      std::printf("band %d %d %.17g %.17g\n", c, l, bacc[c][l][0], bacc[c][l][1]);
  return 0;
}
