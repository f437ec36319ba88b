// harp_amd/spectral.hpp -- the band epilogue after the solve on the device
// (libhdisort.so, include/hdharp.h): band flux sum_g w_g F_g
// (examples/amars_lw.cpp:84-88), heating rates (examples/amars_sw.cpp:291-302)
// and the spherical flux correction (src/utils/spherical_flux_correction.cpp:3-17).
// Device tensors only: there is no CPU compute path.
#pragma once

#include <ATen/hip/HIPContext.h>
#include <torch/torch.h>

#include "../hdharp.h"
#include "../hdisort.h"

namespace harp_amd {

namespace detail {
inline void* spectral_stream(torch::Device dev) {
  return reinterpret_cast<void*>(at::hip::getCurrentHIPStream(dev.index()).stream());
}
}  // namespace detail

//! (ncol, nlev, 2) = sum_g weight[g] flux[g] for flux (G, ncol, nlev, 2)
inline torch::Tensor band_flux(torch::Tensor flux, torch::Tensor weight) {
  TORCH_CHECK(flux.is_cuda(), "band_flux: device tensor expected");
  TORCH_CHECK(flux.dim() == 4 && flux.size(3) == 2, "band_flux: flux must be (G, ncol, nlev, 2)");
  auto o = torch::TensorOptions().dtype(torch::kFloat64).device(flux.device());
  auto f = flux.to(o).contiguous();
  auto w = weight.to(o).contiguous().view({-1});
  TORCH_CHECK(w.size(0) == f.size(0), "band_flux: one weight per g-point");
  auto out = torch::empty({f.size(1), f.size(2), 2}, o);
  int rc = hd_band_flux(f.data_ptr<double>(), w.data_ptr<double>(), (int)f.size(0),
                        (int)f.size(1), (int)f.size(2), out.data_ptr<double>(),
                        detail::spectral_stream(f.device()));
  TORCH_CHECK(rc == HD_OK, "hd_band_flux: ", hd_last_error(nullptr));
  return out;
}

//! dT/dt (ncol, nlyr) [K/s] from the band flux (ncol, nlyr+1, 2); dz, rho (ncol, nlyr) or (nlyr)
inline torch::Tensor heating_rate(torch::Tensor bflux, torch::Tensor dz, torch::Tensor rho,
                                  double cp) {
  TORCH_CHECK(bflux.is_cuda(), "heating_rate: device tensor expected");
  auto o = torch::TensorOptions().dtype(torch::kFloat64).device(bflux.device());
  auto f = bflux.to(o).contiguous();
  const int ncol = f.size(0), nlyr = f.size(1) - 1;
  auto d = dz.to(o).reshape({-1, nlyr}).expand({ncol, nlyr}).contiguous();
  auto r = rho.to(o).reshape({-1, nlyr}).expand({ncol, nlyr}).contiguous();
  auto out = torch::empty({ncol, nlyr}, o);
  int rc = hd_heating_rate(f.data_ptr<double>(), d.data_ptr<double>(), r.data_ptr<double>(), cp,
                           ncol, nlyr, out.data_ptr<double>(), detail::spectral_stream(f.device()));
  TORCH_CHECK(rc == HD_OK, "hd_heating_rate: ", hd_last_error(nullptr));
  return out;
}

//! in place on a contiguous f64 device band flux (ncol, nlev, 2); x1f, area (nlev), vol (nlev-1)
inline torch::Tensor spherical_flux_correction(torch::Tensor bflux, torch::Tensor x1f,
                                               torch::Tensor area, torch::Tensor vol) {
  TORCH_CHECK(bflux.is_cuda() && bflux.is_contiguous() && bflux.dtype() == torch::kFloat64,
              "spherical_flux_correction: contiguous f64 device tensor expected");
  auto o = torch::TensorOptions().dtype(torch::kFloat64).device(bflux.device());
  auto x = x1f.to(o).contiguous(), a = area.to(o).contiguous(), v = vol.to(o).contiguous();
  int rc = hd_spherical_flux_correction(bflux.data_ptr<double>(), x.data_ptr<double>(),
                                        a.data_ptr<double>(), v.data_ptr<double>(),
                                        (int)bflux.size(0), (int)bflux.size(1),
                                        detail::spectral_stream(bflux.device()));
  TORCH_CHECK(rc == HD_OK, "hd_spherical_flux_correction: ", hd_last_error(nullptr));
  return bflux;
}

}  // namespace harp_amd
