"""amars SW case on the device, step for step as pyharp's examples/amars_sw.cpp.

    python examples/amars_sw.py [--nstr 8] [--nwave 500] [--nlyr 40] [--data DIR]

Atmosphere (amars_sw.cpp:228-258): the aerosol profile aerosol_output_data.txt
regridded to nlyr uniform-pressure layers; S8 and H2SO4 aerosol optics from
s8_k_fuller.txt and h2so4.txt (S8Fuller / H2SO4Simple, :221-227), assembled
into prop on the GPU (pyharp_amd.opacity.band_optics, :261-271); a scaled
5772 K blackbody beam at umu0 = 1 over an albedo-1 surface (:273-278); the
DISORT flux solve (:280); the spectral integral with d(wavenumber) weights
(:174-196) and the heating rates (:291-302).  Every step after reading the
text tables runs in libhdisort.so.
"""

from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pyharp_amd import Disort, DisortOptions  # noqa: E402
from pyharp_amd.opacity import (AttenuatorOptions, H2SO4Simple, S8Fuller,  # noqa: E402
                                add_resource_directory, find_resource, read_table)
from pyharp_amd.spectral import band_flux, heating_rate  # noqa: E402

G = 3.711
MEAN_MOL_WEIGHT = 0.044
R_GAS = 8.314472
CP = 844.0
SOLAR_TEMP = 5772.0
LUM_SCALE = 0.7


def _interp1(x, axis, data):
    """the example's interpolate_mixing_ratios (amars_sw.cpp:24-36) on host data"""
    order = np.argsort(axis)
    return np.interp(x, axis[order], data[order])


def atmosphere(nlyr: int):
    """(conc (1, nlyr, 2) [mol/m^3], rho (nlyr,), dz (nlyr,), p (nlyr,)) --
    amars_sw.cpp:128-170, 228-258 (host-side setup of the example)."""
    t = read_table(find_resource("aerosol_output_data.txt"))
    p, T = t[:, 0] * 1e5, t[:, 1]
    mr = [t[:, 2], t[:, 3]]
    p_step = (p.max() - p.min()) / (nlyr - 1)
    T_step = (T.max() - T.min()) / (nlyr - 1)
    new_p = np.array([p.min() + (nlyr - 1 - k) * p_step for k in range(nlyr)])
    new_T = np.array([T.min() + (nlyr - 1 - k) * T_step for k in range(nlyr)])
    new_mr = [_interp1(new_p, p, m) for m in mr]
    conc = np.zeros((1, nlyr, 2))
    conc[0, :, 0] = new_mr[1] * new_p / (R_GAS * new_T)   # S8 (second in the file)
    conc[0, :, 1] = new_mr[0] * new_p / (R_GAS * new_T)   # H2SO4
    rho = new_p * MEAN_MOL_WEIGHT / (R_GAS * new_T)
    dz = np.ones(nlyr)
    dz[:-1] = (new_p[:-1] - new_p[1:]) / (G * rho[:-1])
    dz[-1] = 2.0 * dz[-2]
    return conc, rho, dz, new_p


def bb_toa_flux(wave: np.ndarray, ncol: int) -> np.ndarray:
    """amars_sw.cpp:84-102"""
    c1, c2, sr_sun = 1.19144e-5 * 1e-3, 1.4388, 2.92842e-5
    f = LUM_SCALE * sr_sun * c1 * wave ** 3 / (np.exp(c2 * wave / SOLAR_TEMP) - 1.0)
    return np.repeat(f[:, None], ncol, axis=1)


def run(nstr=8, nwave=500, nlyr=40, device=0):
    dev = torch.device("cuda", device)
    op = AttenuatorOptions().species_names(["S8", "H2SO4"]).species_weights([256.e-3, 98.e-3])
    s8 = S8Fuller(op.copy().species_ids([0]).opacity_files(["s8_k_fuller.txt"]))
    h2so4 = H2SO4Simple(op.copy().species_ids([1]).opacity_files(["h2so4.txt"]))
    from pyharp_amd.opacity import band_optics

    wave = np.linspace(2000.0, 50000.0, nwave)
    conc, rho, dz, p = atmosphere(nlyr)
    kw = {"wavenumber": torch.as_tensor(wave, device=dev)}
    prop = band_optics([s8, h2so4], torch.as_tensor(conc, device=dev),
                       torch.as_tensor(dz, device=dev), kw)
    dop = DisortOptions().header("running amars RT").flags(
        "lamber,quiet,onlyfl,intensity_correction,old_intensity_correction")
    dop.nwave(nwave).ncol(1).device(device)
    dop.ds().nlyr, dop.ds().nstr, dop.ds().nmom = nlyr, nstr, nstr
    bc = {"fbeam": torch.as_tensor(bb_toa_flux(wave, 1), device=dev),
          "umu0": torch.ones((nwave, 1), dtype=torch.float64, device=dev),
          "albedo": torch.ones((nwave, 1), dtype=torch.float64, device=dev)}
    flux = Disort(dop).forward(prop, bc)
    dnu = torch.full((nwave,), wave[1] - wave[0], dtype=torch.float64, device=dev)
    bflx = band_flux(flux, dnu)                      # (1, nlyr+1, 2) W/m^2
    dTdt = heating_rate(bflx, torch.as_tensor(dz, device=dev),
                        torch.as_tensor(rho, device=dev), CP)
    return {"prop": prop, "flux": flux, "bflux": bflx, "dTdt": dTdt, "p": p, "dz": dz,
            "rho": rho, "conc": conc, "wave": wave}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nstr", type=int, default=8)
    ap.add_argument("--nwave", type=int, default=500)
    ap.add_argument("--nlyr", type=int, default=40)
    ap.add_argument("--data", default=os.path.join(ROOT, "tests", "golden", "data"))
    a = ap.parse_args()
    add_resource_directory(a.data)
    r = run(a.nstr, a.nwave, a.nlyr)
    b = r["bflux"].cpu().numpy()[0]
    print(f"tot_flux_down_surf: {b[0, 1]:.6f} W/m^2")
    print(f"tot_flux_down_toa: {b[-1, 1]:.6f} W/m^2")
    print("#p[Pa] dT_ds[K/s]")
    for pk, h in zip(r["p"], r["dTdt"].cpu().numpy()[0]):
        print(f"{pk:.6e} {h:.6e}")


if __name__ == "__main__":
    main()
