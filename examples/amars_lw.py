"""amars LW correlated-k case on the device, as pyharp's examples/amars_lw.cpp.

    python examples/amars_lw.py [--nstr 8] [--ngpoint 16] [--nlyr 40] [--table FILE.nc]

With ``--table`` (an RFM ck file in classic netCDF, e.g. amarsw-ck-B1.nc
converted with ``nccopy -k classic``) this is amars_lw.cpp:40-88 step for
step: RFM CO2 and H2O attenuators on the device (pyharp_amd.opacity.RFM),
prop = prop1 + prop2, the Planck solve and the band flux with the file's ck
weights (read_weights_rfm).  Without it:

The reference reads CO2/H2O k-distributions from amarsw-ck-B1.nc through RFM
(amars_lw.cpp:41-60); that file is git-ignored upstream and netCDF is not in
this image, so the g-point optical depths here are synthetic (SURVEY 8(d) C1:
tau log-uniform [1e-4, 20], omega = 0) and the ck weights are the Gauss
weights of the g interval.  Everything else follows the example: isothermal
300 K layers at 10 bar, temf = layer2level(temp) (:76), albedo 1 and
btemp 300 K (:72-74), wave bounds [1, 150] cm^-1 for every g (:23-31), the
Planck flux solve (:80) and the band flux sum_g w_g F_g (:84-88).
"""

from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pyharp_amd import Disort, DisortOptions, layer2level  # noqa: E402
from pyharp_amd.opacity import RFM, AttenuatorOptions, read_weights_rfm  # noqa: E402
from pyharp_amd.spectral import band_flux  # noqa: E402


def run(nstr=8, ngpoint=16, nlyr=40, ncol=1, device=0, seed=20250217):
    dev = torch.device("cuda", device)
    wmin, wmax = 1.0, 150.0
    op = DisortOptions().header("running amars LW").flags(
        "lamber,quiet,onlyfl,planck,print-input,print-fluxes,print-phase-function")
    op.nwave(ngpoint).ncol(ncol).device(device)
    op.wave_lower([wmin] * ngpoint).wave_upper([wmax] * ngpoint)
    op.ds().nlyr, op.ds().nstr, op.ds().nmom = nlyr, nstr, nstr
    rng = np.random.default_rng(seed)
    prop = torch.zeros((ngpoint, ncol, nlyr, 1), dtype=torch.float64, device=dev)
    prop[..., 0] = torch.as_tensor(10.0 ** rng.uniform(-4, np.log10(20.0), (ngpoint, ncol, nlyr)))
    temp = torch.full((ncol, nlyr), 300.0, dtype=torch.float64, device=dev)
    temf = layer2level(temp)
    bc = {"albedo": torch.ones((ngpoint, ncol), dtype=torch.float64, device=dev),
          "btemp": torch.full((ngpoint, ncol), 300.0, dtype=torch.float64, device=dev)}
    flux = Disort(op).forward(prop, bc, temf)
    x, w = np.polynomial.legendre.leggauss(ngpoint)
    weights = torch.as_tensor(0.5 * w, device=dev)  # ck weights of g in [0, 1]
    return {"prop": prop, "flux": flux, "temf": temf, "bflux": band_flux(flux, weights)}


def run_rfm(table, nstr=8, nlyr=40, ncol=1, device=0):
    """amars_lw.cpp:40-88 with the RFM tables of `table`"""
    dev = torch.device("cuda", device)
    op = AttenuatorOptions().species_names(["CO2", "H2O"]).species_weights([44.0e-3, 18.0e-3])
    co2 = RFM(op.copy().species_ids([0]).opacity_files([table]))
    h2o = RFM(op.copy().species_ids([1]).opacity_files([table]))
    nwave = co2.kdata.shape[0]
    conc = torch.ones((ncol, nlyr, 2), dtype=torch.float64, device=dev)
    kwargs = {"pres": torch.full((ncol, nlyr), 10.e5, dtype=torch.float64, device=dev),
              "temp": torch.full((ncol, nlyr), 300.0, dtype=torch.float64, device=dev)}
    prop = co2.forward(conc, kwargs) + h2o.forward(conc, kwargs)
    dop = DisortOptions().header("running amars lw").flags(
        "lamber,quiet,onlyfl,planck,intensity_correction,old_intensity_correction,"
        "print-input,print-phase-function,print-fluxes")
    dop.nwave(nwave).ncol(ncol).device(device)
    dop.wave_lower([1.0] * nwave).wave_upper([150.0] * nwave)
    dop.ds().nlyr, dop.ds().nstr, dop.ds().nmom = nlyr, nstr, nstr
    bc = {"albedo": torch.ones((nwave, ncol), dtype=torch.float64, device=dev),
          "btemp": torch.full((nwave, ncol), 300.0, dtype=torch.float64, device=dev)}
    temf = layer2level(kwargs["temp"])
    flux = Disort(dop).forward(prop, bc, temf)
    weights = read_weights_rfm(table).to(dev)
    return {"prop": prop, "flux": flux, "temf": temf, "weights": weights,
            "bflux": band_flux(flux, weights)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nstr", type=int, default=8)
    ap.add_argument("--ngpoint", type=int, default=16)
    ap.add_argument("--nlyr", type=int, default=40)
    ap.add_argument("--table", default=None)
    a = ap.parse_args()
    r = run_rfm(a.table, a.nstr, a.nlyr) if a.table else run(a.nstr, a.ngpoint, a.nlyr)
    print("bflx =", r["bflux"].cpu().numpy())


if __name__ == "__main__":
    main()
