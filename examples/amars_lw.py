"""amars LW correlated-k case on the device, as pyharp's examples/amars_lw.cpp.

    python examples/amars_lw.py [--nstr 8] [--ngpoint 16] [--nlyr 40]

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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nstr", type=int, default=8)
    ap.add_argument("--ngpoint", type=int, default=16)
    ap.add_argument("--nlyr", type=int, default=40)
    a = ap.parse_args()
    r = run(a.nstr, a.ngpoint, a.nlyr)
    print("bflx =", r["bflux"].cpu().numpy())


if __name__ == "__main__":
    main()
