"""Generate tests/golden/cases.npz: small seeded batches + numpy-oracle fluxes.

Run from the repo root:  python tests/golden/make_golden.py
The numpy oracle (oracle/disort_np.py) is the DISORT-structured restatement
pinned by tests/golden/disotest1.json; see its header for parity status.
"""

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle.disort_np import disort_forward, layer2level  # noqa: E402

SEED = 20250217


def make_case(rng, nwave, ncol, nlyr, nstr, nmom, planck, beam=True, ssa_max=0.99,
              gmax=0.85, tau_lo=-5.0, tau_hi=0.7):
    nprop = 2 + nmom
    prop = np.zeros((nwave, ncol, nlyr, nprop))
    prop[..., 0] = 10.0 ** rng.uniform(tau_lo, tau_hi, (nwave, ncol, nlyr))
    prop[..., 1] = rng.uniform(0.0, ssa_max, (nwave, ncol, nlyr))
    g = rng.uniform(0.0, gmax, (nwave, ncol, nlyr))
    for l in range(nmom):
        prop[..., 2 + l] = g ** (l + 1)
    bc = {"albedo": rng.uniform(0.0, 1.0, (nwave, ncol))}
    if beam:
        bc["fbeam"] = np.ones((nwave, ncol))
        bc["umu0"] = rng.uniform(0.05, 1.0, (nwave, ncol))
    temf = wl = wu = None
    if planck:
        tlay = np.linspace(300.0, 150.0, nlyr)[None, :] + rng.uniform(-5, 5, (ncol, nlyr))
        temf = layer2level(tlay)
        bc["btemp"] = np.full((nwave, ncol), 300.0) + rng.uniform(-5, 5, (nwave, ncol))
        wl = np.sort(rng.uniform(10.0, 2500.0, nwave))
        wu = wl + rng.uniform(1.0, 300.0, nwave)
    flux = disort_forward(prop, bc, temf, nstr=nstr, nmom=nmom, planck=planck,
                          wave_lower=wl, wave_upper=wu)
    d = {"prop": prop, "flux": flux, "nstr": nstr, "nmom": nmom, "planck": int(planck)}
    for k, v in bc.items():
        d["bc_" + k] = v
    if planck:
        d.update(temf=temf, wave_lower=wl, wave_upper=wu)
    return d


def main():
    rng = np.random.default_rng(SEED)
    cases = {
        "sw_n4_l5": make_case(rng, 3, 2, 5, 4, 4, False),
        "sw_n8_l12": make_case(rng, 2, 3, 12, 8, 8, False),
        "sw_n16_l20": make_case(rng, 2, 2, 20, 16, 16, False),
        "lw_n8_l10": make_case(rng, 3, 2, 10, 8, 8, True, beam=False, ssa_max=0.0),
        "mix_n16_l10": make_case(rng, 2, 2, 10, 16, 16, True),
        "n2_l6": make_case(rng, 2, 2, 6, 2, 2, True),
        "n6_l7_nomom": make_case(rng, 2, 2, 7, 6, 0, False),
        "n12_l9": make_case(rng, 2, 2, 9, 12, 12, False, ssa_max=0.9999, gmax=0.9),
    }
    flat = {}
    for name, d in cases.items():
        for k, v in d.items():
            flat[f"{name}/{k}"] = np.asarray(v)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cases.npz")
    np.savez_compressed(out, **flat)
    print("wrote", out, sorted(cases))


if __name__ == "__main__":
    main()
