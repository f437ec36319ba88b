"""The kernels' formulation (tests/kernel_model.py) against the oracle, on CPU.

Separates a formulation error (symmetric eigenproblem, flux-weighted layer
operators, adding sweep) from a HIP coding error.
"""

import numpy as np
import pytest

from kernel_model import solve_column
from oracle.disort_np import disort_column


@pytest.mark.parametrize("seed", range(6))
def test_model_matches_oracle(seed):
    rng = np.random.default_rng(100 + seed)
    nstr = [4, 8, 16][seed % 3]
    L = int(rng.integers(1, 15))
    tau = 10 ** rng.uniform(-5, 1.5, L)
    ssa = rng.uniform(0, 0.9999, L)
    g = rng.uniform(0, 0.9, L)
    chis = [[gg ** l for l in range(1, nstr + 1)] for gg in g]
    pmom = np.array([[1.0] + c for c in chis])
    planck = seed % 2 == 1
    kw = dict(planck=planck, temper=np.linspace(150, 300, L + 1), btemp=300.0,
              wvnmlo=100.0, wvnmhi=900.0) if planck else {}
    mu0, A = rng.uniform(0.05, 1), rng.uniform(0, 1)
    r = disort_column(tau, ssa, pmom, nstr, umu0=mu0, fbeam=1.0, albedo=A, **kw)
    fu, fd = solve_column(tau, ssa, chis, nstr, umu0=mu0, fbeam=1.0, albedo=A, **kw)
    scale = max(np.abs(r["flup"]).max(), np.abs(r["fdn"]).max())
    for a, b in ((fu, r["flup"]), (fd, r["fdn"])):
        err = np.abs(a - b) / np.maximum(np.abs(b), 1e-6 * scale)
        assert err.max() < 1e-8


def test_model_exact_conservative_without_dither():
    """The symmetric formulation needs no dither: k -> 0 is regular."""
    import kernel_model
    saved = kernel_model.DITHER
    try:
        kernel_model.DITHER = 0.0
        tau = [0.5, 3.0]
        chis = [[0.5 ** l for l in range(1, 9)]] * 2
        fu, fd = solve_column(tau, [1.0, 1.0], chis, 8, umu0=0.7, fbeam=1.0, albedo=1.0)
    finally:
        kernel_model.DITHER = saved
    assert np.all(np.isfinite(fu)) and np.abs(fd - fu).max() < 1e-12


@pytest.mark.parametrize("seed", range(4))
def test_radiance_model_matches_oracle(seed):
    """tests/kernel_model_rad.py (the radiance kernels' formulation) vs the
    radiance oracle, every azimuthal mode, user depths inside layers."""
    import kernel_model_rad as km
    from oracle.disort_np import plkavg
    from oracle.disort_rad_np import disort_rad_column
    rng = np.random.default_rng(300 + seed)
    nstr = [4, 8, 16, 6][seed]
    L = int(rng.integers(1, 7))
    tau = 10 ** rng.uniform(-3, 0.7, L)
    ssa = rng.uniform(0, 0.99, L)
    g = rng.uniform(0, 0.8, L)
    chis = [[gg ** l for l in range(1, nstr + 1)] for gg in g]
    pmom = np.array([[1.0] + c for c in chis])
    planck = seed % 2 == 1
    umu0, fbeam, alb, fisot = rng.uniform(0.1, 1), 1.7, rng.uniform(0, 1), 0.03
    kw = {}
    pk, bsurf, btop = None, 0.0, 0.0
    if planck:
        temper = np.linspace(180, 290, L + 1)
        kw = dict(planck=True, temper=temper, btemp=295.0, ttemp=160.0, temis=0.4,
                  wvnmlo=300.0, wvnmhi=1000.0)
        pk = np.array([plkavg(300.0, 1000.0, t) for t in temper])
        bsurf, btop = plkavg(300.0, 1000.0, 295.0), 0.4 * plkavg(300.0, 1000.0, 160.0)
    taus = np.concatenate([[0.0], np.cumsum(tau)])
    ut = np.sort(np.concatenate([[0.0, taus[-1]], rng.uniform(0, taus[-1], 3)]))
    umu = np.array([-0.9, -0.35, 0.2, 0.65, 1.0])
    r = disort_rad_column(tau, ssa, pmom, nstr, umu=umu, phi=[0.0], utau=ut, umu0=umu0,
                          fbeam=fbeam, albedo=alb, fisot=fisot, **kw)
    for m in range(nstr):
        ops, ip, im, cp, cm = km.solve_mode(tau, ssa, chis, nstr, m, umu0=umu0, fbeam=fbeam,
                                            albedo=alb, fisot=fisot, pk=pk, bsurf=bsurf,
                                            btop=btop)
        ref = r["uum"][m]
        scale = np.abs(r["uum"][0]).max()
        for iu, mu in enumerate(umu):
            got = km.user_radiance(ops, ip, im, cp, cm, nstr, m, mu, ut, umu0=umu0, fbeam=fbeam,
                                   albedo=alb, fisot=fisot, bsurf=bsurf, btop=btop)
            err = np.abs(got - ref[:, iu]).max() / scale
            assert err < 1e-9, (m, mu, got, ref[:, iu])
