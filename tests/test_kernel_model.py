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
