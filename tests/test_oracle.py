"""CPU oracle pinned against known answers (no GPU).

The reference's own solver (pydisort/cdisort) is absent, so the oracle is
pinned by: the DISOTEST problem-1 published fluxes (tests/golden/disotest1.json),
closed-form discrete-ordinate answers, energy conservation, agreement between
the two independent restatements (numpy with numpy.linalg.eig + LAPACK banded
LU; C with Jacobi + LINPACK-style banded LU), and the reference's layer2level
values observed by running its code.
"""

import math

import numpy as np
import pytest

from helpers import TOL, case_bc, disotest, load_cases, rel_err
from oracle import disort_np


@pytest.mark.parametrize("impl", ["numpy", "c"])
@pytest.mark.parametrize("case", ["1a", "1b", "1d"])
def test_disotest1(impl, case, oracle_c):
    c = disotest()["cases"][case]
    pm = np.array([[1.0] + [0.0] * 16])
    col = disort_np.disort_column if impl == "numpy" else oracle_c.column
    r = col([c["tau"]], [c["ssalb"]], pm, 16, umu0=0.1, fbeam=math.pi / 0.1)
    for key in ("rfldir", "rfldn", "flup"):
        got = np.asarray(r[key])
        exp = np.asarray(c[key])
        assert np.all(np.abs(got - exp) <= 5e-6 * np.abs(exp) + 1e-6), (key, got, exp)


def test_disotest1b_energy_conservation():
    c = disotest()["cases"]["1b"]
    incoming = math.pi
    out = c["flup"][0] + c["rfldir"][1] + c["rfldn"][1]
    assert abs(out - incoming) < 1e-5  # the published values themselves conserve energy


@pytest.mark.parametrize("t", [150.0, 300.0, 5772.0])
def test_plkavg_full_range(t, oracle_c):
    sig = 5.67032e-8
    full = disort_np.plkavg(1e-3, 1e6, t)
    assert abs(full * math.pi / (sig * t ** 4) - 1.0) < 1e-6
    assert abs(oracle_c.plkavg(1e-3, 1e6, t) - full) <= 1e-14 * full


@pytest.mark.parametrize("lo,hi,t", [(1.0, 150.0, 300.0), (2000.0, 2000.1, 300.0),
                                     (500.0, 504.0, 200.0), (10.0, 2500.0, 250.0),
                                     (3000.0, 9000.0, 150.0)])
def test_plkavg_numpy_vs_c(lo, hi, t, oracle_c):
    a = disort_np.plkavg(lo, hi, t)
    b = oracle_c.plkavg(lo, hi, t)
    assert abs(a - b) <= 1e-13 * abs(a)


def test_plkavg_simpson_branch_consistent():
    # narrow interval (Simpson) vs difference of two wide (series) integrals
    t = 280.0
    narrow = disort_np.plkavg(700.0, 705.0, t)
    wide = disort_np.plkavg(1e-3, 705.0, t) - disort_np.plkavg(1e-3, 700.0, t)
    assert abs(narrow - wide) / narrow < 1e-5


@pytest.mark.parametrize("nstr", [4, 8, 16])
def test_omega0_beam_closed_form(nstr):
    """omega = 0: diffuse field is only the Lambert-reflected beam."""
    tau = np.array([0.1, 0.5, 0.3])
    mu0, f0, alb = 0.6, 2.0, 0.4
    r = disort_np.disort_column(tau, np.zeros(3), np.ones((3, 1)), nstr, umu0=mu0,
                                fbeam=f0, albedo=alb)
    tc = np.concatenate([[0.0], np.cumsum(tau)])
    np.testing.assert_allclose(r["fdn"], mu0 * f0 * np.exp(-tc / mu0), rtol=1e-13)
    mu, w = disort_np.double_gauss(nstr // 2)
    iup = alb * mu0 * f0 * math.exp(-tc[-1] / mu0) / math.pi
    flup = [2 * math.pi * np.sum(w * mu * iup * np.exp(-(tc[-1] - t) / mu)) for t in tc]
    np.testing.assert_allclose(r["flup"], flup, rtol=1e-12)


@pytest.mark.parametrize("nstr", [2, 8, 16])
def test_isothermal_nonscattering_slab(nstr):
    """omega=0, isothermal atmosphere over a black surface at the same T:
    I+ = B everywhere; I- = B (1 - exp(-tau_above/mu))."""
    tau = np.array([0.2, 1.0, 0.05, 2.0])
    t = 250.0
    lo, hi = 400.0, 900.0
    r = disort_np.disort_column(tau, np.zeros(4), np.ones((4, 1)), nstr, planck=True,
                                temper=np.full(5, t), btemp=t, wvnmlo=lo, wvnmhi=hi)
    b = disort_np.plkavg(lo, hi, t)
    mu, w = disort_np.double_gauss(nstr // 2)
    tc = np.concatenate([[0.0], np.cumsum(tau)])
    np.testing.assert_allclose(r["flup"], math.pi * b, rtol=1e-12)
    fdn = [2 * math.pi * np.sum(w * mu * b * (1 - np.exp(-x / mu))) for x in tc]
    np.testing.assert_allclose(r["fdn"], fdn, rtol=1e-11, atol=1e-14 * b)


def test_conservative_scattering_flux_constant():
    tau = np.array([0.3, 2.0, 5.0, 0.7])
    g = 0.7
    pm = np.array([[g ** l for l in range(17)]] * 4)
    r = disort_np.disort_column(tau, np.ones(4), pm, 16, umu0=0.5, fbeam=1.0, albedo=1.0)
    net = r["fdn"] - r["flup"]
    assert np.abs(net).max() < 1e-5 * 0.5  # dither 4.7e-8 leaves a tiny absorption


def test_numpy_vs_c_random(oracle_c):
    rng = np.random.default_rng(4)
    for nstr in (2, 6, 16):
        W, C, L = 2, 3, 9
        prop = np.zeros((W, C, L, 2 + nstr))
        prop[..., 0] = 10 ** rng.uniform(-4, 1, (W, C, L))
        prop[..., 1] = rng.uniform(0, 0.999, (W, C, L))
        g = rng.uniform(0, 0.9, (W, C, L))
        for l in range(nstr):
            prop[..., 2 + l] = g ** (l + 1)
        bc = {"fbeam": np.ones((W, C)), "umu0": rng.uniform(0.05, 1, (W, C)),
              "albedo": rng.uniform(0, 1, (W, C)), "btemp": np.full((W, C), 290.0)}
        temf = np.linspace(290, 180, L + 1)[None, :].repeat(C, 0)
        wl, wu = np.array([300.0, 800.0]), np.array([600.0, 801.0])
        for planck in (False, True):
            a = disort_np.disort_forward(prop, bc, temf, nstr=nstr, planck=planck,
                                         wave_lower=wl, wave_upper=wu)
            b = oracle_c.forward(prop, bc, temf, nstr=nstr, planck=planck,
                                 wave_lower=wl, wave_upper=wu)
            assert rel_err(b, a).max() < 1e-9


@pytest.mark.parametrize("name", sorted(load_cases()))
def test_c_oracle_reproduces_golden(name, oracle_c):
    d = load_cases()[name]
    f = oracle_c.forward(d["prop"], case_bc(d), d.get("temf"), nstr=int(d["nstr"]),
                         nmom=int(d["nmom"]), planck=bool(d["planck"]),
                         wave_lower=d.get("wave_lower"), wave_upper=d.get("wave_upper"))
    assert rel_err(f, d["flux"]).max() < TOL


def test_layer2level_matches_reference_run():
    # values printed by the reference's own layer2level
    out = disort_np.layer2level([300.0, 280.0, 260.0, 250.0, 240.0])
    np.testing.assert_allclose(out, [310.0, 290.0, 269.1666666667, 254.1666666667, 245.0, 240.0],
                               rtol=1e-10)


@pytest.mark.parametrize("nstr", [8, 32])
def test_umu0_range_check_in_both_oracles(nstr, oracle_c):
    """umu0 is taken as given (pydisort passes it to cdisort; no floor): with fbeam > 0
    a cosine outside (0, 1] is cdisort's input error (c_chekin) in both restatements;
    without a beam it is not looked at; tiny positive cosines solve, numpy == C."""
    rng = np.random.default_rng(77 + nstr)
    nlyr = 6
    u = np.array([[1e-4, 1e-3, 2e-3, 1.0]])
    prop = np.zeros((1, u.shape[1], nlyr, 2 + nstr))
    prop[..., 0] = 10.0 ** rng.uniform(-4, -1, (nlyr,))  # thin: the grazing beam survives
    prop[..., 1] = rng.uniform(0.2, 0.95, (nlyr,))
    g = rng.uniform(0.1, 0.8, (nlyr,))
    for l in range(nstr):
        prop[..., 2 + l] = g ** (l + 1)
    bc = {"fbeam": np.ones_like(u), "umu0": u, "albedo": np.full_like(u, 0.3)}
    fc = oracle_c.forward(prop, bc, nstr=nstr)
    fn = disort_np.disort_forward(prop, bc, nstr=nstr)
    assert rel_err(fn, fc).max() < 1e-9
    assert np.abs(fc[0, 0] - fc[0, 1]).max() > 1e-6 * np.abs(fc[0, 1]).max()
    assert fc[0, 0, -1, 1] > 0.0  # a grazing beam shines at the top
    for bad in (-0.4, 0.0, 1.5, np.nan):
        bb = dict(bc, umu0=np.array([[0.5, bad, 0.5, 0.5]]))
        with pytest.raises(ArithmeticError):
            oracle_c.forward(prop, bb, nstr=nstr)
        with pytest.raises(ValueError):
            disort_np.disort_forward(prop, bb, nstr=nstr)
        # no beam: umu0 is not an input of the solve
        nb = dict(bb, fbeam=np.array([[1.0, 0.0, 1.0, 1.0]]))
        f0 = oracle_c.forward(prop, nb, nstr=nstr)
        assert np.all(np.isfinite(f0)) and np.all(f0[0, 1] == 0.0)
