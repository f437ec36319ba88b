"""CPU pins of the intensity-path oracle (oracle/disort_rad_np.py), no GPU.

cdisort is absent, so the radiance restatement is pinned
by answers that do not depend on it:
  * at the quadrature cosines the source-function integration reproduces the
    discrete-ordinate intensities of the banded solution (m = 0);
  * fluxes at the level depths equal the flux oracle's (oracle/disort_np.py);
  * omega = 0 slab: the Lambert-reflected beam radiance in closed form, and the
    thermal radiance of a linear-in-tau source by independent quadrature;
  * single scattering of an optically thin Rayleigh layer (a phase function the
    truncated expansion represents exactly), azimuth dependence included;
  * isotropic scattering has no azimuth dependence;
  * the Nakajima-Tanaka correction: TMS restores the exact single scattering
    of a thin Henyey-Greenstein layer; the IMS term's xi function equals its
    defining double integral (STWL A.16) by quadrature, and with TMS + IMS the
    aureole radiances of a forward-peaked layer at nstr 16 approach those of
    nstr 64 (where the truncation is negligible) far closer than with TMS
    alone -- the IMS sign and size are pinned by the physics, not by cdisort.
"""

import math

import numpy as np
import pytest
import scipy.integrate

from oracle import disort_np
from oracle import disort_rad_np
from oracle.disort_rad_np import disort_rad_column, disort_rad_forward, lepoly, xi_func


def test_lepoly_normalisation():
    """sum_m (2 - delta_m0) Y_l^m(a) Y_l^m(b) cos(m dphi) = P_l(cos Theta) (addition theorem)"""
    a, b, dphi = 0.3, -0.7, 1.1
    cos_t = a * b + math.sqrt(1 - a * a) * math.sqrt(1 - b * b) * math.cos(dphi)
    nstr = 8
    p = disort_np.legendre_table(nstr, [cos_t])[:, 0]
    s = np.zeros(nstr)
    for m in range(nstr):
        s += (2 - (m == 0)) * lepoly(nstr, m, [a])[:, 0] * lepoly(nstr, m, [b])[:, 0] * \
            math.cos(m * dphi)
    np.testing.assert_allclose(s, p, rtol=1e-12, atol=1e-14)


def _random_column(rng, nlyr, nstr, iso=False):
    dtauc = 10.0 ** rng.uniform(-2, 0.5, nlyr)
    ssalb = rng.uniform(0.0, 0.95, nlyr)
    pm = np.zeros((nlyr, nstr + 1))
    pm[:, 0] = 1.0
    if not iso:
        g = rng.uniform(0.0, 0.7, nlyr)
        for l in range(1, nstr + 1):
            pm[:, l] = g ** l
    return dtauc, ssalb, pm


@pytest.mark.parametrize("planck", [False, True])
def test_quadrature_angles_reproduce_banded_solution(planck):
    rng = np.random.default_rng(3)
    nstr, nlyr = 8, 5
    dtauc, ssalb, pm = _random_column(rng, nlyr, nstr)
    mu, _ = disort_np.double_gauss(nstr // 2)
    umu = np.concatenate([-mu[::-1], mu])
    kw = dict(umu0=0.6, fbeam=1.3, albedo=0.4, fisot=0.02)
    if planck:
        kw.update(planck=True, temper=np.linspace(200, 290, nlyr + 1), btemp=300.0,
                  ttemp=150.0, temis=0.3, wvnmlo=300.0, wvnmhi=900.0)
    tauc = np.concatenate([[0.0], np.cumsum(dtauc)])
    r = disort_rad_column(dtauc, ssalb, pm, nstr, umu=umu, phi=[0.0], utau=tauc,
                          onlyfl=False, **kw)
    ref = disort_np.disort_column(dtauc, ssalb, pm, nstr, return_all=True, **kw)
    # m = 0 part of the radiance at +/- mu_i
    u0 = r["uum"][0]
    nn = nstr // 2
    np.testing.assert_allclose(u0[:, nn:], ref["uu"][:, :nn], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(u0[:, :nn][:, ::-1], ref["uu"][:, nn:], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(r["flup"], ref["flup"], rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(r["fdn"], ref["fdn"], rtol=1e-10, atol=1e-13)


def test_user_depths_inside_layers_match_flux_continuity():
    """fluxes at depths inside layers: net flux of a conservative, non-absorbing
    column is the same at every depth"""
    nstr, nlyr = 8, 4
    dtauc = np.array([0.3, 1.0, 0.2, 2.0])
    ssalb = np.ones(nlyr)
    pm = np.zeros((nlyr, nstr + 1))
    pm[:, 0] = 1.0
    pm[:, 2] = 0.1
    ut = np.sort(np.random.default_rng(0).uniform(0, dtauc.sum(), 9))
    r = disort_rad_column(dtauc, ssalb, pm, nstr, umu=[0.5], phi=[0.0], utau=ut, umu0=0.7,
                          fbeam=2.0, albedo=1.0, onlyfl=True)
    net = r["fdn"] - r["flup"]
    assert np.abs(net).max() < 1e-6 * 2.0 * 0.7


def test_absorbing_slab_reflected_beam_closed_form():
    nstr, nlyr = 8, 3
    dtauc = np.array([0.2, 0.5, 0.3])
    pm = np.zeros((nlyr, nstr + 1))
    pm[:, 0] = 1.0
    umu0, fbeam, alb = 0.55, 3.0, 0.35
    umu = np.array([-0.9, -0.3, 0.2, 0.6, 1.0])
    ut = np.array([0.0, 0.1, 0.7, 1.0])
    r = disort_rad_column(dtauc, np.zeros(nlyr), pm, nstr, umu=umu, phi=[0.0, 90.0], utau=ut,
                          umu0=umu0, fbeam=fbeam, albedo=alb)
    tb = dtauc.sum()
    for k, t in enumerate(ut):
        for iu, mu in enumerate(umu):
            exp = alb / math.pi * umu0 * fbeam * math.exp(-tb / umu0) * math.exp(-(tb - t) / mu) \
                if mu > 0 else 0.0
            np.testing.assert_allclose(r["uu"][:, k, iu], exp, rtol=1e-12, atol=1e-15)


def test_absorbing_slab_thermal_by_quadrature():
    nstr, nlyr = 4, 3
    dtauc = np.array([0.4, 0.1, 0.9])
    pm = np.zeros((nlyr, nstr + 1))
    pm[:, 0] = 1.0
    temper = np.array([180.0, 220.0, 260.0, 300.0])
    wl, wu = 400.0, 700.0
    pk = [disort_np.plkavg(wl, wu, t) for t in temper]
    bsurf, btop = disort_np.plkavg(wl, wu, 310.0), 0.4 * disort_np.plkavg(wl, wu, 120.0)
    alb = 0.25
    tauc = np.concatenate([[0.0], np.cumsum(dtauc)])

    def bsrc(t):
        lc = min(int(np.searchsorted(tauc[1:], t)), nlyr - 1)
        return pk[lc] + (pk[lc + 1] - pk[lc]) * (t - tauc[lc]) / dtauc[lc]

    umu = np.array([-0.8, -0.25, 0.35, 0.9])
    ut = np.array([0.0, 0.3, 0.45, 1.4])
    r = disort_rad_column(dtauc, np.zeros(nlyr), pm, nstr, umu=umu, phi=[0.0], utau=ut,
                          albedo=alb, planck=True, temper=temper, btemp=310.0, ttemp=120.0,
                          temis=0.4, wvnmlo=wl, wvnmhi=wu)
    # the Lambert surface reflects the quadrature (not exact) downward flux: take it from
    # the oracle's own flux at the bottom, which the flux oracle pins separately
    fdn_b = disort_np.disort_column(dtauc, np.zeros(nlyr), pm, nstr, albedo=alb, planck=True,
                                    temper=temper, btemp=310.0, ttemp=120.0, temis=0.4,
                                    wvnmlo=wl, wvnmhi=wu)["fdn"][-1]
    tb = tauc[-1]
    ibot = alb * fdn_b / math.pi + (1 - alb) * bsurf
    for k, t in enumerate(ut):
        for iu, mu in enumerate(umu):
            if mu > 0:
                f = lambda s: bsrc(s) * math.exp(-(s - t) / mu) / mu  # noqa: E731
                val = ibot * math.exp(-(tb - t) / mu) + scipy.integrate.quad(
                    f, t, tb, points=list(tauc[1:-1]), epsabs=1e-14, epsrel=1e-12)[0]
            else:
                am = -mu
                f = lambda s: bsrc(s) * math.exp(-(t - s) / am) / am  # noqa: E731
                val = btop * math.exp(-t / am)
                if t > 0:
                    val += scipy.integrate.quad(f, 0.0, t, points=list(tauc[1:-1]),
                                                epsabs=1e-14, epsrel=1e-12)[0]
            assert abs(r["uu"][0, k, iu] - val) <= 1e-9 * abs(val), (k, iu)


@pytest.mark.parametrize("nstr", [4, 8])
def test_thin_rayleigh_layer_single_scattering(nstr):
    """tau = 1e-5: the radiance is the single-scattering one to O(tau)."""
    tau, om, chi2 = 1e-5, 0.8, 0.1
    pm = np.zeros((1, nstr + 1))
    pm[0, 0] = 1.0
    pm[0, 2] = chi2
    umu0, phi0, fbeam = 0.6, 30.0, 2.0
    umu = np.array([-0.95, -0.4, 0.3, 0.75])
    phi = np.array([0.0, 45.0, 170.0])
    r = disort_rad_column([tau], [om], pm, nstr, umu=umu, phi=phi, utau=[0.0, tau],
                          umu0=umu0, phi0=phi0, fbeam=fbeam)

    def pfun(mu, dphi):  # p(cos Theta) between the beam (-umu0) and (mu, phi)
        ct = -mu * umu0 + math.sqrt(1 - mu * mu) * math.sqrt(1 - umu0 ** 2) * math.cos(dphi)
        return 1.0 + 5.0 * chi2 * 0.5 * (3 * ct * ct - 1)

    for j, ph in enumerate(phi):
        dphi = math.radians(ph - phi0)
        for iu, mu in enumerate(umu):
            p = pfun(mu, dphi)
            if mu > 0:   # reflected, at the top
                got = r["uu"][j, 0, iu]
                exp = om * fbeam / (4 * math.pi) * p * umu0 / (umu0 + mu) * \
                    -math.expm1(-tau * (1 / umu0 + 1 / mu))
            else:        # transmitted diffuse, at the bottom
                am = -mu
                got = r["uu"][j, 1, iu]
                exp = om * fbeam / (4 * math.pi) * p * umu0 / (umu0 - am) * \
                    (math.exp(-tau / umu0) - math.exp(-tau / am))
            assert abs(got - exp) <= 1e-4 * abs(exp), (j, iu, got, exp)


def test_isotropic_scattering_has_no_azimuth_dependence():
    rng = np.random.default_rng(11)
    nstr, nlyr = 8, 3
    dtauc, ssalb, pm = _random_column(rng, nlyr, nstr, iso=True)
    r = disort_rad_column(dtauc, ssalb, pm, nstr, umu=[-0.5, 0.5], phi=[0.0, 60.0, 180.0],
                          utau=[0.0, 0.5 * dtauc.sum()], umu0=0.4, fbeam=1.0, albedo=0.2)
    np.testing.assert_allclose(r["uu"][1], r["uu"][0], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(r["uu"][2], r["uu"][0], rtol=1e-12, atol=1e-15)


def test_forward_driver_levels_match_flux_oracle():
    rng = np.random.default_rng(5)
    nwave, ncol, nlyr, nstr = 2, 2, 4, 8
    prop = np.zeros((nwave, ncol, nlyr, 2 + nstr))
    prop[..., 0] = rng.uniform(0.01, 2, (nwave, ncol, nlyr))
    prop[..., 1] = rng.uniform(0, 0.9, (nwave, ncol, nlyr))
    g = rng.uniform(0, 0.6, (nwave, ncol, nlyr))
    for l in range(nstr):
        prop[..., 2 + l] = g ** (l + 1)
    bc = {"fbeam": np.ones((nwave, ncol)), "umu0": rng.uniform(0.2, 1, (nwave, ncol)),
          "albedo": rng.uniform(0, 1, (nwave, ncol))}
    flux, uu = disort_rad_forward(prop, bc, nstr=nstr, umu=[-0.5, 0.5], phi=[0.0])
    ref = disort_np.disort_forward(prop, bc, nstr=nstr)
    np.testing.assert_allclose(flux, ref, rtol=1e-10, atol=1e-13)
    assert uu.shape == (nwave, ncol, 1, nlyr + 1, 2)


@pytest.mark.parametrize("case", ["1a", "1b", "1d"])
def test_disotest1_intensities(case):
    """DISOTEST problem 1 (= tests/test_disort.cpp's configuration for 1a):
    published radiances at the six user angles, top and bottom."""
    from helpers import disotest
    g = disotest()
    c = g["cases"][case]
    pm = np.zeros((1, 17))
    pm[0, 0] = 1.0
    r = disort_rad_column([c["tau"]], [c["ssalb"]], pm, 16, umu=g["common"]["umu"],
                          phi=[0.0], utau=[0.0, c["tau"]], umu0=0.1, fbeam=math.pi / 0.1)
    exp = np.asarray(c["uu"])
    assert np.all(np.abs(r["uu"][0] - exp) <= 5e-6 * np.abs(exp) + 1e-6)


def test_tms_restores_exact_single_scattering():
    """Thin Henyey-Greenstein layer (g = 0.75, 64 moments) with delta-M at nstr 8:
    the TMS-corrected radiance is the single scattering of the full phase
    function; the uncorrected delta-M radiance is not."""
    tau, om, g, nmom = 1e-5, 0.9, 0.75, 64
    pm = np.array([[g ** l for l in range(nmom + 1)]])
    umu0, phi0, fbeam = 0.5, 0.0, 1.0
    umu = np.array([-0.8, -0.3, 0.2, 0.7])
    phi = np.array([0.0, 90.0, 180.0])
    kw = dict(umu=umu, phi=phi, utau=[0.0, tau], umu0=umu0, phi0=phi0, fbeam=fbeam)
    r = disort_rad_column([tau], [om], pm, 8, corint=True, **kw)
    r0 = disort_rad_column([tau], [om], pm, 8, corint=False, **kw)

    def hg(ct):
        return (1 - g * g) / (1 + g * g - 2 * g * ct) ** 1.5

    worst_c = worst_0 = 0.0
    for j, ph in enumerate(phi):
        for iu, mu in enumerate(umu):
            ct = -mu * umu0 + math.sqrt(1 - mu * mu) * math.sqrt(1 - umu0 ** 2) * \
                math.cos(math.radians(ph - phi0))
            if mu > 0:
                k = 0
                exp = om * fbeam / (4 * math.pi) * hg(ct) * umu0 / (umu0 + mu) * \
                    -math.expm1(-tau * (1 / umu0 + 1 / mu))
            else:
                k = 1
                am = -mu
                exp = om * fbeam / (4 * math.pi) * hg(ct) * umu0 / (umu0 - am) * \
                    (math.exp(-tau / umu0) - math.exp(-tau / am))
            worst_c = max(worst_c, abs(r["uu"][j, k, iu] / exp - 1))
            worst_0 = max(worst_0, abs(r0["uu"][j, k, iu] / exp - 1))
    assert worst_c < 1e-4, worst_c
    assert worst_0 > 1e-2, worst_0      # the correction matters here


def test_tms_vanishes_without_truncation():
    rng = np.random.default_rng(9)
    nstr, nlyr = 8, 3
    dtauc, ssalb, pm = _random_column(rng, nlyr, nstr, iso=True)
    pm[:, 2] = 0.1                                   # Rayleigh: f = chi_8 = 0
    kw = dict(umu=[-0.5, 0.4], phi=[0.0, 120.0], utau=[0.0, 0.3 * dtauc.sum()], umu0=0.6,
              fbeam=1.0, albedo=0.3)
    a = disort_rad_column(dtauc, ssalb, pm, nstr, corint=True, **kw)["uu"]
    b = disort_rad_column(dtauc, ssalb, pm, nstr, corint=False, **kw)["uu"]
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("mu1,mu2,tau", [(0.5, 0.5, 0.3), (0.6, 0.5, 1.0), (0.3, 0.9, 2.0),
                                         (0.5, 0.52, 0.7), (0.9, 0.2, 3.0), (0.4, 0.41, 8.0)])
def test_xi_func_is_its_double_integral(mu1, mu2, tau):
    """STWL (A.16): beam (mu2) scattered twice in the forward peak, then to tau (mu1)."""
    def f(tp, t):
        return math.exp(-(tau - t) / mu1 - (t - tp) / mu2 - tp / mu2) / (mu1 * mu2)
    v, _ = scipy.integrate.dblquad(f, 0.0, tau, 0.0, lambda t: t, epsabs=1e-15, epsrel=1e-12)
    assert abs(xi_func(mu1, mu2, tau) / v - 1.0) < 1e-10


@pytest.mark.parametrize("tau", [0.3, 1.0, 3.0])
def test_ims_corrects_the_aureole(tau, monkeypatch):
    """Forward-peaked HG layer (g = 0.85, omega = 0.95, 200 moments), downward
    directions around the beam: nstr 16 with TMS is 1-5 % off the nstr 64
    radiances in the aureole; adding the IMS term brings it within 0.2 %."""
    g, om, nmom = 0.85, 0.95, 200
    pm = np.array([[g ** k for k in range(nmom + 1)]])
    mus = np.array([-0.62, -0.6, -0.58, -0.55, -0.5, -0.4])
    kw = dict(umu=mus, phi=np.array([0.0, 5.0, 20.0]), utau=[0.0, tau], umu0=0.6, phi0=0.0,
              fbeam=1.0)
    ref = disort_rad_column([tau], [om], pm, 64, corint=True, **kw)["uu"][:, 1, :]
    nt = disort_rad_column([tau], [om], pm, 16, corint=True, **kw)["uu"][:, 1, :]
    monkeypatch.setattr(disort_rad_np, "ims_correction", lambda *a, **k: 0.0)
    tms = disort_rad_column([tau], [om], pm, 16, corint=True, **kw)["uu"][:, 1, :]
    e_tms = np.abs(tms / ref - 1).max()
    e_nt = np.abs(nt / ref - 1).max()
    assert e_tms > 1e-2, e_tms
    assert e_nt < 2e-3, e_nt
    assert e_nt < 0.1 * e_tms


def test_ims_only_downward_and_vanishes_without_truncation():
    g, om, nmom, nstr = 0.8, 0.9, 64, 8
    pm = np.array([[g ** k for k in range(nmom + 1)]] * 2)
    kw = dict(umu=[-0.5, 0.5], phi=[0.0, 90.0], utau=[0.0, 0.4, 1.2], umu0=0.5, fbeam=1.0)
    lay = np.array([0, 0, 1])
    ims = disort_rad_np.ims_correction([0.6, 0.6], [om, om], pm, nstr, np.array(kw["umu"]),
                                       np.array(kw["phi"]), lay, kw["utau"], 0.5, 0.0, 1.0)
    assert np.all(ims[:, :, 1] == 0.0)          # upward: no IMS term
    assert np.all(ims[:, 0, :] == 0.0)          # TOA: no slab above
    assert np.all(ims[:, 1:, 0] > 0.0)
    pm0 = pm.copy()
    pm0[:, nstr:] = 0.0                         # chi_l = 0 from nstr on: f = 0
    ims0 = disort_rad_np.ims_correction([0.6, 0.6], [om, om], pm0, nstr, np.array(kw["umu"]),
                                        np.array(kw["phi"]), lay, kw["utau"], 0.5, 0.0, 1.0)
    assert np.all(ims0 == 0.0)
