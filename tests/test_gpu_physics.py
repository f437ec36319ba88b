"""Physics pins of the HIP path that do not go through the builder's oracle.

DESIGN section 4 lists what the CPU restatement pins and what it cannot (cdisort is
absent, and the reference's own solver test has no assertions).  These tests check
the GPU fluxes against exact properties of the discrete-ordinate equations instead,
so a convention shared by the oracle and the kernels cannot hide in them:

* isothermal equilibrium -- an atmosphere at one temperature T over a Lambert surface
  at T, lit from above by isotropic radiance B(T) (temis = 1, ttemp = T), is in
  radiative equilibrium whatever its optical depths, single-scattering albedos,
  phase moments (delta-M included) and surface albedo: I = B(T) in every stream,
  so F_up = F_dn = pi B(T) at every level.  The discrete equations keep this exact
  (the double-Gauss rule integrates P_l, l < nstr, exactly and the source is B(tau)
  = B for isothermal layers), so the check is to rounding.  It covers Planck
  sources, thermal emission of the surface (1 - albedo) B, top emission, multi-layer
  interfaces and anisotropic delta-M layers, at nstr on both kernel paths.  The
  absolute level pi B is checked against the Planck function integrated with scipy
  (DISORT's PLKAVG constants: sigma = 5.67032e-8, c2 = 1.438786 cm K); PLKAVG is a
  series/Simpson evaluation accurate to ~1e-6.
* layer splitting -- the discrete-ordinate solution inside a homogeneous layer is
  exact in tau, so splitting every layer into two halves (same omega, moments)
  leaves the fluxes at the original levels unchanged (beam + Lambert surface).
* the intensity path in isothermal equilibrium -- I = B(T) at every user depth,
  user angle (off the quadrature nodes) and azimuth.
* superposition of sources -- beam + thermal = beam alone + thermal alone.
"""

import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SIGMA_DISORT = 5.67032e-8   # W m^-2 K^-4, the value PLKAVG uses
C2 = 1.438786               # cm K


def _disort(nstr, nlyr, nwave, ncol, planck=False, wl=None, wu=None):
    from pyharp_amd import Disort, DisortOptions
    op = DisortOptions().flags("lamber,quiet,onlyfl" + (",planck" if planck else ""))
    op.nwave(nwave).ncol(ncol)
    if planck:
        op.wave_lower(list(map(float, wl))).wave_upper(list(map(float, wu)))
    op.ds().nlyr = nlyr
    op.ds().nstr = nstr
    op.ds().nmom = nstr
    return Disort(op)


def _run(d, prop, bc, temf=None):
    dev = torch.device("cuda", 0)
    p = torch.as_tensor(prop, dtype=torch.float64, device=dev)
    b = {k: torch.as_tensor(v, dtype=torch.float64, device=dev) for k, v in bc.items()}
    t = None if temf is None else torch.as_tensor(temf, dtype=torch.float64, device=dev)
    return d.forward(p, b, t).cpu().numpy()


def _planck_band(wlo, whi, t):
    """Band-integrated Planck radiance [W m^-2 sr^-1] by quadrature."""
    from scipy.integrate import quad
    v0, v1 = C2 * wlo / t, C2 * whi / t
    val, _ = quad(lambda x: x ** 3 / math.expm1(x), v0, v1, epsabs=0.0, epsrel=1e-12, limit=200)
    return SIGMA_DISORT / math.pi * t ** 4 * 15.0 / math.pi ** 4 * val


def _random_layers(rng, nwave, ncol, nlyr, nstr, tau_lo=-3.0, tau_hi=1.0):
    prop = np.zeros((nwave, ncol, nlyr, 2 + nstr))
    prop[..., 0] = 10.0 ** rng.uniform(tau_lo, tau_hi, (nwave, ncol, nlyr))
    prop[..., 1] = rng.uniform(0.0, 1.0, (nwave, ncol, nlyr))
    prop[:, 0, ::3, 1] = 1.0     # conservative layers (DISORT's dither)
    prop[:, 1, :, 1] = 0.0       # a purely absorbing column
    g = rng.uniform(0.0, 0.9, (nwave, ncol, nlyr))
    for l in range(nstr):
        prop[..., 2 + l] = g ** (l + 1)
    return prop


@pytest.mark.parametrize("nstr", [4, 8, 16, 24, 32])
def test_isothermal_equilibrium(nstr):
    rng = np.random.default_rng(300 + nstr)
    nwave, ncol, nlyr, T = 3, 16, 30, 260.0
    prop = _random_layers(rng, nwave, ncol, nlyr, nstr)
    wl = np.array([20.0, 600.0, 1800.0])
    wu = np.array([350.0, 640.0, 2600.0])
    bc = {"albedo": rng.uniform(0.0, 1.0, (nwave, ncol)),
          "btemp": np.full((nwave, ncol), T), "ttemp": np.full((nwave, ncol), T),
          "temis": np.ones((nwave, ncol))}
    bc["albedo"][:, 2] = 0.0
    bc["albedo"][:, 3] = 1.0
    temf = np.full((ncol, nlyr + 1), T)
    d = _disort(nstr, nlyr, nwave, ncol, planck=True, wl=wl, wu=wu)
    f = _run(d, prop, bc, temf)
    for w in range(nwave):
        level = f[w].reshape(-1)
        pib = level.mean()
        # every stream carries B(T): all fluxes of the band equal to rounding
        assert np.abs(level / pib - 1.0).max() < 1e-9, (w, np.abs(level / pib - 1.0).max())
        ref = math.pi * _planck_band(wl[w], wu[w], T)
        assert abs(pib / ref - 1.0) < 2e-6, (w, pib, ref)


@pytest.mark.parametrize("nstr", [8, 16, 24])
def test_layer_split_invariance(nstr):
    rng = np.random.default_rng(400 + nstr)
    nwave, ncol, nlyr = 2, 16, 10
    coarse = _random_layers(rng, nwave, ncol, nlyr, nstr, tau_lo=-2.0, tau_hi=1.0)
    fine = np.repeat(coarse, 2, axis=2)
    fine[..., 0] *= 0.5
    bc = {"fbeam": np.ones((nwave, ncol)), "umu0": rng.uniform(0.1, 1.0, (nwave, ncol)),
          "albedo": rng.uniform(0.0, 1.0, (nwave, ncol))}
    fc = _run(_disort(nstr, nlyr, nwave, ncol), coarse, bc)
    ff = _run(_disort(nstr, 2 * nlyr, nwave, ncol), fine, bc)
    assert fc.shape[2] == nlyr + 1 and ff.shape[2] == 2 * nlyr + 1
    scale = np.abs(fc).max(axis=(2, 3), keepdims=True)
    err = np.abs(ff[:, :, ::2] - fc) / scale
    assert err.max() < 1e-9, err.max()


@pytest.mark.parametrize("nstr", [4, 16, 24])
def test_isothermal_equilibrium_radiances(nstr):
    """Intensity path (every azimuthal mode, user depths and user angles off the
    quadrature nodes): in isothermal equilibrium I = B(T) at every depth, angle and
    azimuth -- the user-angle source integrates the phase function over the nodes
    exactly, so the radiances, not only the fluxes, are B to rounding."""
    from pyharp_amd import Disort, DisortOptions
    rng = np.random.default_rng(700 + nstr)
    nwave, ncol, nlyr, T = 2, 4, 8, 245.0
    prop = _random_layers(rng, nwave, ncol, nlyr, nstr)
    wl, wu = np.array([300.0, 1200.0]), np.array([700.0, 1400.0])
    total = prop[..., 0].sum(axis=-1).min()
    utau = [0.0, 0.3 * total, total]
    umu, phi = [-1.0, -0.6, -0.15, 0.1, 0.45, 0.8], [0.0, 75.0, 180.0]
    op = DisortOptions().flags("usrtau,usrang,lamber,quiet,planck").nwave(nwave).ncol(ncol)
    op.wave_lower(list(wl)).wave_upper(list(wu)).user_mu(umu).user_phi(phi).user_tau(utau)
    op.ds().nlyr = nlyr
    op.ds().nstr = nstr
    op.ds().nmom = nstr
    d = Disort(op)
    bc = {"albedo": rng.uniform(0.0, 1.0, (nwave, ncol)),
          "btemp": np.full((nwave, ncol), T), "ttemp": np.full((nwave, ncol), T),
          "temis": np.ones((nwave, ncol))}
    f = _run(d, prop, bc, np.full((ncol, nlyr + 1), T))
    uu = d.get_rad().cpu().numpy()
    for w in range(nwave):
        b = _planck_band(wl[w], wu[w], T)
        assert np.abs(uu[w] / uu[w].mean() - 1.0).max() < 1e-9
        assert abs(uu[w].mean() / b - 1.0) < 2e-6
        assert np.abs(f[w] / (math.pi * uu[w].mean()) - 1.0).max() < 1e-9


@pytest.mark.parametrize("nstr", [8, 16, 32])
def test_source_superposition(nstr):
    """The equations are linear in their sources: fluxes with beam + thermal
    emission (layers, surface, top) = beam alone + thermal alone."""
    rng = np.random.default_rng(800 + nstr)
    nwave, ncol, nlyr = 2, 16, 20
    prop = _random_layers(rng, nwave, ncol, nlyr, nstr)
    wl, wu = np.array([400.0, 900.0]), np.array([650.0, 1300.0])
    temf = np.linspace(290.0, 180.0, nlyr + 1)[None, :] + rng.uniform(-5, 5, (ncol, nlyr + 1))
    alb = rng.uniform(0.0, 1.0, (nwave, ncol))
    beam = {"fbeam": rng.uniform(1.0, 50.0, (nwave, ncol)),
            "umu0": rng.uniform(0.1, 1.0, (nwave, ncol))}
    therm = {"btemp": np.full((nwave, ncol), 295.0), "ttemp": np.full((nwave, ncol), 170.0),
             "temis": np.full((nwave, ncol), 0.4)}
    d = _disort(nstr, nlyr, nwave, ncol, planck=True, wl=wl, wu=wu)
    both = _run(d, prop, dict(albedo=alb, **beam, **therm), temf)
    fb = _run(d, prop, dict(albedo=alb, **beam, btemp=np.zeros((nwave, ncol))),
              np.zeros_like(temf))
    ft = _run(d, prop, dict(albedo=alb, **therm), temf)
    scale = np.abs(both).max(axis=(2, 3), keepdims=True)
    err = np.abs(both - (fb + ft)) / scale
    assert err.max() < 1e-10, err.max()
