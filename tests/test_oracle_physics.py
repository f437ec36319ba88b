"""The physics pins of tests/test_gpu_physics.py applied to the CPU oracle
(oracle/disort_oracle.c): isothermal radiative equilibrium (Planck, surface and top
emission, delta-M, multi-layer interfaces) and layer-splitting invariance.  These
pin the restatement by exact properties of the discrete-ordinate equations rather
than by the builder's own reading of cdisort."""

import math

import numpy as np
import pytest

from test_gpu_physics import _planck_band, _random_layers


@pytest.mark.parametrize("nstr", [4, 16, 32])
def test_oracle_isothermal_equilibrium(oracle_c, nstr):
    rng = np.random.default_rng(500 + nstr)
    nwave, ncol, nlyr, T = 2, 4, 12, 230.0
    prop = _random_layers(rng, nwave, ncol, nlyr, nstr)
    wl, wu = np.array([100.0, 900.0]), np.array([500.0, 1100.0])
    bc = {"albedo": rng.uniform(0.0, 1.0, (nwave, ncol)),
          "btemp": np.full((nwave, ncol), T), "ttemp": np.full((nwave, ncol), T),
          "temis": np.ones((nwave, ncol))}
    temf = np.full((ncol, nlyr + 1), T)
    f = oracle_c.forward(prop, bc, temf, nstr=nstr, planck=True, wave_lower=wl, wave_upper=wu)
    for w in range(nwave):
        level = f[w].reshape(-1)
        pib = level.mean()
        assert np.abs(level / pib - 1.0).max() < 1e-9
        assert abs(pib / (math.pi * _planck_band(wl[w], wu[w], T)) - 1.0) < 2e-6


@pytest.mark.parametrize("nstr", [8, 16])
def test_oracle_layer_split_invariance(oracle_c, nstr):
    rng = np.random.default_rng(600 + nstr)
    nwave, ncol, nlyr = 1, 6, 6
    coarse = _random_layers(rng, nwave, ncol, nlyr, nstr, tau_lo=-2.0, tau_hi=1.0)
    fine = np.repeat(coarse, 2, axis=2)
    fine[..., 0] *= 0.5
    bc = {"fbeam": np.ones((nwave, ncol)), "umu0": rng.uniform(0.1, 1.0, (nwave, ncol)),
          "albedo": rng.uniform(0.0, 1.0, (nwave, ncol))}
    fc = oracle_c.forward(coarse, bc, nstr=nstr)
    ff = oracle_c.forward(fine, bc, nstr=nstr)
    scale = np.abs(fc).max(axis=(2, 3), keepdims=True)
    assert (np.abs(ff[:, :, ::2] - fc) / scale).max() < 1e-9


def test_oracle_source_superposition(oracle_c):
    rng = np.random.default_rng(900)
    nwave, ncol, nlyr, nstr = 1, 4, 8, 16
    prop = _random_layers(rng, nwave, ncol, nlyr, nstr)
    wl, wu = np.array([400.0]), np.array([650.0])
    temf = np.linspace(290.0, 180.0, nlyr + 1)[None, :] + rng.uniform(-5, 5, (ncol, nlyr + 1))
    alb = rng.uniform(0.0, 1.0, (nwave, ncol))
    beam = {"fbeam": rng.uniform(1.0, 50.0, (nwave, ncol)),
            "umu0": rng.uniform(0.1, 1.0, (nwave, ncol))}
    therm = {"btemp": np.full((nwave, ncol), 295.0), "ttemp": np.full((nwave, ncol), 170.0),
             "temis": np.full((nwave, ncol), 0.4)}
    kw = dict(nstr=nstr, planck=True, wave_lower=wl, wave_upper=wu)
    both = oracle_c.forward(prop, dict(albedo=alb, **beam, **therm), temf, **kw)
    fb = oracle_c.forward(prop, dict(albedo=alb, **beam, btemp=np.zeros((nwave, ncol))),
                          np.zeros_like(temf), **kw)
    ft = oracle_c.forward(prop, dict(albedo=alb, **therm), temf, **kw)
    scale = np.abs(both).max(axis=(2, 3), keepdims=True)
    assert (np.abs(both - (fb + ft)) / scale).max() < 1e-10
