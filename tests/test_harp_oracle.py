"""CPU checks of the harp-side oracle (oracle/harp_np.py) and host helpers.

The reference's own tests for these steps print without asserting
(tests/test_attenuator.cpp), so the restatement is pinned here by closed-form
properties and by the amars_sw example's stated TOA flux (amars_sw.cpp:75-77).
"""

import os

import numpy as np
import pytest

from oracle import harp_np as H

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data")


def test_locate_matches_numerical_recipes_contract():
    xx = np.array([1.0, 2.0, 4.0, 8.0])
    assert H.locate(xx, 0.5) == -1
    assert H.locate(xx, 1.0) == 0
    assert H.locate(xx, 3.0) == 1
    assert H.locate(xx, 8.0) == 3
    assert H.locate(xx, 9.0) == 3
    dd = xx[::-1].copy()  # descending axis (the aerosol profile's pressure)
    assert H.locate(dd, 3.0) == 1
    assert H.locate(dd, 9.0) == -1


def test_interp_nodes_linear_and_clamped():
    ax = np.array([0.2, 0.5, 1.0, 3.0])
    data = np.array([[1.0, 0.1], [2.0, 0.3], [5.0, 0.2], [1.0, 0.9]])
    for i, x in enumerate(ax):
        np.testing.assert_array_equal(H.interp1(x, ax, data), data[i])
    np.testing.assert_allclose(H.interp1(0.75, ax, data), 0.5 * (data[1] + data[2]), rtol=1e-15)
    np.testing.assert_array_equal(H.interp1(0.01, ax, data), data[0])
    np.testing.assert_array_equal(H.interp1(7.0, ax, data), data[-1])


def test_tables_and_units():
    kw, kd = H.load_attenuator(os.path.join(DATA, "s8_k_fuller.txt"), 256e-3)
    raw = H.read_table(os.path.join(DATA, "s8_k_fuller.txt"))
    assert raw.shape[1] == 3 and len(kw) == raw.shape[0] > 100
    np.testing.assert_array_equal(kd[:, 0], raw[:, 1] * 256e-3)
    assert np.all(np.diff(kw) > 0)


def test_amars_sw_toa_flux_statement():
    """'nu_max = 50000 cm^-1 gets us within 2 W/m^2 of the correct 410 value'
    (amars_sw.cpp:75-77): sum_w F0(nu_w) mu0 dnu with umu0 = 1, 500 bins."""
    wave = H.short_wavenumber_grid(500)
    f = H.bb_toa_flux(wave, 1, 5772.0, 0.7)[:, 0]
    toa = float((f * (wave[1] - wave[0])).sum())
    assert abs(toa - 410.0) < 2.0


def test_band_optics_sums_and_ssa():
    conc, rho, dz, p = H.amars_sw_atmosphere(os.path.join(DATA, "aerosol_output_data.txt"))
    assert conc.shape == (1, 40, 2) and np.all(dz > 0) and np.all(np.diff(p) < 0)
    s8 = H.load_attenuator(os.path.join(DATA, "s8_k_fuller.txt"), 256e-3)
    h2 = H.load_attenuator(os.path.join(DATA, "h2so4.txt"), 98e-3)
    wave = H.short_wavenumber_grid(50)
    a = H.attenuate(*s8, 0, conc, wavenumber=wave)
    b = H.attenuate(*h2, 1, conc, wavenumber=wave)
    prop = H.band_optics([(s8[0], s8[1], 0), (h2[0], h2[1], 1)], conc, dz, wavenumber=wave)
    np.testing.assert_allclose(prop[..., 0], (a[..., 0] + b[..., 0]) * dz, rtol=1e-14)
    ssa = (a[..., 1] + b[..., 1]) / (a[..., 0] + b[..., 0])
    np.testing.assert_allclose(prop[..., 1], ssa, rtol=1e-14)
    assert np.all((prop[..., 1] > 0) & (prop[..., 1] < 1))


def test_band_flux_and_heating_closed_forms():
    rng = np.random.default_rng(1)
    flux = rng.uniform(0, 10, (7, 3, 6, 2))
    w = np.full(7, 0.25)
    np.testing.assert_allclose(H.band_flux(flux, w), 0.25 * flux.sum(0), rtol=1e-14)
    # linear net flux F_up - F_dn = a + b z -> dT/dt = -b / (rho cp)
    z = np.cumsum(np.r_[0.0, rng.uniform(1, 3, 5)])
    bflux = np.zeros((1, 6, 2))
    bflux[0, :, 0] = 3.0 + 0.5 * z
    bflux[0, :, 1] = 1.0
    dz = np.diff(z)
    h = H.heating_rate(bflux, dz, np.full(5, 1.2), 844.0)
    np.testing.assert_allclose(h, -0.5 / (1.2 * 844.0), rtol=1e-12)


def test_spherical_correction_identity_in_plane_parallel():
    rng = np.random.default_rng(2)
    x1f = np.cumsum(np.r_[0.0, rng.uniform(1, 2, 8)])
    area = np.full(9, 3.0)
    vol = area[:-1] * np.diff(x1f)
    f = rng.uniform(0, 1, (2, 9, 2))
    np.testing.assert_allclose(H.spherical_flux_correction(f, x1f, area, vol), f, rtol=1e-13)


def _band_loop_tables(with_g=(True, True)):
    s8 = H.load_attenuator(os.path.join(DATA, "s8_k_fuller.txt"), 256e-3)
    h2 = H.load_attenuator(os.path.join(DATA, "h2so4.txt"), 98e-3)
    g8 = H.hg_table(s8[0], np.linspace(0.6, 0.85, len(s8[0]))) if with_g[0] else None
    g2 = H.hg_table(h2[0], 0.75) if with_g[1] else None
    return [(s8[0], s8[1], 0, g8), (h2[0], h2[1], 1, g2)]


def _reference_text_order(tables, conc, dz, nmom, wave, ext0=None):
    """radiation_band.cpp:83-116 transcribed statement by statement onto numpy
    arrays: prop (nprop, W, C, L) -- the wave axis the reference's prop lacks added --
    and each attenuator's kdata (nprop_a, W, C, L) = [k c, ssa, g^1..g^nmom]."""
    ncol, nlyr, _ = conc.shape
    W = len(wave)
    prop = np.zeros((2 + nmom, W, ncol, nlyr))
    kds = []
    if ext0 is not None:
        kds.append(ext0[None])  # an nprop = 1 attenuator (RFM)
    for kwave, kd, sp, g in tables:
        na = 2 + nmom if g is not None else 2
        kdata = np.zeros((na, W, ncol, nlyr))
        for w, x in enumerate(1.0e4 / wave):
            k, s, gw = H.interp1(x, kwave, np.stack([kd[:, 0], kd[:, 1],
                                                    g if g is not None else 0 * kd[:, 0]], 1))
            kdata[0, w] = k * conc[:, :, sp]
            kdata[1, w] = s
            chi = gw
            for l in range(na - 2):
                if l:
                    chi = chi * gw
                kdata[2 + l, w] = chi
        kds.append(kdata)
    for kdata in kds:                                   # :86-104
        nprop = kdata.shape[0]
        prop[0] += kdata[0]
        if nprop > 1:
            prop[1] += kdata[1] * kdata[0]
        if nprop > 2:
            prop[2:nprop] += kdata[2:nprop] * kdata[1] * kdata[0]
    nprop = prop.shape[0]                               # :107-116
    if nprop > 2:
        prop[2:] /= (prop[1] + 1e-10)
    if nprop > 1:
        prop[1] /= (prop[0] + 1e-10)
    prop[0] *= dz[None]
    return np.moveaxis(prop, 0, -1)


@pytest.mark.parametrize("nmom", [0, 4, 32])
@pytest.mark.parametrize("with_g", [(True, True), (True, False)])
@pytest.mark.parametrize("rfm", [False, True])
def test_band_loop_restatement_is_the_reference_order(nmom, with_g, rfm):
    """harp_np.band_loop_optics equals a statement-by-statement transcription of
    radiation_band.cpp:86-116 bit for bit (the GPU kernel is then held to it exactly)."""
    rng = np.random.default_rng(11 + nmom)
    ncol, nlyr = 3, 5
    conc = rng.uniform(0, 1e-5, (ncol, nlyr, 2))
    conc[0, 0] = 0.0  # a layer without extinction: ssa 0/(0+1e-10) = 0
    dz = rng.uniform(100, 2000, (ncol, nlyr))
    wave = np.linspace(2000.0, 50000.0, 7)
    ext0 = rng.uniform(0, 1e-3, (7, ncol, nlyr)) if rfm else None
    tabs = _band_loop_tables(with_g)
    got = H.band_loop_optics(tabs, conc, dz, nmom, wavenumber=wave, ext0=ext0)
    ref = _reference_text_order(tabs, conc, dz, nmom, wave, ext0)
    np.testing.assert_array_equal(got, ref)
    if not rfm:
        assert np.all(got[:, 0, 0, 1:] == 0.0)


def test_band_loop_single_attenuator_moments_are_hg():
    """One attenuator: ssa = s kc / (kc + 1e-10) -> s, chi_l -> g^l (the regularisation
    shifts them by ~1e-10 / (k c))."""
    kw, kd, sp, _ = _band_loop_tables()[1]
    g = 0.7
    conc = np.full((1, 1, 2), 1e-2)
    p = H.band_loop_optics([(kw, kd, 1, H.hg_table(kw, g))], conc, np.ones((1, 1)), 6,
                           wavelength=np.array([kw[3]]))
    np.testing.assert_allclose(p[0, 0, 0, 1], kd[3, 1], rtol=1e-7)
    np.testing.assert_allclose(p[0, 0, 0, 2:], g ** np.arange(1, 7), rtol=1e-7)
    np.testing.assert_allclose(p[0, 0, 0, 0], kd[3, 0] * 1e-2, rtol=1e-15)
