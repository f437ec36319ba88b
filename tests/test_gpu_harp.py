"""HIP parity of the harp-side steps (include/hdharp.h) and the amars_sw case
end to end, against oracle/harp_np.py + the C DISORT oracle.

Tolerances: the optics and epilogue kernels do the reference's arithmetic in
the reference's order, so they are held to 1e-13 relative (interpolation /
sums in f64); fluxes to the north-star bound 1e-6 (tests/helpers.py); heating
rates, being differences of fluxes, to 1e-6 of the column's largest |dT/dt|.
"""

import os
import sys

import numpy as np
import pytest
import torch

from helpers import TOL, rel_err, margin
from oracle import harp_np as H

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(HERE, "golden", "data")
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module", autouse=True)
def _resources():
    from pyharp_amd.opacity import add_resource_directory
    add_resource_directory(DATA)


def _attenuators():
    from pyharp_amd.opacity import AttenuatorOptions, H2SO4Simple, S8Fuller
    op = AttenuatorOptions().species_names(["S8", "H2SO4"]).species_weights([256.e-3, 98.e-3])
    s8 = S8Fuller(op.copy().species_ids([0]).opacity_files(["s8_k_fuller.txt"]))
    h2 = H2SO4Simple(op.copy().species_ids([1]).opacity_files(["h2so4.txt"]))
    return s8, h2


def _oracle_tables():
    s8 = H.load_attenuator(os.path.join(DATA, "s8_k_fuller.txt"), 256e-3)
    h2 = H.load_attenuator(os.path.join(DATA, "h2so4.txt"), 98e-3)
    return [(s8[0], s8[1], 0), (h2[0], h2[1], 1)]


def test_attenuator_forward_matches_oracle():
    s8, h2 = _attenuators()
    tabs = _oracle_tables()
    rng = np.random.default_rng(5)
    conc = rng.uniform(0, 1e-5, (3, 7, 2))
    # wavenumbers inside, at and beyond both table ends
    wave = np.r_[np.linspace(2000.0, 50000.0, 97), 1e4 / tabs[0][0][0], 1e4 / tabs[1][0][-1],
                 100.0, 1e6]
    for att, (kw, kd, sp) in zip((s8, h2), tabs):
        got = att.forward(torch.as_tensor(conc, device=DEV),
                          {"wavenumber": torch.as_tensor(wave, device=DEV)}).cpu().numpy()
        ref = H.attenuate(kw, kd, sp, conc, wavenumber=wave)
        np.testing.assert_allclose(got, ref, rtol=1e-13, atol=0)
    # wavelength coordinate
    wl = np.linspace(0.1, 6.0, 33)
    got = s8.forward(torch.as_tensor(conc, device=DEV),
                     {"wavelength": torch.as_tensor(wl, device=DEV)}).cpu().numpy()
    ref = H.attenuate(tabs[0][0], tabs[0][1], 0, conc, wavelength=wl)
    np.testing.assert_allclose(got, ref, rtol=1e-13, atol=0)


@pytest.mark.parametrize("nprop", [2, 10])
def test_band_optics_matches_oracle(nprop):
    from pyharp_amd.opacity import band_optics
    conc, rho, dz, p = H.amars_sw_atmosphere(os.path.join(DATA, "aerosol_output_data.txt"))
    conc = np.repeat(conc, 3, axis=0) * np.array([1.0, 0.5, 0.0])[:, None, None]  # 3 columns
    wave = H.short_wavenumber_grid(500)
    got = band_optics(list(_attenuators()), torch.as_tensor(conc, device=DEV),
                      torch.as_tensor(dz, device=DEV),
                      {"wavenumber": torch.as_tensor(wave, device=DEV)}, nprop=nprop)
    ref = H.band_optics(_oracle_tables(), conc, dz, nprop=nprop, wavenumber=wave)
    np.testing.assert_allclose(got.cpu().numpy(), ref, rtol=1e-13, atol=0)
    assert np.all(got[:, 2].cpu().numpy() == 0.0)  # empty column: tau 0, ssa 0 (not NaN)


def test_band_flux_many_bins_few_outputs():
    """one column line-by-line (C3-like): the wave-per-output reduction"""
    from pyharp_amd.spectral import band_flux
    rng = np.random.default_rng(61)
    flux = rng.uniform(0, 1, (19990, 1, 11, 2))
    w = rng.uniform(0, 0.1, 19990)
    b = band_flux(torch.as_tensor(flux, device=DEV), torch.as_tensor(w, device=DEV))
    np.testing.assert_allclose(b.cpu().numpy(), H.band_flux(flux, w), rtol=1e-12)


def test_band_flux_heating_spherical_match_oracle():
    from pyharp_amd.spectral import band_flux, heating_rate, spherical_flux_correction
    rng = np.random.default_rng(6)
    G, C, L = 37, 5, 24
    flux = rng.uniform(0, 100, (G, C, L + 1, 2))
    w = rng.uniform(0, 1, G)
    b = band_flux(torch.as_tensor(flux, device=DEV), torch.as_tensor(w, device=DEV))
    bref = H.band_flux(flux, w)
    np.testing.assert_allclose(b.cpu().numpy(), bref, rtol=1e-13)
    dz = rng.uniform(100, 2000, (C, L))
    rho = rng.uniform(0.01, 1.5, (C, L))
    h = heating_rate(b, torch.as_tensor(dz, device=DEV), torch.as_tensor(rho, device=DEV), 844.0)
    np.testing.assert_allclose(h.cpu().numpy(), H.heating_rate(bref, dz, rho, 844.0),
                               rtol=1e-9, atol=1e-12 * np.abs(H.heating_rate(bref, dz, rho,
                                                                             844.0)).max())
    x1f = 6.4e6 + np.cumsum(np.r_[0.0, rng.uniform(1e3, 2e3, L)])
    area = 4 * np.pi * x1f ** 2
    vol = 4 / 3 * np.pi * np.diff(x1f ** 3)
    sref = H.spherical_flux_correction(b.cpu().numpy(), x1f, area, vol)
    spherical_flux_correction(b, torch.as_tensor(x1f, device=DEV),
                              torch.as_tensor(area, device=DEV), torch.as_tensor(vol, device=DEV))
    np.testing.assert_allclose(b.cpu().numpy(), sref, rtol=1e-12)


@pytest.mark.parametrize("nstr", [8, 16])
def test_amars_sw_end_to_end(oracle_c, nstr):
    """examples/amars_sw.py (all on the GPU) vs the oracle pipeline on the same
    atmosphere: prop, per-bin fluxes, band flux and heating rates."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "examples"))
    import amars_sw
    r = amars_sw.run(nstr=nstr, nwave=500, nlyr=40)
    conc, rho, dz, p = H.amars_sw_atmosphere(os.path.join(DATA, "aerosol_output_data.txt"))
    np.testing.assert_allclose(r["conc"], conc, rtol=1e-12)
    np.testing.assert_allclose(r["dz"], dz, rtol=1e-12)
    wave = H.short_wavenumber_grid(500)
    prop = H.band_optics(_oracle_tables(), conc, dz, wavenumber=wave)
    np.testing.assert_allclose(r["prop"].cpu().numpy(), prop, rtol=1e-11)
    bc = {"fbeam": H.bb_toa_flux(wave, 1, 5772.0, 0.7), "umu0": np.ones((500, 1)),
          "albedo": np.ones((500, 1))}
    fref = oracle_c.forward(r["prop"].cpu().numpy(), bc, nstr=nstr, nmom=nstr)
    f = r["flux"].cpu().numpy()
    assert margin(rel_err(f, fref).max()) < TOL
    bref = H.band_flux(fref, np.full(500, wave[1] - wave[0]))
    assert margin(rel_err(r["bflux"].cpu().numpy()[None], bref[None]).max()) < TOL
    href = H.heating_rate(bref, dz, rho, 844.0)
    h = r["dTdt"].cpu().numpy()
    assert np.abs(h - href).max() <= 1e-6 * np.abs(href).max()
    # the example's own statement (amars_sw.cpp:75-77): TOA down within 2 W/m^2 of 410
    assert abs(r["bflux"][0, -1, 1].item() - 410.0) < 2.0


def test_amars_lw_example(oracle_c):
    """examples/amars_lw.py: isothermal 300 K layers over an albedo-1 surface
    (emissivity 0); per-g fluxes vs the oracle, no diffuse flux entering at the
    top, and F_up = F_dn at the perfectly reflecting surface."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "examples"))
    import amars_lw
    r = amars_lw.run(nstr=8, ngpoint=16, nlyr=40)
    prop = r["prop"].cpu().numpy()
    temf = r["temf"].cpu().numpy()
    bc = {"albedo": np.ones((16, 1)), "btemp": np.full((16, 1), 300.0)}
    ref = oracle_c.forward(prop, bc, temf, nstr=8, planck=True, wave_lower=np.full(16, 1.0),
                           wave_upper=np.full(16, 150.0))
    f = r["flux"].cpu().numpy()
    assert margin(rel_err(f, ref).max()) < TOL
    assert np.all(np.abs(f[:, 0, -1, 1]) <= 1e-12 * np.abs(f).max())
    np.testing.assert_allclose(f[:, 0, 0, 0], f[:, 0, 0, 1], rtol=1e-12)
    assert r["bflux"].shape == (1, 41, 2)


@pytest.mark.parametrize("nstr", [8, 16])
def test_cpp_amars_sw(oracle_c, nstr):
    """tests/cpp/amars_sw_dropin.cpp: the reference's amars_sw main() with the
    harp_amd C++ modules (include/harp_amd/{opacity,spectral,disort}.hpp) --
    band flux and heating rates vs the oracle pipeline."""
    import subprocess
    root = os.path.dirname(HERE)
    exe = os.path.join(root, "tests", "cpp", "amars_sw_dropin")
    if not os.path.exists(exe):
        subprocess.run([os.path.join(root, "tests", "cpp", "build.sh")], check=True)
    out = subprocess.run([exe, DATA, str(nstr)], check=True, capture_output=True,
                         text=True).stdout.split("\n")
    lev = np.array([[float(x) for x in l.split()[2:]] for l in out if l.startswith("level")])
    lay = np.array([float(l.split()[2]) for l in out if l.startswith("layer")])
    conc, rho, dz, p = H.amars_sw_atmosphere(os.path.join(DATA, "aerosol_output_data.txt"))
    wave = H.short_wavenumber_grid(500)
    prop = H.band_optics(_oracle_tables(), conc, dz, wavenumber=wave)
    bc = {"fbeam": H.bb_toa_flux(wave, 1, 5772.0, 0.7), "umu0": np.ones((500, 1)),
          "albedo": np.ones((500, 1))}
    fref = oracle_c.forward(prop, bc, nstr=nstr, nmom=nstr)
    bref = H.band_flux(fref, np.full(500, wave[1] - wave[0]))
    assert margin(rel_err(lev[None], bref).max()) < TOL
    href = H.heating_rate(bref, dz, rho, 844.0)[0]
    assert np.abs(lay - href).max() <= 1e-6 * np.abs(href).max()


def test_rfm_forward_matches_oracle():
    """RFM (hd_rfm_attenuate) vs the interpn restatement: pressures and
    temperatures inside, at and beyond the table nodes (clamped)."""
    from pyharp_amd.opacity import RFM
    rng = np.random.default_rng(21)
    nw, npr, nt = 9, 7, 4
    wave = np.linspace(10.0, 90.0, nw)
    pres = np.logspace(6.5, 3, npr)
    tgrid = np.linspace(-30.0, 30.0, nt)
    tref = np.linspace(300.0, 180.0, npr)
    kdata = rng.uniform(-6, 3, (nw, npr, nt))
    m = RFM.from_arrays(wave, pres, tgrid, tref, kdata, species=1)
    ncol, nlyr = 3, 11
    p = np.exp(rng.uniform(np.log(5e2), np.log(8e6), (ncol, nlyr)))
    p[0, :3] = pres[:3]                        # exactly at pressure nodes
    t = rng.uniform(120.0, 360.0, (ncol, nlyr))
    conc = rng.uniform(0.1, 2.0, (ncol, nlyr, 2))
    got = m.forward(torch.as_tensor(conc, device=DEV),
                    {"pres": torch.as_tensor(p, device=DEV),
                     "temp": torch.as_tensor(t, device=DEV)}).cpu().numpy()
    ref = H.rfm_forward(wave, np.log(pres), tgrid, tref, kdata, conc, p, t, 1)
    assert got.shape == (nw, ncol, nlyr, 1)
    np.testing.assert_allclose(got, ref, rtol=1e-13, atol=0)


def test_amars_lw_with_rfm_tables(oracle_c, tmp_path):
    """examples/amars_lw.py --table: amars_lw.cpp:40-88 on a synthetic classic-netCDF
    RFM file -- RFM optics, Planck solve, ck-weighted band flux -- vs the oracles."""
    from rfm_fixture import write_rfm_table
    from pyharp_amd.opacity import add_resource_directory
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "examples"))
    import amars_lw
    fx = write_rfm_table(str(tmp_path / "amarsw-ck-B1.nc"))
    add_resource_directory(str(tmp_path))
    r = amars_lw.run_rfm("amarsw-ck-B1.nc", nstr=8, nlyr=40)
    nw = len(fx["wave"])
    conc = np.ones((1, 40, 2))
    p = np.full((1, 40), 10.e5)
    t = np.full((1, 40), 300.0)
    lnp = np.log(fx["pres"])
    prop = sum(H.rfm_forward(fx["wave"], lnp, fx["tgrid"], fx["tref"], fx["tables"][sp], conc,
                             p, t, i) for i, sp in enumerate(("CO2", "H2O")))
    np.testing.assert_allclose(r["prop"].cpu().numpy(), prop, rtol=1e-13)
    temf = r["temf"].cpu().numpy()
    bc = {"albedo": np.ones((nw, 1)), "btemp": np.full((nw, 1), 300.0)}
    fref = oracle_c.forward(prop, bc, temf, nstr=8, planck=True, wave_lower=np.full(nw, 1.0),
                            wave_upper=np.full(nw, 150.0))
    assert margin(rel_err(r["flux"].cpu().numpy(), fref).max()) < TOL
    np.testing.assert_array_equal(r["weights"].cpu().numpy(), fx["weights"])
    bref = H.band_flux(fref, fx["weights"])
    assert margin(rel_err(r["bflux"].cpu().numpy()[None], bref[None]).max()) < TOL


def test_cpp_amars_lw(oracle_c, tmp_path):
    """tests/cpp/amars_lw_dropin.cpp: amars_lw.cpp's main() against harp_amd::RFM,
    harp_amd::Disort and harp_amd::read_weights_rfm on a synthetic ck table."""
    import subprocess
    from rfm_fixture import write_rfm_table
    root = os.path.dirname(HERE)
    exe = os.path.join(root, "tests", "cpp", "amars_lw_dropin")
    if not os.path.exists(exe):
        subprocess.run([os.path.join(root, "tests", "cpp", "build.sh")], check=True)
    fx = write_rfm_table(str(tmp_path / "amarsw-ck-B1.nc"))
    out = subprocess.run([exe, str(tmp_path)], check=True, capture_output=True,
                         text=True).stdout.split("\n")
    prop_c = np.array([float(l.split()[2]) for l in out if l.startswith("prop")])
    bflx = np.array([[float(x) for x in l.split()[2:]] for l in out if l.startswith("bflx")])
    nw = len(fx["wave"])
    conc = np.ones((1, 40, 2))
    lnp = np.log(fx["pres"])
    prop = sum(H.rfm_forward(fx["wave"], lnp, fx["tgrid"], fx["tref"], fx["tables"][sp], conc,
                             np.full((1, 40), 10.e5), np.full((1, 40), 300.0), i)
               for i, sp in enumerate(("CO2", "H2O")))
    np.testing.assert_allclose(prop_c, prop[:, 0, 0, 0], rtol=1e-13)
    bc = {"albedo": np.ones((nw, 1)), "btemp": np.full((nw, 1), 300.0)}
    fref = oracle_c.forward(prop, bc, np.full((1, 41), 300.0), nstr=8, planck=True,
                            wave_lower=np.full(nw, 1.0), wave_upper=np.full(nw, 150.0))
    bref = H.band_flux(fref, fx["weights"])
    assert margin(rel_err(bflx[None], bref).max()) < TOL


@pytest.mark.parametrize("nmom", [0, 8, 32])
@pytest.mark.parametrize("rfm", [False, True])
def test_band_loop_optics_bit_identical(nmom, rfm):
    """hd_band_loop_optics (radiation_band.cpp:86-116 on the device) equals the numpy
    restatement bit for bit on the reference's data tables (which
    tests/test_harp_oracle.py pins to the reference's statement order): s8 with a
    wavelength-dependent HG asymmetry, h2so4 with a constant one; wavenumbers inside,
    at and beyond the table ends; an RFM-like extinction added first."""
    from pyharp_amd.opacity import band_loop_optics
    s8, h2 = _attenuators()
    tabs = _oracle_tables()
    g8 = np.linspace(0.6, 0.85, s8.kwave.numel())
    s8.set_asymmetry(g8)
    h2.set_asymmetry(0.75)
    otabs = [(tabs[0][0], tabs[0][1], 0, g8), (tabs[1][0], tabs[1][1], 1, H.hg_table(tabs[1][0], 0.75))]
    rng = np.random.default_rng(31 + nmom)
    ncol, nlyr = 4, 9
    conc = rng.uniform(0, 1e-5, (ncol, nlyr, 2))
    conc[1, 2] = 0.0
    dz = rng.uniform(100, 2000, (ncol, nlyr))
    wave = np.r_[np.linspace(2000.0, 50000.0, 37), 1e4 / tabs[0][0][0], 100.0, 1e6]
    ext0 = rng.uniform(0, 1e-3, (wave.size, ncol, nlyr)) if rfm else None
    got = band_loop_optics([s8, h2], torch.as_tensor(conc, device=DEV), torch.as_tensor(dz),
                           {"wavenumber": torch.as_tensor(wave, device=DEV)}, nmom,
                           ext0=None if ext0 is None else torch.as_tensor(ext0, device=DEV))
    ref = H.band_loop_optics(otabs, conc, dz, nmom, wavenumber=wave, ext0=ext0)
    np.testing.assert_array_equal(got.cpu().numpy(), ref)


def test_optics_refuse_bad_out():
    """A caller-supplied ``out`` is written through its pointer by the kernel: a wrong
    shape, dtype, device or layout is refused before the launch (band_optics and
    band_loop_optics); a correct one is filled in place."""
    from pyharp_amd.opacity import band_loop_optics, band_optics
    s8, h2 = _attenuators()
    s8.set_asymmetry(0.7)
    h2.set_asymmetry(0.75)
    ncol, nlyr, nmom = 2, 5, 4
    conc = torch.full((ncol, nlyr, 2), 1e-6, dtype=torch.float64, device=DEV)
    dz = torch.full((ncol, nlyr), 500.0, dtype=torch.float64)
    kw = {"wavenumber": torch.linspace(2000.0, 40000.0, 3, dtype=torch.float64, device=DEV)}
    f64 = torch.float64
    bad = [torch.empty((3, ncol, nlyr, 2 + nmom + 1), dtype=f64, device=DEV),
           torch.empty((3, ncol, nlyr, 2 + nmom), dtype=torch.float32, device=DEV),
           torch.empty((3, ncol, nlyr, 2 + nmom), dtype=f64),
           torch.empty((3, ncol, 2 + nmom, nlyr), dtype=f64, device=DEV).transpose(2, 3)]
    for out in bad:
        with pytest.raises(RuntimeError, match="out must be"):
            band_loop_optics([s8, h2], conc, dz, kw, nmom, out=out)
        o2 = out[..., :2] if out.dim() == 4 and out.shape[-1] >= 2 else out
        with pytest.raises(RuntimeError, match="out must be"):
            band_optics([s8, h2], conc, dz, kw, 2, out=o2 if o2.shape[-1] == 2 else out)
    good = torch.full((3, ncol, nlyr, 2 + nmom), float("nan"), dtype=f64, device=DEV)
    ret = band_loop_optics([s8, h2], conc, dz, kw, nmom, out=good)
    assert ret is good and bool(torch.isfinite(good).all())
    np.testing.assert_array_equal(good.cpu().numpy(),
                                  band_loop_optics([s8, h2], conc, dz, kw, nmom).cpu().numpy())
