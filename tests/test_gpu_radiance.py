"""HIP intensity path (hd_solve_radiance through pyharp_amd.Disort) vs the
radiance oracle (oracle/disort_rad_np.py) and DISOTEST-1's published radiances.

Tolerance: the north-star bound 1e-6, relative to the largest radiance of the
column (radiances of high azimuthal modes and of the dark hemisphere are small
differences of large terms; the oracle itself is exact to ~1e-10 there).
"""

import math

import numpy as np
import pytest
import torch

from helpers import TOL, disotest, rel_err, margin
from oracle.disort_rad_np import disort_rad_forward

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _disort(nstr, nlyr, nwave, ncol, *, flags, umu=None, phi=None, utau=None, planck=False,
            wl=None, wu=None, nmom=None):
    from pyharp_amd import Disort, DisortOptions
    op = DisortOptions().flags(flags + (",planck" if planck else "")).nwave(nwave).ncol(ncol)
    if planck:
        op.wave_lower(list(map(float, wl))).wave_upper(list(map(float, wu)))
    if umu is not None:
        op.user_mu(list(umu))
    if phi is not None:
        op.user_phi(list(phi))
    if utau is not None:
        op.user_tau(list(utau))
    op.ds().nlyr = nlyr
    op.ds().nstr = nstr
    op.ds().nmom = nstr if nmom is None else nmom
    return Disort(op)


def _dev(d):
    return {k: torch.as_tensor(v, dtype=torch.float64, device=DEV) for k, v in d.items()}


def _col_err(got, ref):
    """max |got - ref| / max |ref| per (wave, col)"""
    g = got.reshape(got.shape[0] * got.shape[1], -1)
    r = ref.reshape(ref.shape[0] * ref.shape[1], -1)
    scale = np.maximum(np.abs(r).max(axis=1, keepdims=True), 1e-300)
    return (np.abs(g - r) / scale).max()


@pytest.mark.parametrize("case", ["1a", "1b", "1d"])
def test_disotest1_radiances(case):
    """tests/test_disort.cpp's configuration (usrtau, usrang, isotropic, nstr 16,
    umu0 = 0.1, fbeam = pi/umu0): DISOTEST-1 published fluxes and radiances."""
    g = disotest()
    c = g["cases"][case]
    d = _disort(16, 1, 1, 1, flags="usrtau,usrang,lamber,quiet,intensity_correction,"
                "old_intensity_correction,print-input,print-phase-function",
                umu=g["common"]["umu"], phi=[0.0], utau=[0.0, c["tau"]])
    assert d.ds().utau[1] == c["tau"]
    prop = torch.zeros((1, 1, 1, 18), dtype=torch.float64, device=DEV)
    prop[..., 0] = d.ds().utau[1]
    prop[..., 1] = c["ssalb"]
    bc = {"umu0": torch.full((1, 1), 0.1, dtype=torch.float64, device=DEV)}
    bc["fbeam"] = math.pi / bc["umu0"]
    flux = d.forward(prop, bc).cpu().numpy()
    uu = d.get_rad().cpu().numpy()
    assert uu.shape == (1, 1, 1, 2, 6)
    exp = np.asarray(c["uu"])
    assert np.all(np.abs(uu[0, 0, 0] - exp) <= 5e-6 * np.abs(exp) + 1e-6), (uu[0, 0, 0], exp)
    # fluxes: index 0 = the deepest user depth
    up = [c["flup"][0], c["flup"][1]]
    dn = [c["rfldir"][0] + c["rfldn"][0], c["rfldir"][1] + c["rfldn"][1]]
    for k in range(2):
        assert abs(flux[0, 0, 1 - k, 0] - up[k]) <= 5e-6 * abs(up[k]) + 1e-6
        assert abs(flux[0, 0, 1 - k, 1] - dn[k]) <= 5e-6 * abs(dn[k]) + 1e-6


def _random_case(rng, nwave, ncol, nlyr, nstr, planck, rayleigh=False):
    prop = np.zeros((nwave, ncol, nlyr, 2 + nstr))
    prop[..., 0] = 10.0 ** rng.uniform(-3, 0.7, (nwave, ncol, nlyr))
    prop[..., 1] = rng.uniform(0, 0.99, (nwave, ncol, nlyr))
    if rayleigh:
        prop[..., 3] = 0.1
    else:
        gg = rng.uniform(0, 0.8, (nwave, ncol, nlyr))
        for l in range(nstr):
            prop[..., 2 + l] = gg ** (l + 1)
    bc = {"fbeam": rng.uniform(0.5, 2, (nwave, ncol)),
          "umu0": rng.uniform(0.1, 1, (nwave, ncol)),
          "phi0": rng.uniform(0, 360, (nwave, ncol)),
          "albedo": rng.uniform(0, 1, (nwave, ncol)),
          "fisot": np.full((nwave, ncol), 0.01)}
    kw = {}
    if planck:
        from oracle.disort_np import layer2level
        kw["temf"] = layer2level(np.linspace(290, 180, nlyr)[None, :] +
                                 rng.uniform(-5, 5, (ncol, nlyr)))
        bc["btemp"] = np.full((nwave, ncol), 295.0)
        bc["ttemp"] = np.full((nwave, ncol), 150.0)
        bc["temis"] = np.full((nwave, ncol), 0.3)
        kw["wave_lower"] = np.sort(rng.uniform(100, 1500, nwave))
        kw["wave_upper"] = kw["wave_lower"] + rng.uniform(10, 300, nwave)
    return prop, bc, kw


@pytest.mark.parametrize("nstr", [2, 4, 6, 8, 12, 16, 18, 24, 32])
@pytest.mark.parametrize("planck", [False, True])
def test_radiances_vs_oracle(nstr, planck):
    """Every azimuthal mode, user depths and angles; nstr 18..32 run the same
    kernels compiled with rolled loops (hd_rad_wide.hip)."""
    rng = np.random.default_rng(500 + nstr + 50 * planck)
    nwave, ncol, nlyr = 2, 3, 6
    prop, bc, kw = _random_case(rng, nwave, ncol, nlyr, nstr, planck)
    total = prop[..., 0].sum(axis=-1).min()
    utau = np.sort(np.concatenate([[0.0, total], rng.uniform(0, total, 3)]))
    umu = [-1.0, -0.6, -0.15, 0.1, 0.45, 0.8]
    phi = [0.0, 75.0, 180.0, 300.0]
    d = _disort(nstr, nlyr, nwave, ncol, flags="usrtau,usrang,lamber,quiet", umu=umu, phi=phi,
                utau=utau, planck=planck, wl=kw.get("wave_lower"), wu=kw.get("wave_upper"))
    t = None if "temf" not in kw else torch.as_tensor(kw["temf"], device=DEV)
    flux = d.forward(torch.as_tensor(prop, device=DEV), _dev(bc), t).cpu().numpy()
    uu = d.get_rad().cpu().numpy()
    fref, uref = disort_rad_forward(prop, bc, kw.get("temf"), nstr=nstr, umu=umu, phi=phi,
                                    utau=utau, planck=planck, wave_lower=kw.get("wave_lower"),
                                    wave_upper=kw.get("wave_upper"))
    assert uu.shape == uref.shape
    assert margin(_col_err(uu, uref)) < TOL, _col_err(uu, uref)
    assert margin(rel_err(flux, fref).max()) < TOL


@pytest.mark.parametrize("numu", [8, 9, 16])
@pytest.mark.parametrize("nstr,planck", [(4, False), (16, False), (16, True), (24, False),
                                         (32, True)])
def test_radiances_many_angles_vs_oracle(numu, nstr, planck):
    """bench-like angle counts (numu 8 = the bench's, 9 = down/up unbalanced, 16);
    ncol*nwave*numu not a multiple of the 64-lane block, so the last block is partial"""
    rng = np.random.default_rng(900 + numu + nstr + 7 * planck)
    nwave, ncol, nlyr = 2, 5, 7
    prop, bc, kw = _random_case(rng, nwave, ncol, nlyr, nstr, planck)
    total = prop[..., 0].sum(axis=-1).min()
    utau = np.sort(np.concatenate([[0.0, total], rng.uniform(0, total, 2)]))
    umu = list(np.concatenate([-np.linspace(1.0, 0.12, numu // 2),
                               np.linspace(0.1, 1.0, numu - numu // 2)]))
    phi = [0.0, 120.0]
    d = _disort(nstr, nlyr, nwave, ncol, flags="usrtau,usrang,lamber,quiet", umu=umu, phi=phi,
                utau=utau, planck=planck, wl=kw.get("wave_lower"), wu=kw.get("wave_upper"))
    t = None if "temf" not in kw else torch.as_tensor(kw["temf"], device=DEV)
    flux = d.forward(torch.as_tensor(prop, device=DEV), _dev(bc), t).cpu().numpy()
    uu = d.get_rad().cpu().numpy()
    fref, uref = disort_rad_forward(prop, bc, kw.get("temf"), nstr=nstr, umu=umu, phi=phi,
                                    utau=utau, planck=planck, wave_lower=kw.get("wave_lower"),
                                    wave_upper=kw.get("wave_upper"))
    assert uu.shape == uref.shape
    assert margin(_col_err(uu, uref)) < TOL, _col_err(uu, uref)
    assert margin(rel_err(flux, fref).max()) < TOL


def test_rayleigh_nonuniform_azimuth_vs_oracle():
    """Rayleigh layers (no delta-M truncation) with a beam: strong azimuth dependence"""
    rng = np.random.default_rng(77)
    prop, bc, kw = _random_case(rng, 2, 2, 5, 8, False, rayleigh=True)
    umu = [-0.9, -0.3, 0.3, 0.9]
    phi = list(np.linspace(0, 180, 7))
    d = _disort(8, 5, 2, 2, flags="usrang,lamber", umu=umu, phi=phi)
    flux = d.forward(torch.as_tensor(prop, device=DEV), _dev(bc)).cpu().numpy()
    uu = d.get_rad().cpu().numpy()
    fref, uref = disort_rad_forward(prop, bc, nstr=8, umu=umu, phi=phi)
    assert uu.shape == (2, 2, 7, 6, 4)
    assert margin(_col_err(uu, uref)) < TOL
    assert margin(rel_err(flux, fref).max()) < TOL
    assert np.abs(uu[:, :, 0] - uu[:, :, -1]).max() > 1e-3 * np.abs(uu).max()


@pytest.mark.parametrize("nstr", [4, 16])
def test_level_fluxes_match_flux_path(nstr):
    """Radiance path without usrtau returns the level fluxes of the flux path."""
    rng = np.random.default_rng(90 + nstr)
    prop, bc, kw = _random_case(rng, 3, 4, 10, nstr, True)
    a = _disort(nstr, 10, 3, 4, flags="lamber,usrang", umu=[-0.5, 0.5], phi=[0.0], planck=True,
                wl=kw["wave_lower"], wu=kw["wave_upper"])
    b = _disort(nstr, 10, 3, 4, flags="lamber,onlyfl", planck=True, wl=kw["wave_lower"],
                wu=kw["wave_upper"])
    p = torch.as_tensor(prop, device=DEV)
    t = torch.as_tensor(kw["temf"], device=DEV)
    fa = a.forward(p, _dev(bc), t).cpu().numpy()
    fb = b.forward(p, _dev(bc), t).cpu().numpy()
    assert rel_err(fa, fb).max() < 1e-9


def test_onlyfl_user_depths_vs_oracle():
    rng = np.random.default_rng(12)
    prop, bc, kw = _random_case(rng, 2, 2, 7, 8, False)
    total = prop[..., 0].sum(axis=-1).min()
    utau = np.linspace(0, total, 9)
    d = _disort(8, 7, 2, 2, flags="usrtau,onlyfl,lamber", utau=utau)
    flux = d.forward(torch.as_tensor(prop, device=DEV), _dev(bc)).cpu().numpy()
    fref, _ = disort_rad_forward(prop, bc, nstr=8, umu=[0.5], phi=[0.0], utau=utau, onlyfl=True)
    assert flux.shape == (2, 2, 9, 2)
    assert margin(rel_err(flux, fref).max()) < TOL
    with pytest.raises(RuntimeError):
        d.get_rad()


def test_radiance_chunking_invariance():
    from pyharp_amd.disort import _context
    rng = np.random.default_rng(4)
    prop, bc, _ = _random_case(rng, 3, 5, 4, 6, False)
    d = _disort(6, 4, 3, 5, flags="usrang,lamber", umu=[-0.7, 0.2, 1.0], phi=[0.0, 90.0])
    p = torch.as_tensor(prop, device=DEV)
    f1 = d.forward(p, _dev(bc)).cpu().numpy()
    u1 = d.get_rad().cpu().numpy()
    ctx = _context(0)
    ctx.set_chunk(4)
    try:
        f2 = d.forward(p, _dev(bc)).cpu().numpy()
        u2 = d.get_rad().cpu().numpy()
    finally:
        ctx.set_chunk(0)
    assert np.array_equal(f1, f2) and np.array_equal(u1, u2)


def test_radiance_argument_errors():
    with pytest.raises(RuntimeError):
        _disort(34, 2, 1, 1, flags="usrang,lamber", umu=[0.5], phi=[0.0])
    with pytest.raises(RuntimeError):
        _disort(8, 2, 1, 1, flags="usrang,lamber", umu=[0.0], phi=[0.0])
    with pytest.raises(RuntimeError):
        _disort(8, 2, 1, 1, flags="usrtau,onlyfl,lamber", utau=[0.5, 0.1])


def test_cpp_disort_rad():
    """tests/cpp/disort_rad_dropin.cpp: the reference's tests/test_disort.cpp
    main() against harp_amd::Disort (include/harp_amd/disort.hpp)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tests", "cpp", "disort_rad_dropin")
    if not os.path.exists(exe):
        subprocess.run([os.path.join(root, "tests", "cpp", "build.sh")], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split("\n")
    c = disotest()["cases"]["1a"]
    rad = {(int(l.split()[1]), int(l.split()[2])): float(l.split()[3])
           for l in out if l.startswith("rad")}
    exp = np.asarray(c["uu"])
    for (lu, iu), v in rad.items():
        assert abs(v - exp[lu, iu]) <= 5e-6 * abs(exp[lu, iu]) + 1e-6, (lu, iu, v)
    assert len(rad) == 12
    flux = {int(l.split()[1]): (float(l.split()[2]), float(l.split()[3]))
            for l in out if l.startswith("flux")}
    # index 0 = the deepest user depth (tau = 0.03125)
    assert abs(flux[1][0] - c["flup"][0]) <= 5e-6 * c["flup"][0]
    dn_bot = c["rfldir"][1] + c["rfldn"][1]
    assert abs(flux[0][1] - dn_bot) <= 5e-6 * dn_bot


@pytest.mark.parametrize("nstr", [8, 16, 24])
def test_tms_corrected_radiances_vs_oracle(nstr):
    """intensity_correction on forward-peaked HG layers with 48 moments (delta-M
    truncation active): the TMS-corrected radiances vs the oracle's"""
    rng = np.random.default_rng(600 + nstr)
    nwave, ncol, nlyr, nmom = 2, 2, 5, 48
    prop = np.zeros((nwave, ncol, nlyr, 2 + nmom))
    prop[..., 0] = 10.0 ** rng.uniform(-3, 0.5, (nwave, ncol, nlyr))
    prop[..., 1] = rng.uniform(0.3, 0.99, (nwave, ncol, nlyr))
    g = rng.uniform(0.6, 0.85, (nwave, ncol, nlyr))
    for l in range(nmom):
        prop[..., 2 + l] = g ** (l + 1)
    bc = {"fbeam": np.ones((nwave, ncol)), "umu0": rng.uniform(0.2, 1, (nwave, ncol)),
          "phi0": rng.uniform(0, 360, (nwave, ncol)), "albedo": rng.uniform(0, 1, (nwave, ncol))}
    total = prop[..., 0].sum(axis=-1).min()
    utau = [0.0, 0.5 * total, total]
    umu, phi = [-0.9, -0.4, 0.3, 0.8], [0.0, 60.0, 180.0]
    d = _disort(nstr, nlyr, nwave, ncol, flags="usrtau,usrang,lamber,intensity_correction,"
                "old_intensity_correction", umu=umu, phi=phi, utau=utau, nmom=nmom)
    d.forward(torch.as_tensor(prop, device=DEV), _dev(bc))
    uu = d.get_rad().cpu().numpy()
    _, uref = disort_rad_forward(prop, bc, nstr=nstr, nmom=nmom, umu=umu, phi=phi, utau=utau,
                                 corint=True)
    _, u0 = disort_rad_forward(prop, bc, nstr=nstr, nmom=nmom, umu=umu, phi=phi, utau=utau)
    assert margin(_col_err(uu, uref)) < TOL
    assert _col_err(uref, u0) > 1e-3   # the correction is not a no-op here


@pytest.mark.parametrize("nstr", [16, 32])
def test_ims_aureole_vs_oracle(nstr, monkeypatch):
    """The IMS term of the Nakajima-Tanaka correction (STWL A.13-A.16) on
    forward-peaked HG layers (g 0.8-0.9, 96 moments) seen in the aureole:
    downward directions around the beam at depths inside and below the layers,
    GPU vs the oracle (TMS + IMS); the IMS term itself is not negligible here."""
    from oracle import disort_rad_np
    rng = np.random.default_rng(700 + nstr)
    nwave, ncol, nlyr, nmom = 2, 2, 3, 96
    prop = np.zeros((nwave, ncol, nlyr, 2 + nmom))
    prop[..., 0] = rng.uniform(0.05, 0.6, (nwave, ncol, nlyr))
    prop[..., 1] = rng.uniform(0.9, 0.99, (nwave, ncol, nlyr))
    g = rng.uniform(0.8, 0.9, (nwave, ncol, nlyr))
    for l in range(nmom):
        prop[..., 2 + l] = g ** (l + 1)
    umu0 = rng.uniform(0.5, 0.7, (nwave, ncol))
    bc = {"fbeam": np.ones((nwave, ncol)), "umu0": umu0, "phi0": np.zeros((nwave, ncol)),
          "albedo": rng.uniform(0, 0.3, (nwave, ncol))}
    total = prop[..., 0].sum(axis=-1).min()
    utau = [0.0, 0.3 * total, 0.7 * total, total]
    umu, phi = [-0.7, -0.62, -0.58, -0.5, 0.6], [0.0, 4.0, 15.0, 180.0]
    d = _disort(nstr, nlyr, nwave, ncol, flags="usrtau,usrang,lamber,intensity_correction,"
                "old_intensity_correction", umu=umu, phi=phi, utau=utau, nmom=nmom)
    d.forward(torch.as_tensor(prop, device=DEV), _dev(bc))
    uu = d.get_rad().cpu().numpy()
    _, uref = disort_rad_forward(prop, bc, nstr=nstr, nmom=nmom, umu=umu, phi=phi, utau=utau,
                                 corint=True)
    assert margin(_col_err(uu, uref)) < TOL
    monkeypatch.setattr(disort_rad_np, "ims_correction", lambda *a, **k: 0.0)
    _, utms = disort_rad_forward(prop, bc, nstr=nstr, nmom=nmom, umu=umu, phi=phi, utau=utau,
                                 corint=True)
    assert _col_err(uref, utms) > 1e-4   # the IMS term is resolved by the comparison


def test_radiance_umu0_as_given():
    """The intensity path takes umu0 as given like the flux path: tiny positive
    cosines {1e-4, 5e-4, 1e-3, 2e-3} against the radiance oracle; umu0 = 0 with a
    beam is cdisort's input error (the call raises)."""
    rng = np.random.default_rng(5150)
    nwave, ncol, nlyr, nstr = 1, 4, 4, 8
    prop, bc, _ = _random_case(rng, nwave, ncol, nlyr, nstr, False)
    prop[..., 0] = 10.0 ** rng.uniform(-4, -2, (nwave, ncol, nlyr))
    bc["umu0"] = np.array([[1e-4, 5e-4, 1e-3, 2e-3]])
    total = prop[..., 0].sum(axis=-1).min()
    utau = [0.0, 0.5 * total, total]
    umu = [-1.0, -0.3, 0.2, 0.9]
    phi = [0.0, 120.0]
    d = _disort(nstr, nlyr, nwave, ncol, flags="usrtau,usrang,lamber,quiet", umu=umu, phi=phi,
                utau=utau)
    flux = d.forward(torch.as_tensor(prop, device=DEV), _dev(bc)).cpu().numpy()
    uu = d.get_rad().cpu().numpy()
    fref, uref = disort_rad_forward(prop, bc, None, nstr=nstr, umu=umu, phi=phi, utau=utau)
    assert margin(_col_err(uu, uref)) < TOL, _col_err(uu, uref)
    assert margin(rel_err(flux, fref).max()) < TOL
    bc0 = dict(bc, umu0=np.array([[0.5, 0.0, 0.5, 0.5]]))
    with pytest.raises(RuntimeError):
        d.forward(torch.as_tensor(prop, device=DEV), _dev(bc0))


_USER_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + '/tests')
from test_gpu_radiance import _user_case
np.save(sys.argv[5], _user_case(int(sys.argv[2]), sys.argv[3] == '1', sys.argv[4] == '1',
                                int(sys.argv[6]), int(sys.argv[7])))
"""


def _user_case(nstr, planck, usrtau, nwave=2, nang=9):
    rng = np.random.default_rng(3100 + nstr + 10 * planck + 20 * usrtau)
    ncol, nlyr = 5, 9
    prop, bc, kw = _random_case(rng, nwave, ncol, nlyr, nstr, planck)
    total = prop[..., 0].sum(axis=-1).min()
    utau = np.sort(np.concatenate([[0.0, total], rng.uniform(0, total, 4)])) if usrtau else None
    umu = [-1.0, -0.7, -0.31, -0.12, 0.1, 0.37, 0.66, 0.93, 1.0]
    if nang == 8:
        umu.remove(0.66)
    elif nang == 4:
        umu = [-0.7, -0.12, 0.37, 1.0]
    d = _disort(nstr, nlyr, nwave, ncol, flags="lamber,quiet,usrang" + (",usrtau" if usrtau else ""),
                umu=umu, phi=[0.0, 90.0], utau=utau, planck=planck, wl=kw.get("wave_lower"),
                wu=kw.get("wave_upper"))
    t = None if "temf" not in kw else torch.as_tensor(kw["temf"], device=DEV)
    d.forward(torch.as_tensor(prop, device=DEV), _dev(bc), t)
    return d.get_rad().cpu().numpy()


@pytest.mark.parametrize("nstr,planck,usrtau,nwave", [(20, False, False, 2), (32, True, False, 2),
                                                      (24, True, True, 2), (32, False, True, 2),
                                                      (18, True, True, 1)])
def test_team_user_kernel_matches_rolled(nstr, planck, usrtau, nwave, tmp_path):
    """nstr 18..32 user angles: the team/MFMA kernel pair (per-(unit, layer) maps on
    the matrix core + per-ray scan) against the one-lane-per-(unit, angle) kernel
    (HD_RAD_USER=rolled, in a child process): the same integrals in another order,
    to rounding -- levels only (the scaled level depths that miss tau' by an ulp
    take the interior branch) and caller depths inside layers, nine angles (two
    angle blocks); 5 solves x 18 modes = 90 units leaves the last wave's group of
    four units half empty."""
    import os
    import subprocess
    import sys
    here = _user_case(nstr, planck, usrtau, nwave)
    out = tmp_path / "rolled.npy"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HD_AB="1", HD_RAD_USER="rolled")
    subprocess.run([sys.executable, "-c", _USER_CHILD, root, str(nstr), "1" if planck else "0",
                    "1" if usrtau else "0", str(out), str(nwave), "9"], check=True, env=env,
                   timeout=300)
    other = np.load(out)
    assert np.all(np.isfinite(here))
    assert margin(_col_err(here, other)) < 1e-10, _col_err(here, other)


def test_many_user_angles_fallback_vs_oracle():
    """More user angles than a layer record holds (nstr 18: 109): the one-lane
    const and user-angle kernels run on the team kernels' unit-contiguous records"""
    rng = np.random.default_rng(4242)
    nstr, nwave, ncol, nlyr = 18, 1, 2, 4
    prop, bc, kw = _random_case(rng, nwave, ncol, nlyr, nstr, False)
    umu = list(np.concatenate([-np.linspace(1.0, 0.05, 60), np.linspace(0.05, 1.0, 60)]))
    total = prop[..., 0].sum(axis=-1).min()
    utau = [0.0, 0.37 * total, total]
    d = _disort(nstr, nlyr, nwave, ncol, flags="usrtau,usrang,lamber,quiet", umu=umu,
                phi=[0.0, 90.0], utau=utau)
    flux = d.forward(torch.as_tensor(prop, device=DEV), _dev(bc)).cpu().numpy()
    uu = d.get_rad().cpu().numpy()
    fref, uref = disort_rad_forward(prop, bc, nstr=nstr, umu=umu, phi=[0.0, 90.0], utau=utau)
    assert uu.shape == uref.shape
    assert margin(_col_err(uu, uref)) < TOL, _col_err(uu, uref)
    assert margin(rel_err(flux, fref).max()) < TOL
