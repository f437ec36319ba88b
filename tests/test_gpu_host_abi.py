"""The host-array entry points of the boundary (include/hdisort.h: hd_solve_host,
hd_solve_band_host) -- pydisort's own CPU-tensor contract -- called through ctypes
with numpy arrays and from a plain-C program (tests/cpp/host_abi.c), against the
CPU oracle.  The solve itself runs on the device (no CPU arithmetic in the product).
"""

import ctypes
import os
import subprocess

import numpy as np
import pytest

from helpers import TOL, rel_err, margin

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _solve_host(lib, ctx, nstr, prop, bc, temf=None, wl=None, wu=None, weight=None,
                keep_flux=True):
    from pyharp_amd import _lib
    nwave, ncol, nlyr, nprop = prop.shape
    planck = temf is not None
    cfg = _lib.HdConfig(nstr, nstr, nlyr, nprop,
                        _lib.HD_FLAG_LAMBER | _lib.HD_FLAG_ONLYFL | (_lib.HD_FLAG_PLANCK if planck else 0))
    arr = {k: np.ascontiguousarray(v, np.float64) for k, v in bc.items()}
    prop = np.ascontiguousarray(prop)
    temf = None if temf is None else np.ascontiguousarray(temf, np.float64)
    wl = None if wl is None else np.ascontiguousarray(wl, np.float64)
    wu = None if wu is None else np.ascontiguousarray(wu, np.float64)
    inp = _lib.HdInputs(nwave, ncol, _ptr(prop), _ptr(arr.get("fbeam")), _ptr(arr.get("umu0")),
                        _ptr(arr.get("albedo")), _ptr(arr.get("btemp")), _ptr(arr.get("ttemp")),
                        _ptr(arr.get("temis")), _ptr(arr.get("fisot")), _ptr(temf), _ptr(wl),
                        _ptr(wu))
    status = np.zeros((nwave, ncol), np.int32)
    flux = np.zeros((nwave, ncol, nlyr + 1, 2)) if keep_flux else None
    if weight is None:
        rc = lib.hd_solve_host(ctx, ctypes.byref(cfg), ctypes.byref(inp), _ptr(flux),
                               _ptr(status))
        return rc, flux, None, status
    w = np.ascontiguousarray(weight, np.float64)
    bflux = np.zeros((ncol, nlyr + 1, 2))
    rc = lib.hd_solve_band_host(ctx, ctypes.byref(cfg), ctypes.byref(inp), _ptr(w), _ptr(bflux),
                                _ptr(flux), _ptr(status))
    return rc, flux, bflux, status


@pytest.fixture(scope="module")
def hd():
    from pyharp_amd import _lib
    lib = _lib.load()
    ctx = ctypes.c_void_p()
    assert lib.hd_context_create(ctypes.byref(ctx), 0) == 0
    yield lib, ctx
    lib.hd_context_destroy(ctx)


def _batch(rng, nwave, ncol, nlyr, nstr, planck):
    prop = np.zeros((nwave, ncol, nlyr, 2 + nstr))
    prop[..., 0] = 10.0 ** rng.uniform(-3, 0.7, (nwave, ncol, nlyr))
    prop[..., 1] = rng.uniform(0.0, 0.99, (nwave, ncol, nlyr))
    g = rng.uniform(0.0, 0.85, (nwave, ncol, nlyr))
    for l in range(nstr):
        prop[..., 2 + l] = g ** (l + 1)
    bc = {"fbeam": np.ones((nwave, ncol)), "umu0": rng.uniform(0.1, 1.0, (nwave, ncol)),
          "albedo": rng.uniform(0.0, 1.0, (nwave, ncol))}
    kw = {}
    if planck:
        bc["btemp"] = rng.uniform(200, 320, (nwave, ncol))
        kw["temf"] = rng.uniform(150, 300, (ncol, nlyr + 1))
        kw["wl"] = rng.uniform(100, 2000, nwave)
        kw["wu"] = kw["wl"] + rng.uniform(1, 300, nwave)
    return prop, bc, kw


@pytest.mark.parametrize("nstr,planck", [(8, False), (16, True), (24, False)])
def test_solve_host_matches_oracle(hd, oracle_c, nstr, planck):
    lib, ctx = hd
    rng = np.random.default_rng(800 + nstr + planck)
    nwave, ncol, nlyr = 3, 17, 20
    prop, bc, kw = _batch(rng, nwave, ncol, nlyr, nstr, planck)
    rc, flux, _, status = _solve_host(lib, ctx, nstr, prop, bc, kw.get("temf"), kw.get("wl"),
                                      kw.get("wu"))
    assert rc == 0, lib.hd_last_error(ctx)
    assert not (status & 0x0F).any()
    ref = oracle_c.forward(prop, bc, kw.get("temf"), nstr=nstr, planck=planck,
                           wave_lower=kw.get("wl"), wave_upper=kw.get("wu"))
    assert margin(rel_err(flux, ref).max()) < TOL


@pytest.mark.parametrize("nstr,keep", [(16, True), (16, False), (32, False)])
def test_solve_band_host_matches_oracle(hd, oracle_c, nstr, keep):
    lib, ctx = hd
    rng = np.random.default_rng(900 + nstr + keep)
    nwave, ncol, nlyr = 6, 9, 16
    prop, bc, _ = _batch(rng, nwave, ncol, nlyr, nstr, False)
    w = rng.uniform(0.1, 1.0, nwave)
    rc, flux, bflux, _ = _solve_host(lib, ctx, nstr, prop, bc, weight=w, keep_flux=keep)
    assert rc == 0, lib.hd_last_error(ctx)
    ref = oracle_c.forward(prop, bc, nstr=nstr)
    bref = (ref * w[:, None, None, None]).sum(axis=0)
    scale = np.abs(bref).max()
    assert margin((np.abs(bflux - bref) / np.maximum(np.abs(bref), 1e-6 * scale)).max()) < TOL
    if keep:
        assert margin(rel_err(flux, ref).max()) < TOL


@pytest.mark.parametrize("band", [False, True])
def test_host_pieces_pipeline(hd, oracle_c, band):
    """Batches above ~128 k solves go over in pieces of whole waves (the copy of piece
    j+1 beside the solve of piece j): 7 waves x 40 000 columns = three pieces, the
    last one short; every solve of a sample and the band sum against the oracle."""
    lib, ctx = hd
    rng = np.random.default_rng(77 + band)
    nwave, ncol, nlyr, nstr = 7, 40000, 6, 8
    prop, bc, _ = _batch(rng, nwave, ncol, nlyr, nstr, False)
    w = rng.uniform(0.1, 1.0, nwave) if band else None
    rc, flux, bflux, status = _solve_host(lib, ctx, nstr, prop, bc, weight=w)
    assert rc == 0, lib.hd_last_error(ctx)
    assert not (status & 0x0F).any()
    idx = rng.choice(nwave * ncol, 200, replace=False)
    ref = np.zeros_like(flux)
    for q in idx:
        oracle_c.forward(prop, bc, nstr=nstr, first=int(q), count=1, out=ref)
    got = flux.reshape(-1, nlyr + 1, 2)[idx]
    assert margin(rel_err(got, ref.reshape(-1, nlyr + 1, 2)[idx]).max()) < TOL
    if band:
        cols = rng.choice(ncol, 20, replace=False)
        sub = {k: v[:, cols] for k, v in bc.items()}
        rsub = oracle_c.forward(np.ascontiguousarray(prop[:, cols]), sub, nstr=nstr)
        bref = (rsub * w[:, None, None, None]).sum(axis=0)
        assert np.abs(bflux[cols] - bref).max() <= 1e-9 * np.abs(bref).max()


def test_solve_host_reports_bad_input(hd):
    from pyharp_amd import _lib
    lib, ctx = hd
    rng = np.random.default_rng(5)
    prop, bc, _ = _batch(rng, 2, 3, 5, 8, False)
    prop[1, 2, 3, 1] = 1.5  # single-scattering albedo > 1
    rc, _, _, status = _solve_host(lib, ctx, 8, prop, bc)
    assert rc == _lib.HD_ENUMERIC
    assert status[1, 2] & _lib.HD_STATUS_BAD_INPUT
    assert not (status.reshape(-1)[:-1] & 0x0F).any()


def test_plain_c_caller(oracle_c):
    exe = os.path.join(HERE, "cpp", "host_abi")
    if not os.path.exists(exe):
        pytest.skip("tests/cpp/host_abi not built (tests/cpp/build.sh, run by build())")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    NW, NC, NL, NSTR = 3, 5, 12, 8
    flux = np.zeros((NW, NC, NL + 1, 2))
    band = np.zeros((NC, NL + 1, 2))
    for line in out.stdout.splitlines():
        f = line.split()
        if f[0] == "flux":
            flux[int(f[1]), int(f[2]), int(f[3])] = float(f[4]), float(f[5])
        elif f[0] == "band":
            band[int(f[1]), int(f[2])] = float(f[3]), float(f[4])
    # the program's inputs, restated
    prop = np.zeros((NW, NC, NL, 2 + NSTR))
    bc = {k: np.zeros((NW, NC)) for k in ("fbeam", "umu0", "albedo")}
    for w in range(NW):
        for c in range(NC):
            bc["fbeam"][w, c] = 1.0 + 0.1 * w
            bc["umu0"][w, c] = 0.3 + 0.12 * c
            bc["albedo"][w, c] = 0.05 + 0.15 * c
            for l in range(NL):
                g = 0.1 + 0.06 * ((w + c + l) % 10)
                prop[w, c, l, 0] = 0.01 * 1.7 ** ((l + 2 * w + c) % 11)
                prop[w, c, l, 1] = 0.3 + 0.05 * ((3 * l + w) % 13)
                prop[w, c, l, 2:] = g ** np.arange(1, NSTR + 1)
    ref = oracle_c.forward(prop, bc, nstr=NSTR)
    assert margin(rel_err(flux, ref).max()) < TOL
    bref = (ref * np.array([0.2, 0.3, 0.5])[:, None, None, None]).sum(axis=0)
    assert np.abs(band - bref).max() <= 1e-9 * np.abs(bref).max()
