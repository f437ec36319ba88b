"""Fused band epilogue (hd_solve_band / Disort.forward_band) vs the oracle.

SURVEY 8(f) rank 2: the band flux bflx = sum_w w_w F_w that every harp caller
forms from forward's result (examples/amars_lw.cpp:84-88, amars_sw.cpp:169-196)
is summed inside the solve.  Checked against the C oracle's per-point fluxes
summed in numpy (TOL of tests/helpers.py), against the unfused GPU path
(forward + hd_band_flux, 1e-12: only the summation order differs), for
bitwise reproducibility, and with chunk sizes that split columns across chunks
and waves (register path) or wave-points across chunks (team path).
"""

import numpy as np
import pytest
import torch

from helpers import TOL, rel_err, margin
from test_gpu_parity import _disort, _random_batch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _dev(x):
    return torch.as_tensor(x, dtype=torch.float64, device=DEV)


def _inputs(prop, bc, kw):
    return _dev(prop), {k: _dev(v) for k, v in bc.items()}, \
        (None if kw.get("temf") is None else _dev(kw["temf"]))


def _band_ref(ref_flux, wts):
    return np.einsum("w,wclk->clk", wts, ref_flux)


def _with_chunk(chunk, fn):
    from pyharp_amd.disort import _context
    ctx = _context(0)
    ctx.set_chunk(chunk)
    try:
        return fn()
    finally:
        ctx.set_chunk(0)


# (nstr, nwave, ncol, planck, chunk): chunk 0 = automatic (one chunk here);
# odd chunk sizes put column boundaries inside waves and chunks
CASES = [
    (16, 64, 24, False, 0),
    (16, 64, 24, False, 1000),   # 1000 = 15 columns + 40 points: straddles
    (16, 8, 50, False, 77),      # 8 columns per wave, misaligned chunks
    (8, 3, 40, True, 0),         # nwave not a power of two
    (8, 100, 5, True, 130),      # nwave > 64: a column spans several waves
    (8, 200, 1, True, 96),       # one column (line-by-line shape), many chunks
    (4, 1, 70, False, 0),        # nwave = 1: every lane its own column
    (12, 17, 9, False, 40),
    (24, 6, 10, False, 0),       # team path
    (32, 5, 7, False, 11),       # team path, chunks split the wave axis
]


@pytest.mark.parametrize("nstr,nwave,ncol,planck,chunk", CASES)
def test_band_matches_oracle(oracle_c, nstr, nwave, ncol, planck, chunk):
    rng = np.random.default_rng(7000 + nstr + nwave + ncol + chunk)
    nlyr = 20
    prop, bc, kw = _random_batch(rng, nwave, ncol, nlyr, nstr, planck)
    wts = rng.uniform(0.1, 1.0, nwave)
    ref = oracle_c.forward(prop, bc, kw.get("temf"), nstr=nstr, planck=planck,
                           wave_lower=kw.get("wave_lower"), wave_upper=kw.get("wave_upper"))
    bref = _band_ref(ref, wts)
    d = _disort(nstr, nlyr, nwave, ncol, planck=planck, wl=kw.get("wave_lower"),
                wu=kw.get("wave_upper"))
    p, b, t = _inputs(prop, bc, kw)
    w = _dev(wts)
    band = _with_chunk(chunk, lambda: d.forward_band(p, b, t, weights=w)).cpu().numpy()
    err = rel_err(band, bref).max()
    assert margin(err) < TOL, f"fused band vs oracle: {err:.3e}"
    # unfused GPU path: per-point fluxes, then hd_band_flux
    from pyharp_amd.spectral import band_flux
    flux = d.forward(p, b, t)
    bunf = band_flux(flux, w).cpu().numpy()
    scale = np.abs(bunf).max()
    assert np.abs(band - bunf).max() <= 1e-12 * scale


@pytest.mark.parametrize("nstr,chunk", [(16, 0), (16, 333), (8, 50), (28, 0), (28, 13)])
def test_band_keeps_point_fluxes_and_is_deterministic(nstr, chunk):
    """With `flux` given the per-point fluxes are the plain forward's, bit for bit
    (each solve's arithmetic does not depend on its lane); two calls give
    bitwise-identical band fluxes."""
    rng = np.random.default_rng(99 + nstr + chunk)
    nwave, ncol, nlyr = 16, 30, 24
    prop, bc, kw = _random_batch(rng, nwave, ncol, nlyr, nstr, False)
    d = _disort(nstr, nlyr, nwave, ncol)
    p, b, t = _inputs(prop, bc, kw)
    w = _dev(rng.uniform(0, 1, nwave))
    flux = torch.empty((nwave, ncol, nlyr + 1, 2), dtype=torch.float64, device=DEV)

    def run():
        b1 = d.forward_band(p, b, t, weights=w, flux=flux).clone()
        b2 = d.forward_band(p, b, t, weights=w)
        return b1, b2
    b1, b2 = _with_chunk(chunk, run)
    plain = _with_chunk(chunk, lambda: d.forward(p, b, t))
    assert torch.equal(flux, plain)
    assert torch.equal(b1, b2)


def test_band_rejects_bad_shapes():
    d = _disort(8, 10, 4, 3)
    p = torch.zeros((4, 3, 10, 10), dtype=torch.float64, device=DEV)
    p[..., 0] = 0.1
    with pytest.raises(RuntimeError, match="weights"):
        d.forward_band(p, {}, weights=_dev(np.ones(3)))
    with pytest.raises(RuntimeError, match="out must be"):
        d.forward_band(p, {}, weights=_dev(np.ones(4)),
                       out=torch.empty((3, 10, 2), dtype=torch.float64, device=DEV))


def test_band_status_flags_bad_input():
    """Errors keep their per-solve semantics in the column-major order."""
    nwave, ncol, nlyr = 8, 9, 6
    d = _disort(8, nlyr, nwave, ncol)
    p = torch.zeros((nwave, ncol, nlyr, 10), dtype=torch.float64, device=DEV)
    p[..., 0] = 0.2
    p[..., 1] = 0.5
    p[5, 7, 2, 1] = 1.5  # bad ssa in solve (w=5, c=7)
    st = torch.zeros(nwave * ncol, dtype=torch.int32, device=DEV)
    d.forward_band(p, {}, weights=_dev(np.ones(nwave)), status=st)
    bad = (st & 0xF).nonzero().flatten().cpu().tolist()
    assert bad == [5 * ncol + 7]
