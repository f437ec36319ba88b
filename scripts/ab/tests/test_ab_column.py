"""The nstr-16 column kernel (hd_column_kernel: layer setup, adding sweep and
back-substitution of a solve in one pass, the layer records kept on chip) against
the three-kernel register path (hd_layer_kernel + hd_sweep_kernel + the
back-substitution, records in HBM).  Both run the same layer_body / sweep_body /
backsub_body code, so they agree to rounding (relative 1e-12 of the column's flux
scale; the compiler may contract a product into an FMA differently in the two
inlining contexts).  The switch HD_COLUMN is read when a context is created, so
the other variant runs in a child process.  Cases: beam and Planck, one chunk and
chunks with partial waves (lanes past the chunk), per-point fluxes and the fused
band sum (the chunked run of each variant equals its one-chunk run bit for bit)."""
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
pytestmark = pytest.mark.gpu

CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + '/tests')
sys.path.insert(0, sys.argv[1] + '/scripts/ab/tests')
from test_ab_column import _solve
f, b = _solve(sys.argv[2] == '1')
np.save(sys.argv[3], f); np.save(sys.argv[4], b)
"""


def _solve(planck):
    import torch
    from test_gpu_parity import _disort, _random_batch
    from pyharp_amd.disort import _context
    rng = np.random.default_rng(7300 + planck)
    nwave, ncol, nlyr, nstr = 5, 29, 17, 16
    prop, bc, kw = _random_batch(rng, nwave, ncol, nlyr, nstr, planck)
    wts = rng.uniform(0.1, 1.0, nwave)
    dev = torch.device("cuda", 0)
    t = lambda x: None if x is None else torch.as_tensor(x, dtype=torch.float64, device=dev)
    p, b, tf, w = t(prop), {k: t(v) for k, v in bc.items()}, t(kw.get("temf")), t(wts)
    d = _disort(nstr, nlyr, nwave, ncol, planck=planck, wl=kw.get("wave_lower"),
                wu=kw.get("wave_upper"))
    ctx = _context(0)
    flux, band = [], []
    for chunk in (0, 23, 64):
        ctx.set_chunk(chunk)
        try:
            flux.append(d.forward(p, b, tf).cpu().numpy())
            band.append(d.forward_band(p, b, tf, weights=w).cpu().numpy())
        finally:
            ctx.set_chunk(0)
    return np.stack(flux), np.stack(band)


@pytest.mark.parametrize("planck", [False, True])
def test_column_kernel_matches_three_kernel_path(planck, tmp_path, ab_lib):
    here_f, here_b = _solve(planck)
    col_here = os.environ.get("HD_AB") == "1" and os.environ.get("HD_COLUMN") == "1"
    of, ob = tmp_path / "f.npy", tmp_path / "b.npy"
    env = dict(os.environ, HD_LIB_PATH=ab_lib, HD_AB="1", HD_COLUMN="0" if col_here else "1")
    subprocess.run([sys.executable, "-c", CHILD, ROOT, "1" if planck else "0", str(of), str(ob)],
                   check=True, env=env, timeout=300)
    other_f, other_b = np.load(of), np.load(ob)
    for here, other in ((here_f, other_f), (here_b, other_b)):
        assert np.all(np.isfinite(here)) and np.all(np.isfinite(other))
        scale = np.abs(here).max(axis=(-1, -2), keepdims=True)
        assert np.all(np.abs(here - other) <= 1e-12 * scale + 1e-300)
    for x in (here_f, other_f):  # per-point fluxes: the chunk plan changes no bit
        np.testing.assert_array_equal(x[0], x[1])
        np.testing.assert_array_equal(x[0], x[2])
