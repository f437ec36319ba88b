"""The nstr 4 / 8 sweep in NN-lane teams (hd_sweep_quad_kernel) against the
one-lane sweep (hd_sweep_kernel): the switch HD_SWEEP_QUAD is read when a context
is created, so the other variant runs in a child process.  The team sweep replaces
the LU of W1 by a Gauss-Jordan elimination with the same pivots, so the fluxes
agree to rounding (relative 1e-11 of the column's flux scale) -- beam and Planck,
one chunk and several, ragged last team."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + '/tests')
from test_gpu_quad_sweep import _solve
np.save(sys.argv[4], _solve(int(sys.argv[2]), sys.argv[3] == '1'))
"""


def _solve(nstr, planck, chunk=23):
    from test_gpu_parity import _disort, _random_batch, _run
    from pyharp_amd.disort import _context
    rng = np.random.default_rng(5000 + nstr + planck)
    nwave, ncol, nlyr = 3, 31, 14
    prop, bc, kw = _random_batch(rng, nwave, ncol, nlyr, nstr, planck)
    d = _disort(nstr, nlyr, nwave, ncol, planck=planck, wl=kw.get("wave_lower"),
                wu=kw.get("wave_upper"))
    out = [_run(d, prop, bc, kw.get("temf"))]
    ctx = _context(0)
    ctx.set_chunk(chunk)
    try:
        out.append(_run(d, prop, bc, kw.get("temf")))
    finally:
        ctx.set_chunk(0)
    return np.stack(out)


@pytest.mark.parametrize("nstr,planck", [(4, False), (4, True), (8, False), (8, True)])
def test_quad_sweep_matches_one_lane(nstr, planck, tmp_path):
    here = _solve(nstr, planck)
    quad_here = not (os.environ.get("HD_AB") == "1" and os.environ.get("HD_SWEEP_QUAD") == "0")
    out = tmp_path / "other.npy"
    env = dict(os.environ, HD_AB="1", HD_SWEEP_QUAD="0" if quad_here else "1")
    subprocess.run([sys.executable, "-c", CHILD, ROOT, str(nstr), "1" if planck else "0",
                    str(out)], check=True, env=env, timeout=300)
    other = np.load(out)
    assert np.all(np.isfinite(here)) and np.all(np.isfinite(other))
    # per column (axis -3 of [..., ncol, nlev, 2]): scale of its fluxes
    scale = np.abs(here).max(axis=(-1, -2), keepdims=True)
    assert np.all(np.abs(here - other) <= 1e-11 * scale + 1e-300)
    # the chunked run of each variant equals its one-chunk run bit for bit
    np.testing.assert_array_equal(here[0], here[1])
    np.testing.assert_array_equal(other[0], other[1])
