"""The nstr-16 sweep with the stack state in LDS (hd_sweep_lean_kernel, two waves
per SIMD; an A/B variant, off by default) against the register-resident one-lane
sweep (hd_sweep_kernel, the default): the switch HD_SWEEP_LEAN8 is read when a context is created,
so the other variant runs in a child process.  The lean sweep forms M1 = Ra W1^-1
from its upper triangle and carries the direct beam as a running product of the
layers' transmissions instead of exp(-tau_c/mu0), so the fluxes agree to rounding
(relative 1e-11 of the column's flux scale) -- beam and Planck, one chunk and
several (the chunked run of each variant equals its one-chunk run bit for bit)."""
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
from test_ab_lean8_sweep import _solve
np.save(sys.argv[3], _solve(sys.argv[2] == '1'))
"""


def _solve(planck, chunk=23):
    from test_gpu_parity import _disort, _random_batch, _run
    from pyharp_amd.disort import _context
    rng = np.random.default_rng(7100 + planck)
    nwave, ncol, nlyr, nstr = 3, 31, 14, 16
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


@pytest.mark.parametrize("planck", [False, True])
def test_lean8_sweep_matches_register_sweep(planck, tmp_path, ab_lib):
    here = _solve(planck)
    lean_here = os.environ.get("HD_AB") == "1" and os.environ.get("HD_SWEEP_LEAN8") == "1"
    out = tmp_path / "other.npy"
    env = dict(os.environ, HD_LIB_PATH=ab_lib, HD_AB="1", HD_SWEEP_LEAN8="0" if lean_here else "1")
    subprocess.run([sys.executable, "-c", CHILD, ROOT, "1" if planck else "0", str(out)],
                   check=True, env=env, timeout=300)
    other = np.load(out)
    assert np.all(np.isfinite(here)) and np.all(np.isfinite(other))
    scale = np.abs(here).max(axis=(-1, -2), keepdims=True)
    assert np.all(np.abs(here - other) <= 1e-11 * scale + 1e-300)
    np.testing.assert_array_equal(here[0], here[1])
    np.testing.assert_array_equal(other[0], other[1])
