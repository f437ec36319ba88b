"""The lean team sweep (hd_team_mfma_sweep_lean_kernel: the same arithmetic in
at most 256 registers, two waves per SIMD) against the one-wave team sweep: the
switch HD_TEAM_SWEEP_LEAN is read when a context is created, so the other variant
runs in a child process.  The operands only live elsewhere between their uses, so
the fluxes must agree bit for bit -- nstr 18..32, beam and Planck, one chunk and
several (the two-stream pipeline)."""
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
from test_ab_team_sweep import _solve
np.save(sys.argv[4], _solve(int(sys.argv[2]), sys.argv[3] == '1'))
"""


def _solve(nstr, planck, chunk=23):
    from test_gpu_parity import _disort, _random_batch, _run
    from pyharp_amd.disort import _context
    rng = np.random.default_rng(4000 + nstr + planck)
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


@pytest.mark.parametrize("nstr,planck", [(18, False), (24, True), (32, False), (32, True)])
def test_lean_sweep_bitwise(nstr, planck, tmp_path, ab_lib):
    here = _solve(nstr, planck)
    lean_here = not (os.environ.get("HD_AB") == "1" and os.environ.get("HD_TEAM_SWEEP_LEAN") == "0")
    out = tmp_path / "other.npy"
    env = dict(os.environ, HD_LIB_PATH=ab_lib, HD_AB="1", HD_TEAM_SWEEP_LEAN="0" if lean_here else "1")
    subprocess.run([sys.executable, "-c", CHILD, ROOT, str(nstr), "1" if planck else "0",
                    str(out)], check=True, env=env, timeout=300)
    other = np.load(out)
    assert np.all(np.isfinite(here))
    np.testing.assert_array_equal(here, other)
