"""nstr <= 16 user angles: hd_rad_user_map_kernel (the product: per-(unit, layer)
angle-independent maps formed by the const kernel) against the per-angle
hd_rad_user_kernel (HD_RAD_USER=direct, compiled only into the A/B build), run in a
child process on the A/B library.  Moved here from tests/test_gpu_radiance.py when
the not-kept variants left the product library (round 6)."""
import numpy as np
import pytest

from helpers import margin
from test_gpu_radiance import _USER_CHILD, _col_err, _user_case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nstr,planck,usrtau,nwave,nang", [
    (16, False, False, 2, 9), (16, True, True, 2, 9), (8, True, False, 1, 9), (12, False, True, 2, 9),
    (4, True, True, 1, 9), (16, False, True, 2, 8), (16, True, False, 1, 8), (10, True, True, 2, 8),
    (16, True, True, 2, 4)])
def test_user_map_kernel_matches_direct(nstr, planck, usrtau, nwave, nang, tmp_path, ab_lib):
    """nstr <= 16 user angles: the const kernel's per-(unit, layer) maps + the
    per-angle dot products (hd_rad_user_map_kernel, the default) against the
    per-angle Legendre sums, triangular solve and V^T products of
    hd_rad_user_kernel (HD_RAD_USER=direct, in a child process): the same
    integrals regrouped, to rounding -- level depths and caller depths inside
    layers, beam and thermal sources, nine angles of both signs.  Every angle count
    runs the one map kernel (hd_rad_user_map_kernel); the eight- and four-angle cases
    exercise its partial waves."""
    import os
    import subprocess
    import sys
    here = _user_case(nstr, planck, usrtau, nwave, nang)
    out = tmp_path / "direct.npy"
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    env = dict(os.environ, HD_LIB_PATH=ab_lib, HD_AB="1", HD_RAD_USER="direct")
    subprocess.run([sys.executable, "-c", _USER_CHILD, root, str(nstr), "1" if planck else "0",
                    "1" if usrtau else "0", str(out), str(nwave), str(nang)], check=True, env=env,
                   timeout=300)
    other = np.load(out)
    assert np.all(np.isfinite(here))
    assert margin(_col_err(here, other)) < 1e-10, _col_err(here, other)
