"""ctypes front-end for the C oracle ``oracle/lib/libhdoracle.so``.

TEST INFRASTRUCTURE ONLY (checker and timed CPU baseline); see
``oracle/disort_oracle.c`` for what it restates and its parity status.
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libhdoracle.so")
_lib = None

_dp = ctypes.POINTER(ctypes.c_double)


def build(force: bool = False) -> str:
    """Compile the C oracle with gcc (``make -C oracle``; make skips an up-to-date build)."""
    cmd = ["make", "-C", _HERE] + (["-B"] if force else [])
    subprocess.run(cmd, check=True, capture_output=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.hdo_plkavg.restype = ctypes.c_double
        _lib.hdo_plkavg.argtypes = [ctypes.c_double] * 3
        _lib.hdo_forward.restype = ctypes.c_long
        _lib.hdo_forward.argtypes = ([ctypes.c_int] * 7 + [_dp] * 11 +
                                     [_dp, ctypes.c_int, ctypes.c_long, ctypes.c_long])
        _lib.hdo_column.restype = ctypes.c_int
        _lib.hdo_column.argtypes = ([ctypes.c_int] * 3 + [_dp] * 3 + [ctypes.c_int, _dp] +
                                    [ctypes.c_double] * 9 + [_dp] * 3)
    return _lib


def _ptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(_dp)


def plkavg(wnumlo, wnumhi, t):
    return lib().hdo_plkavg(float(wnumlo), float(wnumhi), float(t))


def column(dtauc, ssalb, pmom, nstr, *, umu0=1.0, fbeam=0.0, albedo=0.0,
           fisot=0.0, planck=False, temper=None, btemp=0.0, ttemp=0.0,
           temis=0.0, wvnmlo=0.0, wvnmhi=0.0):
    """One solve in cdisort conventions (layers top->bottom)."""
    dtauc = np.ascontiguousarray(dtauc, np.float64)
    nlyr = dtauc.size
    ssalb = np.ascontiguousarray(ssalb, np.float64)
    pmom = np.ascontiguousarray(np.asarray(pmom, np.float64).reshape(nlyr, -1))
    nmom = pmom.shape[1] - 1
    tem = np.ascontiguousarray(temper if temper is not None else np.zeros(nlyr + 1), np.float64)
    out = [np.zeros(nlyr + 1) for _ in range(3)]
    rc = lib().hdo_column(nstr, nlyr, nmom, _ptr(dtauc), _ptr(ssalb), _ptr(pmom),
                          int(planck), _ptr(tem), umu0, fbeam, albedo, fisot, btemp,
                          ttemp, temis, wvnmlo, wvnmhi, *[_ptr(o) for o in out])
    if rc:
        raise ArithmeticError(f"hdo_column failed ({rc})")
    return {"rfldir": out[0], "rfldn": out[1], "flup": out[2], "fdn": out[0] + out[1]}


def forward(prop, bc, temf=None, *, nstr, nmom=None, planck=False,
            wave_lower=None, wave_upper=None, nthreads=0, first=0, count=-1,
            out=None):
    """harp-layout batch solve; same contract as ``disort_np.disort_forward``."""
    prop = np.ascontiguousarray(prop, np.float64)
    nwave, ncol, nlyr, nprop = prop.shape
    if nmom is None:
        nmom = nstr

    def bca(key):
        v = bc.get(key) if bc else None
        if v is None:
            return None
        return np.ascontiguousarray(np.broadcast_to(np.asarray(v, np.float64), (nwave, ncol)))

    arrs = [bca(k) for k in ("fbeam", "umu0", "albedo", "btemp", "ttemp", "temis", "fisot")]
    tf = None if temf is None else np.ascontiguousarray(temf, np.float64)
    wl = None if wave_lower is None else np.ascontiguousarray(wave_lower, np.float64)
    wu = None if wave_upper is None else np.ascontiguousarray(wave_upper, np.float64)
    if out is None:
        out = np.zeros((nwave, ncol, nlyr + 1, 2))
    nfail = lib().hdo_forward(nwave, ncol, nlyr, nprop, nstr, nmom, int(planck), _ptr(prop),
                              *[_ptr(a) for a in arrs], _ptr(tf), _ptr(wl), _ptr(wu),
                              _ptr(out), int(nthreads), int(first), int(count))
    if nfail:
        raise ArithmeticError(f"hdo_forward: {nfail} failed solves")
    return out
