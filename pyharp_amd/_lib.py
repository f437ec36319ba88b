"""ctypes binding of libhdisort.so (C-ABI declared in include/hdisort.h).

This is the reference-side binding a pyharp maintainer would add (the
Python analogue of the cgo/JNI stub in INTEGRATION.md).  It loads the in-tree
shared library and fails loudly when it is missing: there is no CPU fallback.
"""

from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libhdisort.so")

HD_OK, HD_EINVAL, HD_ENUMERIC, HD_EHIP, HD_ENOMEM = 0, 1, 2, 3, 4
HD_FLAG_LAMBER, HD_FLAG_PLANCK, HD_FLAG_ONLYFL = 0x1, 0x2, 0x4
HD_STATUS_BAD_INPUT = 0x01
HD_STATUS_EIGEN = 0x02
HD_STATUS_NONFINITE = 0x04
HD_STATUS_RESONANCE = 0x10
HD_STATUS_PIVOT = 0x20
HD_STATUS_ERROR_MASK = 0x0F

# every symbol include/hdisort.h declares
EXPORTED = ("hd_version", "hd_last_error", "hd_context_create", "hd_context_destroy",
            "hd_context_set_chunk", "hd_context_set_timing", "hd_context_set_max_sweeps",
            "hd_context_get_timing",
            "hd_context_reserve", "hd_solve", "hd_solve_band", "hd_solve_host",
            "hd_solve_band_host", "hd_solve_radiance", "hd_quadrature", "hd_chunk_solves")

# every symbol include/hdharp.h declares (harp-side steps around the solve)
HARP_EXPORTED = ("hd_attenuate", "hd_band_optics", "hd_band_loop_optics", "hd_rfm_attenuate",
                 "hd_band_flux", "hd_heating_rate", "hd_spherical_flux_correction")
HD_COORD_WAVELENGTH, HD_COORD_WAVENUMBER = 0, 1

# every symbol include/hdnc.h declares (netCDF readers, host code)
NC_EXPORTED = ("hd_nc_open", "hd_nc_close", "hd_nc_dim_len", "hd_nc_var_size",
               "hd_nc_get_var_double")

_dp = ctypes.c_void_p


class HdAttenuator(ctypes.Structure):
    _fields_ = [("nrow", ctypes.c_int), ("wavelength", _dp), ("kext", _dp), ("ssa", _dp),
                ("species", ctypes.c_int)]


class HdBandAttenuator(ctypes.Structure):
    _fields_ = [("table", HdAttenuator), ("gasym", _dp)]


class HdRfmTable(ctypes.Structure):
    _fields_ = [("nwave", ctypes.c_int), ("npres", ctypes.c_int), ("ntemp", ctypes.c_int),
                ("wave", _dp), ("lnp", _dp), ("tgrid", _dp), ("tref", _dp), ("kdata", _dp),
                ("species", ctypes.c_int)]


class HdConfig(ctypes.Structure):
    _fields_ = [("nstr", ctypes.c_int), ("nmom", ctypes.c_int), ("nlyr", ctypes.c_int),
                ("nprop", ctypes.c_int), ("flags", ctypes.c_uint)]


class HdInputs(ctypes.Structure):
    _fields_ = [("nwave", ctypes.c_int), ("ncol", ctypes.c_int), ("prop", _dp),
                ("fbeam", _dp), ("umu0", _dp), ("albedo", _dp), ("btemp", _dp),
                ("ttemp", _dp), ("temis", _dp), ("fisot", _dp), ("temf", _dp),
                ("wave_lower", _dp), ("wave_upper", _dp)]


class HdRadiance(ctypes.Structure):
    _fields_ = [("ntau", ctypes.c_int), ("utau", _dp), ("numu", ctypes.c_int), ("umu", _dp),
                ("nphi", ctypes.c_int), ("phi", _dp), ("phi0", _dp), ("onlyfl", ctypes.c_int),
                ("corint", ctypes.c_int)]


class HdBand(ctypes.Structure):
    _fields_ = [("weight", _dp), ("bflux", _dp)]


class HdTiming(ctypes.Structure):
    _fields_ = [("layer_ms", ctypes.c_double), ("sweep_ms", ctypes.c_double),
                ("layer_launches", ctypes.c_int), ("sweep_launches", ctypes.c_int)]


_lib = None


def load(path: str = LIB_PATH):
    """Load libhdisort.so; raises OSError if it has not been built.

    HD_LIB_PATH overrides the path (A/B runs of kernel variants built
    out of tree by mb/build_variant.sh)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("HD_LIB_PATH", path)
    if not os.path.exists(path):
        raise OSError(f"pyharp_amd: {path} not found -- build it with "
                      "`python -m pyharp_amd._build` (hipcc, gfx950); there is no CPU fallback")
    lib = ctypes.CDLL(path)
    lib.hd_version.restype = ctypes.c_int
    lib.hd_last_error.restype = ctypes.c_char_p
    lib.hd_last_error.argtypes = [ctypes.c_void_p]
    lib.hd_context_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int]
    lib.hd_context_destroy.argtypes = [ctypes.c_void_p]
    lib.hd_context_set_chunk.argtypes = [ctypes.c_void_p, ctypes.c_long]
    lib.hd_context_set_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.hd_context_set_max_sweeps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.hd_context_get_timing.argtypes = [ctypes.c_void_p, ctypes.POINTER(HdTiming)]
    lib.hd_context_reserve.argtypes = [ctypes.c_void_p, ctypes.POINTER(HdConfig), ctypes.c_long]
    lib.hd_chunk_solves.restype = ctypes.c_long
    lib.hd_chunk_solves.argtypes = [ctypes.POINTER(HdConfig), ctypes.c_long]
    lib.hd_solve.argtypes = [ctypes.c_void_p, ctypes.POINTER(HdConfig), ctypes.POINTER(HdInputs),
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.hd_solve_band.argtypes = [ctypes.c_void_p, ctypes.POINTER(HdConfig),
                                  ctypes.POINTER(HdInputs), ctypes.POINTER(HdBand),
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.hd_solve_host.argtypes = [ctypes.c_void_p, ctypes.POINTER(HdConfig),
                                  ctypes.POINTER(HdInputs), ctypes.c_void_p, ctypes.c_void_p]
    lib.hd_solve_band_host.argtypes = [ctypes.c_void_p, ctypes.POINTER(HdConfig),
                                       ctypes.POINTER(HdInputs), ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.hd_solve_radiance.argtypes = [ctypes.c_void_p, ctypes.POINTER(HdConfig),
                                      ctypes.POINTER(HdInputs), ctypes.POINTER(HdRadiance),
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p]
    lib.hd_quadrature.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                  ctypes.POINTER(ctypes.c_double)]
    ci, cd = ctypes.c_int, ctypes.c_double
    lib.hd_attenuate.argtypes = [ctypes.POINTER(HdAttenuator), _dp, ci, ci, _dp, ci, ci, ci, _dp,
                                 _dp]
    lib.hd_band_optics.argtypes = [ctypes.POINTER(HdAttenuator), ci, _dp, ci, ci, _dp, ci, ci, ci,
                                   _dp, ci, _dp, _dp]
    lib.hd_band_loop_optics.argtypes = [ctypes.POINTER(HdBandAttenuator), ci, _dp, _dp, ci, ci,
                                        _dp, ci, ci, ci, _dp, ci, _dp, _dp]
    lib.hd_rfm_attenuate.argtypes = [ctypes.POINTER(HdRfmTable), _dp, ci, ci, ci, _dp, _dp, _dp,
                                     _dp]
    lib.hd_band_flux.argtypes = [_dp, _dp, ci, ci, ci, _dp, _dp]
    lib.hd_heating_rate.argtypes = [_dp, _dp, _dp, cd, ci, ci, _dp, _dp]
    lib.hd_spherical_flux_correction.argtypes = [_dp, _dp, _dp, _dp, ci, ci, _dp]
    lib.hd_nc_open.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p),
                               ctypes.POINTER(ctypes.c_int)]
    lib.hd_nc_close.argtypes = [ctypes.c_void_p]
    lib.hd_nc_dim_len.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_long)]
    lib.hd_nc_var_size.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_long)]
    lib.hd_nc_get_var_double.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p,
                                         ctypes.c_long]
    for name in EXPORTED + HARP_EXPORTED + NC_EXPORTED:
        getattr(lib, name)
    _lib = lib
    return lib


def last_error(ctx=None) -> str:
    msg = load().hd_last_error(ctx)
    return msg.decode() if msg else ""


def check(rc: int, ctx=None) -> None:
    if rc != HD_OK:
        kind = {HD_EINVAL: "invalid argument", HD_ENUMERIC: "numerical failure",
                HD_EHIP: "HIP error", HD_ENOMEM: "out of device memory"}.get(rc, f"code {rc}")
        raise RuntimeError(f"hdisort ({kind}): {last_error(ctx)}")


class Context:
    """One hd_context per device (scratch + status + timing events)."""

    def __init__(self, device: int = 0):
        lib = load()
        h = ctypes.c_void_p()
        check(lib.hd_context_create(ctypes.byref(h), int(device)))
        self.handle = h
        self.device = int(device)

    def close(self):
        if getattr(self, "handle", None):
            load().hd_context_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_chunk(self, n: int):
        check(load().hd_context_set_chunk(self.handle, int(n)), self.handle)

    def set_timing(self, on: bool):
        check(load().hd_context_set_timing(self.handle, int(bool(on))), self.handle)

    def reserve(self, cfg: HdConfig, nsolve: int):
        """hd_context_reserve: size scratch (hd_solve and hd_solve_band) and status."""
        check(load().hd_context_reserve(self.handle, ctypes.byref(cfg), int(nsolve)),
              self.handle)

    def set_max_sweeps(self, n: int):
        """Debug: cap the eigensolver's Jacobi sweeps (0 = default)."""
        check(load().hd_context_set_max_sweeps(self.handle, int(n)), self.handle)

    def timing(self) -> HdTiming:
        t = HdTiming()
        check(load().hd_context_get_timing(self.handle, ctypes.byref(t)), self.handle)
        return t

    def solve(self, cfg: HdConfig, inp: HdInputs, flux_ptr: int, status_ptr: int | None,
              stream_ptr: int | None):
        rc = load().hd_solve(self.handle, ctypes.byref(cfg), ctypes.byref(inp),
                             ctypes.c_void_p(flux_ptr), ctypes.c_void_p(status_ptr or 0),
                             ctypes.c_void_p(stream_ptr or 0))
        check(rc, self.handle)

    def solve_band(self, cfg: HdConfig, inp: HdInputs, band: HdBand, flux_ptr: int | None,
                   status_ptr: int | None, stream_ptr: int | None):
        rc = load().hd_solve_band(self.handle, ctypes.byref(cfg), ctypes.byref(inp),
                                  ctypes.byref(band), ctypes.c_void_p(flux_ptr or 0),
                                  ctypes.c_void_p(status_ptr or 0),
                                  ctypes.c_void_p(stream_ptr or 0))
        check(rc, self.handle)

    def solve_host(self, cfg: HdConfig, inp: HdInputs, flux_ptr: int):
        """hd_solve_host: every pointer a host address; synchronous."""
        check(load().hd_solve_host(self.handle, ctypes.byref(cfg), ctypes.byref(inp),
                                   ctypes.c_void_p(flux_ptr), None), self.handle)

    def solve_band_host(self, cfg: HdConfig, inp: HdInputs, weight_ptr: int, bflux_ptr: int,
                        flux_ptr: int | None):
        check(load().hd_solve_band_host(self.handle, ctypes.byref(cfg), ctypes.byref(inp),
                                        ctypes.c_void_p(weight_ptr), ctypes.c_void_p(bflux_ptr),
                                        ctypes.c_void_p(flux_ptr or 0), None), self.handle)

    def solve_radiance(self, cfg: HdConfig, inp: HdInputs, rad: HdRadiance, flux_ptr: int,
                       uu_ptr: int | None, status_ptr: int | None, stream_ptr: int | None):
        rc = load().hd_solve_radiance(self.handle, ctypes.byref(cfg), ctypes.byref(inp),
                                      ctypes.byref(rad), ctypes.c_void_p(flux_ptr),
                                      ctypes.c_void_p(uu_ptr or 0),
                                      ctypes.c_void_p(status_ptr or 0),
                                      ctypes.c_void_p(stream_ptr or 0))
        check(rc, self.handle)


def quadrature(nstr: int):
    nn = nstr // 2
    mu = (ctypes.c_double * nn)()
    w = (ctypes.c_double * nn)()
    check(load().hd_quadrature(int(nstr), mu, w))
    return list(mu), list(w)


def chunk_solves(nstr: int, nlyr: int, nsolve: int, planck: bool = False) -> int:
    """hd_chunk_solves: solves per internal chunk under the automatic chunking."""
    cfg = HdConfig(nstr=int(nstr), nmom=int(nstr), nlyr=int(nlyr), nprop=2 + int(nstr),
                   flags=HD_FLAG_LAMBER | HD_FLAG_ONLYFL | (HD_FLAG_PLANCK if planck else 0))
    n = load().hd_chunk_solves(ctypes.byref(cfg), int(nsolve))
    if n < 0:
        raise RuntimeError(f"hd_chunk_solves: bad args (nstr={nstr}, nlyr={nlyr}, nsolve={nsolve})")
    return n
