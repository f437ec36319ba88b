"""Drop-in DISORT flux module (pydisort ``disort::Disort`` contract) on MI355X.

Mirrors the API pyharp uses at its call sites
(``examples/amars_sw.cpp:43-65,216,280``, ``examples/amars_lw.cpp:18-38,60,80``,
``tests/test_disort.cpp:13-55``, ``src/radiation/radiation_band.cpp:57-69,123-128``)::

    op = DisortOptions().header("...").flags("lamber,quiet,onlyfl")
    op.nwave(500).ncol(1)
    op.ds().nlyr = 40; op.ds().nstr = 8; op.ds().nmom = 8
    disort = Disort(op)
    flux = disort.forward(prop, bc)            # or forward(prop, bc, temf)

``prop`` (nwave, ncol, nlyr, nprop) f64, layer 0 = bottom; ``bc`` dict of
(nwave, ncol) tensors; ``temf`` (ncol, nlyr+1) level temperatures bottom->top.
Returns ``flux`` (nwave, ncol, nlyr+1, 2): level 0 = surface, [...,0] upward,
[...,1] downward (rfldir + rfldn).  CPU tensors are staged through the GPU and
the result is returned on the input's device; CUDA tensors stay on device.

Intensity path (``tests/test_disort.cpp:13-55``): without ``onlyfl`` the module
also computes radiances -- at ``user_mu`` x ``user_phi`` with ``usrang``, else at
the quadrature cosines and ``user_phi`` (default [0]) -- at ``user_tau`` with
``usrtau`` (else at the level depths); ``get_rad()`` returns them as
(nwave, ncol, nphi, ntau, numu).  With ``usrtau`` the fluxes are at the user
depths, (nwave, ncol, ntau, 2), index 0 = the deepest.  Every nstr 2..32.

The arithmetic runs in libhdisort.so (HIP, gfx950) through the C-ABI in
include/hdisort.h.  There is no CPU fallback: without a HIP device or without
the built library, ``forward`` raises.
"""

from __future__ import annotations

import threading
from typing import Dict, Optional

import torch

from . import _lib
from .index import IEX, ISS, IPM  # noqa: F401  (re-exported like disort::index)
from .rtsolver import RTSolver

# cdisort's disort_flag fields as pydisort's flag string names them (the Disort-flags
# block of examples/amarsw-ck.yaml:74-90, tests/test_disort.cpp:16-18)
_KNOWN_FLAGS = {
    "lamber", "quiet", "onlyfl", "planck", "usrtau", "usrang", "intensity_correction",
    "old_intensity_correction", "print-input", "print-fluxes", "print-intensity",
    "print-transmissivity", "print-phase-function", "ibcnd", "spher", "general_source",
    "output_uum",
}
# cdisort flags this solver does not implement: rejected, never silently ignored
_UNSUPPORTED_FLAGS = {
    "spher": "pseudo-spherical geometry is not implemented",
    "general_source": "general (user-supplied) sources are not implemented",
    "output_uum": "per-mode intensities (uum) are not output",
}


def check_flags(flags: set) -> None:
    """The flag semantics of the boundary, shared by reset():
    unknown names raise; ``ibcnd`` raises as harp's DISORT driver does
    (rt_solver_disort.cpp_:67-68, ``ValueError("RTSolverDisort::CalRadtranFlux",
    "ibcnd", ds_.flag.ibcnd, 0)``: the albedo/transmissivity mode of cdisort is not
    harp's); cdisort's new (Buras-Emde-Dowling) intensity correction --
    ``intensity_correction`` without ``old_intensity_correction`` -- raises when
    radiances are requested (with ``onlyfl`` cdisort applies no correction, so the
    flag has no effect there, as in examples/amarsw-ck.yaml:79-82)."""
    unknown = flags - _KNOWN_FLAGS
    if unknown:
        raise RuntimeError(f"Disort: unknown flags {sorted(unknown)}")
    if "ibcnd" in flags:
        raise RuntimeError("RTSolverDisort::CalRadtranFlux: ibcnd = 1, expected 0 (the "
                           "special-case albedo/transmissivity mode is not supported)")
    for f in sorted(flags & set(_UNSUPPORTED_FLAGS)):
        raise RuntimeError(f"Disort: flag '{f}': {_UNSUPPORTED_FLAGS[f]}")
    if ("intensity_correction" in flags and "old_intensity_correction" not in flags
            and "onlyfl" not in flags):
        raise RuntimeError("Disort: intensity_correction without old_intensity_correction "
                           "selects cdisort's new (Buras-Emde-Dowling) correction, which is "
                           "not implemented; add old_intensity_correction for the "
                           "Nakajima-Tanaka correction (TMS + IMS) or use onlyfl")
_BC_KEYS = ("fbeam", "umu0", "albedo", "btemp", "ttemp", "temis", "fisot")
_BC_IGNORED = ("phi0",)  # azimuth of the beam: used by the radiances only


def night_side_beam(bc: Dict[str, torch.Tensor], mode: str = "dark",
                    umu0_min: float = 1.0e-3) -> Dict[str, torch.Tensor]:
    """Boundary conditions a GCM-style caller can pass for a whole globe.

    The solver takes umu0 as given, as pydisort's forward hands it to cdisort, whose
    input check (c_chekin) rejects a beam (fbeam > 0) with umu0 outside (0, 1]: such a
    solve is flagged HD_STATUS_BAD_INPUT and a synchronous call fails.  A caller that
    passes one fbeam with cos(zenith) over day and night side picks a convention here:

      mode="dark"  -- fbeam = 0 where umu0 <= 0 (no direct beam on the night side;
                      umu0 there is then not read);
      mode="clamp" -- umu0 = max(umu0, umu0_min) where fbeam > 0 (harp's legacy driver
                      floored umu0 at 1e-3 before calling cdisort,
                      src/rtsolver/rt_solver_disort.cpp_:80).

    Returns a new dict (the caller's tensors are not modified); umu0 > 1 stays an
    error in both modes."""
    if mode not in ("dark", "clamp"):
        raise ValueError(f"night_side_beam: mode must be 'dark' or 'clamp', got {mode!r}")
    out = dict(bc)
    if "fbeam" not in bc or "umu0" not in bc or bc["fbeam"] is None or bc["umu0"] is None:
        return out
    fb = torch.as_tensor(bc["fbeam"])
    mu = torch.as_tensor(bc["umu0"])
    if mode == "dark":
        fb, mu = torch.broadcast_tensors(fb, mu)
        out["fbeam"] = torch.where(mu > 0.0, fb, torch.zeros_like(fb))
    else:
        fb, mu = torch.broadcast_tensors(fb, mu)
        out["umu0"] = torch.where(fb > 0.0, torch.clamp(mu, min=umu0_min), mu)
    return out


def _beam_hint(bc) -> str:
    """After a failed synchronous call: name the beam inputs cdisort's c_chekin rejects."""
    try:
        if not bc or bc.get("fbeam") is None or bc.get("umu0") is None:
            return ""
        fb, mu = torch.broadcast_tensors(torch.as_tensor(bc["fbeam"]), torch.as_tensor(bc["umu0"]))
        bad = int(((fb > 0.0) & ~((mu > 0.0) & (mu <= 1.0))).sum())
    except Exception:  # the hint must never mask the original error
        return ""
    if not bad:
        return ""
    return (f" -- {bad} solve(s) have fbeam > 0 with umu0 outside (0, 1], which cdisort's "
            "c_chekin rejects; for a day/night batch use "
            "pyharp_amd.night_side_beam(bc, mode='dark' or 'clamp')")


class _DisortState:
    """Subset of cdisort's disort_state exposed by ``DisortOptions.ds()``."""

    def __init__(self):
        self.nlyr = 1
        self.nstr = 4
        self.nmom = 4
        self.nphi = 0
        self.ntau = 0
        self.numu = 0
        self.utau = []

    def __repr__(self):
        return (f"disort_state(nlyr={self.nlyr}, nstr={self.nstr}, nmom={self.nmom}, "
                f"nphi={self.nphi}, ntau={self.ntau}, numu={self.numu})")


def _arg(name, default):
    """harp ADD_ARG idiom: obj.name(value) sets and returns obj; obj.name() reads."""

    def accessor(self, *value):
        if value:
            setattr(self, "_" + name, value[0])
            return self
        return getattr(self, "_" + name, default() if callable(default) else default)

    accessor.__name__ = name
    return accessor


class DisortOptions:
    header = _arg("header", "")
    flags = _arg("flags", "")
    nwave = _arg("nwave", 1)
    ncol = _arg("ncol", 1)
    wave_lower = _arg("wave_lower", list)
    wave_upper = _arg("wave_upper", list)
    user_tau = _arg("user_tau", list)
    user_mu = _arg("user_mu", list)
    user_phi = _arg("user_phi", list)
    device = _arg("device", 0)

    def __init__(self):
        self._ds = _DisortState()

    def ds(self) -> _DisortState:
        return self._ds

    def flag_set(self) -> set:
        return {f.strip() for f in self.flags().split(",") if f.strip()}

    def __repr__(self):
        return (f"DisortOptions(flags='{self.flags()}', nwave={self.nwave()}, "
                f"ncol={self.ncol()}, ds={self._ds})")


_THREAD = threading.local()


def _context(device: int) -> _lib.Context:
    """The calling host thread's hd_context on ``device`` (SURVEY 8(b) "Threading":
    one context per (device, host thread)).  Modules of one thread share it; the
    library orders their solves on any streams behind each other (hd_solve waits
    for the context's previous solve), so scratch is never used twice at once."""
    ctxs = getattr(_THREAD, "contexts", None)
    if ctxs is None:
        ctxs = _THREAD.contexts = {}
    ctx = ctxs.get(device)
    if ctx is None:
        ctx = _lib.Context(device)
        ctxs[device] = ctx
    return ctx


class Disort(RTSolver):
    """MI355X flux-only DISORT module (drop-in for pydisort's DisortImpl)."""

    def __init__(self, options: Optional[DisortOptions] = None):
        self.options = options if options is not None else DisortOptions()
        self._waves = None
        self.reset()

    def reset(self):
        op = self.options
        flags = op.flag_set()
        check_flags(flags)
        ds = op.ds()
        if ds.nstr < 2 or ds.nstr % 2 or ds.nstr > 32:
            raise RuntimeError(f"Disort: nstr={ds.nstr} must be even and in [2, 32]")
        if ds.nlyr < 1:
            raise RuntimeError(f"Disort: nlyr={ds.nlyr} must be >= 1")
        if "lamber" not in flags:
            raise RuntimeError("Disort: only Lambertian lower boundaries are supported "
                               "(set the 'lamber' flag)")
        self.planck = "planck" in flags
        if self.planck:
            if len(op.wave_lower()) != op.nwave() or len(op.wave_upper()) != op.nwave():
                raise RuntimeError("Disort: planck needs wave_lower/wave_upper of size nwave")
        # intensity path: radiances (onlyfl off) and/or fluxes at user depths
        self.onlyfl = "onlyfl" in flags
        self.usrtau = "usrtau" in flags
        self.usrang = "usrang" in flags
        self.radiance = (not self.onlyfl) or self.usrtau
        # Nakajima-Tanaka correction, TMS + IMS: cdisort applies it with both
        # intensity_correction and old_intensity_correction; old_intensity_correction
        # alone applies none (check_flags refuses the new method)
        self.corint = {"intensity_correction", "old_intensity_correction"} <= flags
        self._rad = None
        if self.radiance:
            if self.usrtau:
                ut = [float(x) for x in op.user_tau()]
                if not ut:
                    raise RuntimeError("Disort: usrtau set but user_tau is empty")
                if any(x < 0 for x in ut) or any(b < a for a, b in zip(ut, ut[1:])):
                    raise RuntimeError("Disort: user_tau must be >= 0 and ascending")
                ds.utau = ut
                ds.ntau = len(ut)
            else:
                ds.utau = []
                ds.ntau = ds.nlyr + 1
            if self.usrang:
                umu = [float(x) for x in op.user_mu()]
                if not umu or any(x == 0 or abs(x) > 1 for x in umu):
                    raise RuntimeError("Disort: usrang needs user_mu in [-1,0)U(0,1]")
            else:
                mu, _ = _lib.quadrature(ds.nstr) if _lib_loaded() else _gauss(ds.nstr)
                umu = [-x for x in reversed(mu)] + list(mu)
            phi = [float(x) for x in op.user_phi()] or [0.0]
            self._umu, self._phi = umu, phi
            ds.numu, ds.nphi = (len(umu), len(phi)) if not self.onlyfl else (0, 0)

    def ds(self):
        return self.options.ds()

    def get_rad(self, *args, **kwargs) -> torch.Tensor:
        """Radiances of the last forward, (nwave, ncol, nphi, ntau, numu)
        (pydisort DisortImpl::get_rad, tests/test_disort.cpp:52)."""
        if self.onlyfl:
            raise RuntimeError("Disort.get_rad: radiances are off (onlyfl flag)")
        if self._rad is None:
            raise RuntimeError("Disort.get_rad: call forward first")
        return self._rad

    # ------------------------------------------------------------------ #
    def forward(self, prop: torch.Tensor, bc: Optional[Dict[str, torch.Tensor]] = None,
                temf: Optional[torch.Tensor] = None, *, status: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
        try:
            return self._forward(prop, bc, temf, status=status, out=out)
        except RuntimeError as err:
            if "at least one solve failed" in str(err) and _beam_hint(bc):
                raise RuntimeError(str(err) + _beam_hint(bc)) from err
            raise

    def forward_band(self, prop: torch.Tensor, bc: Optional[Dict[str, torch.Tensor]] = None,
                     temf: Optional[torch.Tensor] = None, *, weights: torch.Tensor,
                     out: Optional[torch.Tensor] = None, flux: Optional[torch.Tensor] = None,
                     status: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The band flux (ncol, nlyr+1, 2) = sum_w weights[w] F_w of this batch, with
        the sum fused into the solve (hd_solve_band): what every harp caller does
        with forward's result next (examples/amars_lw.cpp:84-88
        ``(flux * weights.view({-1,1,1,1})).sum(0)``; amars_sw.cpp:169-196 with
        weights = d(wavenumber)).  Per-point fluxes are stored only if ``flux``
        (nwave, ncol, nlyr+1, 2) is given.  Fixed summation order, no atomics."""
        if self.radiance:
            raise RuntimeError("Disort.forward_band: the fused band sum is a flux-only path "
                               "(onlyfl without usrtau)")
        try:
            return self._forward(prop, bc, temf, status=status, out=flux, band=(weights, out))
        except RuntimeError as err:
            if "at least one solve failed" in str(err) and _beam_hint(bc):
                raise RuntimeError(str(err) + _beam_hint(bc)) from err
            raise

    def _forward(self, prop, bc, temf, *, status=None, out=None, band=None):
        op = self.options
        ds = op.ds()
        bc = {} if bc is None else bc
        if prop.dim() != 4:
            raise RuntimeError(f"Disort.forward: prop must be (nwave, ncol, nlyr, nprop), got "
                               f"{tuple(prop.shape)}")
        nwave, ncol, nlyr, nprop = prop.shape
        if nlyr != ds.nlyr:
            raise RuntimeError(f"Disort.forward: prop has {nlyr} layers, ds().nlyr = {ds.nlyr}")
        for k in bc:
            if k not in _BC_KEYS and k not in _BC_IGNORED:
                raise RuntimeError(f"Disort.forward: unknown boundary condition '{k}'")
        if self.planck and temf is None:
            raise RuntimeError("Disort.forward: planck flag set but temf not given")
        if self.planck and not (nwave == len(op.wave_lower()) == len(op.wave_upper())):
            # the kernels read wave_lower/upper[w] for every w < prop.shape[0]
            raise RuntimeError(f"Disort.forward: planck: prop has {nwave} waves but "
                               f"wave_lower/wave_upper hold {len(op.wave_lower())}/"
                               f"{len(op.wave_upper())}")
        if not torch.cuda.is_available():
            raise RuntimeError("Disort.forward: no HIP device available (pyharp_amd has no "
                               "CPU path)")
        in_dev = prop.device
        dev = in_dev if in_dev.type == "cuda" else torch.device("cuda", int(op.device()))
        f64 = torch.float64
        if in_dev.type != "cuda" and not self.radiance and out is None and status is None:
            # pydisort's CPU-tensor contract: the library's host-array entry points
            # (hd_solve_host / hd_solve_band_host) copy the arrays over in pieces
            # beside the solve of the previous piece
            return self._forward_host(prop, bc, temf, band, dev, nwave, ncol, nlyr, nprop)

        def dev_tensor(x, shape=None):
            if x is None:
                return None
            t = torch.as_tensor(x, dtype=f64)
            if shape is not None:
                t = t.expand(shape) if t.dim() < len(shape) or t.shape != shape else t
            return t.to(dev).contiguous()

        p = dev_tensor(prop)
        keep = [p]
        bct = {}
        for k in _BC_KEYS:
            if k in bc and bc[k] is not None:
                t = dev_tensor(bc[k], (nwave, ncol))
                if tuple(t.shape) != (nwave, ncol):
                    raise RuntimeError(f"Disort.forward: bc['{k}'] must be (nwave, ncol)")
                bct[k] = t
                keep.append(t)
        tf = wl = wu = None
        if self.planck:
            tf = dev_tensor(temf)
            if tuple(tf.shape) != (ncol, nlyr + 1):
                raise RuntimeError(f"Disort.forward: temf must be (ncol, nlyr+1) = "
                                   f"{(ncol, nlyr + 1)}, got {tuple(tf.shape)}")
            # cached per device: no host->device copy per call (keeps forward
            # capturable into a HIP graph once warmed up)
            key = (str(dev), tuple(op.wave_lower()), tuple(op.wave_upper()))
            if self._waves is None or self._waves[0] != key:
                self._waves = (key, torch.tensor(op.wave_lower(), dtype=f64, device=dev),
                               torch.tensor(op.wave_upper(), dtype=f64, device=dev))
            wl, wu = self._waves[1], self._waves[2]
            keep += [tf, wl, wu]
        nlev = ds.ntau if self.radiance else nlyr + 1
        if out is None:
            flux = None if band is not None else \
                torch.empty((nwave, ncol, nlev, 2), dtype=f64, device=dev)
        else:
            if (out.device != dev or out.dtype != f64 or not out.is_contiguous()
                    or tuple(out.shape) != (nwave, ncol, nlev, 2)):
                raise RuntimeError("Disort.forward: out must be a contiguous float64 tensor "
                                   f"of shape {(nwave, ncol, nlev, 2)} on {dev}")
            flux = out
        if status is not None and (status.device != dev or status.dtype != torch.int32
                                   or not status.is_contiguous()
                                   or status.numel() < nwave * ncol):
            raise RuntimeError(f"Disort.forward: status must be a contiguous int32 tensor of "
                               f">= {nwave * ncol} elements on {dev}")

        def ptr(t):
            return t.data_ptr() if t is not None else None

        cfg = _lib.HdConfig(nstr=ds.nstr, nmom=ds.nmom, nlyr=nlyr, nprop=nprop,
                            flags=_lib.HD_FLAG_LAMBER | _lib.HD_FLAG_ONLYFL |
                            (_lib.HD_FLAG_PLANCK if self.planck else 0))
        inp = _lib.HdInputs(nwave=nwave, ncol=ncol, prop=ptr(p),
                            fbeam=ptr(bct.get("fbeam")), umu0=ptr(bct.get("umu0")),
                            albedo=ptr(bct.get("albedo")), btemp=ptr(bct.get("btemp")),
                            ttemp=ptr(bct.get("ttemp")), temis=ptr(bct.get("temis")),
                            fisot=ptr(bct.get("fisot")), temf=ptr(tf), wave_lower=ptr(wl),
                            wave_upper=ptr(wu))
        stream = torch.cuda.current_stream(dev)
        if band is not None:
            wts = torch.as_tensor(band[0], dtype=f64).to(dev).reshape(-1).contiguous()
            if wts.numel() != nwave:
                raise RuntimeError(f"Disort.forward_band: {wts.numel()} weights for {nwave} "
                                   "waves")
            bout = band[1]
            if bout is None:
                bout = torch.empty((ncol, nlyr + 1, 2), dtype=f64, device=dev)
            elif (bout.device != dev or bout.dtype != f64 or not bout.is_contiguous()
                  or tuple(bout.shape) != (ncol, nlyr + 1, 2)):
                raise RuntimeError("Disort.forward_band: out must be a contiguous float64 "
                                   f"tensor of shape {(ncol, nlyr + 1, 2)} on {dev}")
            keep.append(wts)
            hb = _lib.HdBand(weight=wts.data_ptr(), bflux=bout.data_ptr())
            with torch.cuda.device(dev):
                _context(dev.index).solve_band(cfg, inp, hb, ptr(flux),
                                               status.data_ptr() if status is not None else None,
                                               stream.cuda_stream)
            del keep
            return bout.to(in_dev) if in_dev.type != "cuda" else bout
        if self.radiance:
            self._forward_radiance(cfg, inp, flux, status, stream, bc, dev, keep, nwave, ncol)
        else:
            with torch.cuda.device(dev):
                _context(dev.index).solve(cfg, inp, flux.data_ptr(),
                                          status.data_ptr() if status is not None else None,
                                          stream.cuda_stream)
        del keep
        if self._rad is not None and in_dev.type != "cuda":
            self._rad = self._rad.to(in_dev)
        if in_dev.type != "cuda":
            return flux.to(in_dev)
        return flux

    def _forward_host(self, prop, bc, temf, band, dev, nwave, ncol, nlyr, nprop):
        ds = self.options.ds()
        op = self.options
        f64 = torch.float64

        def host(x, shape=None):
            if x is None:
                return None
            t = torch.as_tensor(x, dtype=f64, device="cpu")
            if shape is not None and tuple(t.shape) != shape:
                t = t.expand(shape)
            return t.contiguous()

        keep = [host(prop)]
        bct = {}
        for k in _BC_KEYS:
            if k in bc and bc[k] is not None:
                t = host(bc[k], (nwave, ncol))
                if tuple(t.shape) != (nwave, ncol):
                    raise RuntimeError(f"Disort.forward: bc['{k}'] must be (nwave, ncol)")
                bct[k] = t
                keep.append(t)
        tf = wl = wu = None
        if self.planck:
            tf = host(temf)
            if tuple(tf.shape) != (ncol, nlyr + 1):
                raise RuntimeError(f"Disort.forward: temf must be (ncol, nlyr+1) = "
                                   f"{(ncol, nlyr + 1)}, got {tuple(tf.shape)}")
            wl = torch.tensor(op.wave_lower(), dtype=f64)
            wu = torch.tensor(op.wave_upper(), dtype=f64)
            keep += [tf, wl, wu]

        def ptr(t):
            return t.data_ptr() if t is not None else None

        cfg = _lib.HdConfig(nstr=ds.nstr, nmom=ds.nmom, nlyr=nlyr, nprop=nprop,
                            flags=_lib.HD_FLAG_LAMBER | _lib.HD_FLAG_ONLYFL |
                            (_lib.HD_FLAG_PLANCK if self.planck else 0))
        inp = _lib.HdInputs(nwave=nwave, ncol=ncol, prop=ptr(keep[0]),
                            fbeam=ptr(bct.get("fbeam")), umu0=ptr(bct.get("umu0")),
                            albedo=ptr(bct.get("albedo")), btemp=ptr(bct.get("btemp")),
                            ttemp=ptr(bct.get("ttemp")), temis=ptr(bct.get("temis")),
                            fisot=ptr(bct.get("fisot")), temf=ptr(tf), wave_lower=ptr(wl),
                            wave_upper=ptr(wu))
        ctx = _context(dev.index)
        if band is not None:
            wts = host(band[0]).reshape(-1).contiguous()
            if wts.numel() != nwave:
                raise RuntimeError(f"Disort.forward_band: {wts.numel()} weights for {nwave} "
                                   "waves")
            bout = torch.empty((ncol, nlyr + 1, 2), dtype=f64)
            with torch.cuda.device(dev):
                ctx.solve_band_host(cfg, inp, wts.data_ptr(), bout.data_ptr(), None)
            if band[1] is not None:
                band[1].copy_(bout)
                return band[1]
            return bout
        flux = torch.empty((nwave, ncol, nlyr + 1, 2), dtype=f64)
        with torch.cuda.device(dev):
            ctx.solve_host(cfg, inp, flux.data_ptr())
        return flux

    def _forward_radiance(self, cfg, inp, flux, status, stream, bc, dev, keep, nwave, ncol):
        import ctypes
        ds = self.options.ds()
        f64 = torch.float64
        phi0 = None
        if bc.get("phi0") is not None:
            phi0 = torch.as_tensor(bc["phi0"], dtype=f64).expand((nwave, ncol)).to(dev)
            phi0 = phi0.contiguous()
            keep.append(phi0)
        arr = lambda xs: (ctypes.c_double * max(1, len(xs)))(*xs)  # noqa: E731
        ut, mu, ph = arr(ds.utau), arr(self._umu), arr(self._phi)
        rad = _lib.HdRadiance(ntau=len(ds.utau) if self.usrtau else 0,
                              utau=ctypes.cast(ut, ctypes.c_void_p),
                              numu=len(self._umu), umu=ctypes.cast(mu, ctypes.c_void_p),
                              nphi=len(self._phi), phi=ctypes.cast(ph, ctypes.c_void_p),
                              phi0=phi0.data_ptr() if phi0 is not None else None,
                              onlyfl=int(self.onlyfl), corint=int(self.corint))
        uu = None
        if not self.onlyfl:
            uu = torch.empty((nwave, ncol, len(self._phi), ds.ntau, len(self._umu)), dtype=f64,
                             device=dev)
        with torch.cuda.device(dev):
            _context(dev.index).solve_radiance(
                cfg, inp, rad, flux.data_ptr(), uu.data_ptr() if uu is not None else None,
                status.data_ptr() if status is not None else None, stream.cuda_stream)
        self._rad = uu


def _lib_loaded() -> bool:
    try:
        _lib.load()
        return True
    except OSError:
        return False


def _gauss(nstr):
    import numpy as np
    x, w = np.polynomial.legendre.leggauss(nstr // 2)
    return list(0.5 * (x + 1.0)), list(0.5 * w)
