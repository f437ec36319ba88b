"""Table-driven attenuators on the device (the optics step before the solve).

Mirrors the two attenuators pyharp's SW example builds its optics from
(examples/amars_sw.cpp:221-271):

* ``AttenuatorOptions``  -- src/opacity/attenuator_options.hpp:8-19 (fluent
  setters, as ADD_ARG generates them);
* ``S8Fuller`` / ``H2SO4Simple`` -- src/opacity/s8_fuller.cpp,
  src/opacity/h2so4_simple.cpp: ``reset()`` reads the 3-column table
  (wavelength [um], k_ext [m^2/kg], ssa; '#' comments) and converts k_ext to
  m^2/mol with the species weight (:64-66); ``forward(conc, kwargs)`` returns
  (nwave, ncol, nlyr, 2) = (k c, ssa k c) [1/m] (:72-117), interpolated
  linearly in wavelength and clamped at the table ends (interpn.h, locate.h);
* ``band_optics`` -- the assembly amars_sw.cpp:261-271 performs by hand
  (sum of attenuators, x dz, ssa = sum ssa k c / sum k c), fused into one
  kernel that writes the solver's prop layout directly;
* ``band_loop_optics`` -- the library band loop's mixing
  (src/radiation/radiation_band.cpp:86-116: tau-weighted ssa, tau*ssa-weighted
  phase moments, the +1e-10 regularisation), with Henyey-Greenstein moments
  from an attenuator's asymmetry table (``set_asymmetry``), into the same layout.

The arithmetic runs in libhdisort.so (include/hdharp.h); tables are read on
the host (file parsing is not on the device path).  There is no CPU compute
path: forward() on a machine without a HIP device raises.
"""

from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib

_SEARCH_PATHS: List[str] = ["."]


def add_resource_directory(d: str) -> None:
    """Prepend a search directory (src/utils/find_resource.cpp add_resource_directory)."""
    d = os.path.expanduser(d)
    if d in _SEARCH_PATHS:
        _SEARCH_PATHS.remove(d)
    _SEARCH_PATHS.insert(0, d)


def find_resource(name: str) -> str:
    """Path of a data file: as given, then the search directories, then
    $HARP_RESOURCE_PATH (os.pathsep-separated) -- src/utils/find_resource.cpp."""
    if os.path.isabs(name) and os.path.exists(name):
        return name
    dirs = list(_SEARCH_PATHS)
    env = os.environ.get("HARP_RESOURCE_PATH")
    if env:
        dirs += [p for p in env.split(os.pathsep) if p]
    for d in dirs:
        p = os.path.join(d, name)
        if os.path.exists(p):
            return os.path.abspath(p)
    raise RuntimeError(f"find_resource: cannot find '{name}' in {dirs}")


def read_table(path: str) -> np.ndarray:
    """Decommented whitespace table (src/utils/fileio.cpp decomment_file)."""
    rows = []
    with open(path) as f:
        for line in f:
            line = line.split("#", 1)[0].strip()
            if line:
                rows.append([float(x) for x in line.split()])
    if not rows:
        raise RuntimeError(f"Empty file: {path}")
    t = np.asarray(rows, dtype=np.float64)
    return t


class AttenuatorOptions:
    """src/opacity/attenuator_options.hpp:8-19."""

    def __init__(self):
        self._type = ""
        self._opacity_files: List[str] = []
        self._species_ids: List[int] = [0]
        self._species_names: List[str] = []
        self._species_weights: List[float] = []

    def _get_set(name):  # noqa: N805
        def f(self, *v):
            if not v:
                return getattr(self, name)
            val = v[0]
            setattr(self, name, list(val) if isinstance(val, (list, tuple)) else val)
            return self
        return f

    type = _get_set("_type")
    opacity_files = _get_set("_opacity_files")
    species_ids = _get_set("_species_ids")
    species_names = _get_set("_species_names")
    species_weights = _get_set("_species_weights")
    del _get_set

    def copy(self) -> "AttenuatorOptions":
        o = AttenuatorOptions()
        o._type, o._opacity_files = self._type, list(self._opacity_files)
        o._species_ids, o._species_names = list(self._species_ids), list(self._species_names)
        o._species_weights = list(self._species_weights)
        return o


def _coord(kwargs: Dict[str, torch.Tensor]):
    if "wavelength" in kwargs:
        return kwargs["wavelength"], _lib.HD_COORD_WAVELENGTH
    if "wavenumber" in kwargs:
        return kwargs["wavenumber"], _lib.HD_COORD_WAVENUMBER
    raise RuntimeError("wavelength or wavenumber is required in kwargs")


def _device(*ts) -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("pyharp_amd.opacity: no HIP device available (no CPU path)")
    for t in ts:
        if isinstance(t, torch.Tensor) and t.device.type == "cuda":
            return t.device
    return torch.device("cuda", torch.cuda.current_device())


def _f64(x, dev) -> torch.Tensor:
    return torch.as_tensor(x, dtype=torch.float64).to(dev).contiguous()


class _TableAttenuator:
    """Common body of S8FullerImpl / H2SO4SimpleImpl (identical but for the type)."""

    TYPE = ""

    def __init__(self, options: AttenuatorOptions):
        self.options = options.copy()
        op = self.options
        if len(op.opacity_files()) != 1:
            raise RuntimeError("Only one opacity file is allowed")
        if len(op.species_ids()) != 1:
            raise RuntimeError("Only one species is allowed")
        if op.species_ids()[0] < 0:
            raise RuntimeError(f"Invalid species_id: {op.species_ids()[0]}")
        if op.type() and op.type() != self.TYPE:
            raise RuntimeError(f"Mismatch type: {op.type()}")
        self.reset()

    def reset(self):
        path = find_resource(self.options.opacity_files()[0])
        t = read_table(path)
        if t.ndim != 2 or t.shape[1] != 3:
            raise RuntimeError(f"Invalid file: {path}")
        sid = self.options.species_ids()[0]
        w = self.options.species_weights()
        if sid >= len(w):
            raise RuntimeError(f"species_weights has no entry for species {sid}")
        self.kwave = torch.as_tensor(t[:, 0].copy())              # [um]
        self.kdata = torch.as_tensor(t[:, 1:].copy())             # (rows, 2)
        self.kdata[:, 0] *= w[sid]                                # m^2/kg -> m^2/mol
        self.gasym = None                                         # HG asymmetry per row
        self._dev_tables = {}

    def set_asymmetry(self, g) -> "_TableAttenuator":
        """Henyey-Greenstein asymmetry g(lambda) per table row (scalar: every row),
        the phase moments chi_l = g^l this attenuator brings to band_loop_optics
        (the reference's tables carry none: data/*.txt hold k_ext and ssa only)."""
        g = np.broadcast_to(np.asarray(g, np.float64), (self.kwave.numel(),)).copy()
        if not np.all(np.abs(g) < 1.0):
            raise RuntimeError("set_asymmetry: |g| must be < 1")
        self.gasym = torch.as_tensor(g)
        self._dev_tables = {}
        return self

    def _tables(self, dev):
        key = str(dev)
        if key not in self._dev_tables:
            self._dev_tables[key] = (_f64(self.kwave, dev), _f64(self.kdata[:, 0], dev),
                                     _f64(self.kdata[:, 1], dev),
                                     None if self.gasym is None else _f64(self.gasym, dev))
        return self._dev_tables[key]

    def hd_struct(self, dev) -> _lib.HdAttenuator:
        wl, k, s, _ = self._tables(dev)
        return _lib.HdAttenuator(nrow=int(wl.numel()), wavelength=wl.data_ptr(),
                                 kext=k.data_ptr(), ssa=s.data_ptr(),
                                 species=int(self.options.species_ids()[0]))

    def forward(self, conc: torch.Tensor, kwargs: Dict[str, torch.Tensor]) -> torch.Tensor:
        coord, kind = _coord(kwargs)
        dev = _device(conc, coord)
        c = _f64(conc, dev)
        if c.dim() != 3:
            raise RuntimeError("conc must be (ncol, nlyr, nspecies)")
        x = _f64(coord, dev).reshape(-1)
        ncol, nlyr, nsp = c.shape
        out = torch.empty((x.numel(), ncol, nlyr, 2), dtype=torch.float64, device=dev)
        att = self.hd_struct(dev)
        lib = _lib.load()
        with torch.cuda.device(dev):
            _lib.check(lib.hd_attenuate(ctypes.byref(att), x.data_ptr(), kind, x.numel(),
                                        c.data_ptr(), ncol, nlyr, nsp, out.data_ptr(),
                                        torch.cuda.current_stream(dev).cuda_stream))
        return out if conc.device.type == "cuda" else out.to(conc.device)

    __call__ = forward


class S8Fuller(_TableAttenuator):
    """S8 aerosol, Fuller et al. optical constants (src/opacity/s8_fuller.cpp)."""
    TYPE = "s8_fuller"


class H2SO4Simple(_TableAttenuator):
    """H2SO4 aerosol (src/opacity/h2so4_simple.cpp)."""
    TYPE = "h2so4_simple"


def _check_out(name, out, shape, dev):
    """A caller-supplied ``out`` is written through its data pointer by the kernel:
    it must be exactly the contiguous float64 device tensor the kernel assumes."""
    if (tuple(out.shape) != tuple(shape) or out.dtype != torch.float64
            or out.device != dev or not out.is_contiguous()):
        raise RuntimeError(f"{name}: out must be a contiguous float64 tensor of shape "
                           f"{tuple(shape)} on {dev}, got {tuple(out.shape)} {out.dtype} "
                           f"on {out.device}")


def band_optics(attenuators: Sequence[_TableAttenuator], conc: torch.Tensor, dz: torch.Tensor,
                kwargs: Dict[str, torch.Tensor], nprop: int = 2,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """prop (nwave, ncol, nlyr, nprop) for Disort.forward: tau = dz sum_a k_a c_a,
    ssa = sum_a ssa_a k_a c_a / sum_a k_a c_a, moments 0 -- the amars_sw
    assembly (``prop = s8(conc) + h2so4(conc); prop *= dz; prop[...,1] /= prop[...,0]``,
    examples/amars_sw.cpp:261-271) in one kernel.  dz: (nlyr,), (nlyr, 1) or
    (ncol, nlyr) [m].  Layers without extinction get ssa = 0 (the reference's
    0/0 would be NaN)."""
    coord, kind = _coord(kwargs)
    dev = _device(conc, coord, dz)
    c = _f64(conc, dev)
    ncol, nlyr, nsp = c.shape
    d = torch.as_tensor(dz, dtype=torch.float64)
    if d.dim() == 2 and d.shape == (nlyr, 1):
        d = d[:, 0]
    d = _f64(d.expand(ncol, nlyr), dev)
    x = _f64(coord, dev).reshape(-1)
    nwave = x.numel()
    if out is None:
        out = torch.empty((nwave, ncol, nlyr, nprop), dtype=torch.float64, device=dev)
    _check_out("band_optics", out, (nwave, ncol, nlyr, nprop), dev)
    atts = (_lib.HdAttenuator * len(attenuators))(*[a.hd_struct(dev) for a in attenuators])
    lib = _lib.load()
    with torch.cuda.device(dev):
        _lib.check(lib.hd_band_optics(atts, len(attenuators), x.data_ptr(), kind, nwave,
                                      c.data_ptr(), ncol, nlyr, nsp, d.data_ptr(), nprop,
                                      out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream))
    return out


def band_loop_optics(attenuators: Sequence[_TableAttenuator], conc: torch.Tensor,
                     dz: torch.Tensor, kwargs: Dict[str, torch.Tensor], nmom: int,
                     ext0: Optional[torch.Tensor] = None,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """prop (nwave, ncol, nlyr, 2 + nmom) by RadiationBandImpl::forward's mixing
    (src/radiation/radiation_band.cpp:86-116), on the device (hd_band_loop_optics):
    ext = ext0 + sum_a k_a c_a, ssa = sum_a ssa_a k_a c_a / (ext + 1e-10), moments
    sum_a g_a^l ssa_a k_a c_a / (sum_a ssa_a k_a c_a + 1e-10) over the attenuators
    with an asymmetry table, tau = ext dz -- in the reference's operation order.
    ext0: (nwave, ncol, nlyr[, 1]) extinction of attenuators without ssa (an RFM
    module's forward), added first."""
    coord, kind = _coord(kwargs)
    dev = _device(conc, coord, dz)
    c = _f64(conc, dev)
    ncol, nlyr, nsp = c.shape
    d = torch.as_tensor(dz, dtype=torch.float64)
    if d.dim() == 2 and d.shape == (nlyr, 1):
        d = d[:, 0]
    d = _f64(d.expand(ncol, nlyr), dev)
    x = _f64(coord, dev).reshape(-1)
    nwave = x.numel()
    e0 = None
    if ext0 is not None:
        e0 = _f64(ext0, dev)
        if e0.numel() != nwave * ncol * nlyr:
            raise RuntimeError(f"band_loop_optics: ext0 must hold {(nwave, ncol, nlyr)}")
    if out is None:
        out = torch.empty((nwave, ncol, nlyr, 2 + nmom), dtype=torch.float64, device=dev)
    _check_out("band_loop_optics", out, (nwave, ncol, nlyr, 2 + nmom), dev)
    structs = []
    for a in attenuators:
        g = a._tables(dev)[3]
        structs.append(_lib.HdBandAttenuator(table=a.hd_struct(dev),
                                             gasym=None if g is None else g.data_ptr()))
    atts = (_lib.HdBandAttenuator * len(structs))(*structs)
    lib = _lib.load()
    with torch.cuda.device(dev):
        _lib.check(lib.hd_band_loop_optics(atts, len(structs),
                                           None if e0 is None else e0.data_ptr(), x.data_ptr(),
                                           kind, nwave, c.data_ptr(), ncol, nlyr, nsp,
                                           d.data_ptr(), int(nmom), out.data_ptr(),
                                           torch.cuda.current_stream(dev).cuda_stream))
    return out


class RFM:
    """RFM absorption tables (harp::RFMImpl, src/opacity/rfm.hpp, rfm.cpp).

    ``reset()`` reads the table the way rfm.cpp:30-120 does -- dimensions
    ``Wavenumber``, ``Pressure``, ``TempGrid``; variables of the same names
    (pressure converted to ln p), the reference ``Temperature`` profile, and
    the absorption variable named after ``species_names[species_ids[0]]``
    (nwave, npres, ntemp) in ln(m^2/kmol) -- through the classic-netCDF reader
    (``pyharp_amd.ncread``: netCDF-4/HDF5 as rfm.cpp:39 opens them, or classic).  ``from_arrays``
    builds the same module from in-memory tables.  ``forward(conc, kwargs)``
    with ``kwargs["pres"]`` [Pa] and ``kwargs["temp"]`` [K] (ncol, nlyr) returns
    (nwave, ncol, nlyr, 1) = 1e-3 exp(k) conc [1/m], interpolated on the device
    (include/hdharp.h hd_rfm_attenuate).
    """

    IPR, ITM = 0, 1

    def __init__(self, options: Optional[AttenuatorOptions] = None):
        self.options = (options or AttenuatorOptions()).copy()
        op = self.options
        if options is None:
            return
        if len(op.opacity_files()) != 1:
            raise RuntimeError("Only one opacity file is allowed")
        if len(op.species_ids()) != 1:
            raise RuntimeError("Only one species is allowed")
        if op.species_ids()[0] < 0:
            raise RuntimeError(f"Invalid species_id: {op.species_ids()[0]}")
        if op.type() and op.type() != "rfm":
            raise RuntimeError(f"Mismatch type: {op.type()}")
        self.reset()

    @classmethod
    def from_arrays(cls, wave, pres, tgrid, tref, kdata, species: int = 0) -> "RFM":
        m = cls()
        m.options.species_ids([int(species)])
        m._set(np.asarray(wave, np.float64), np.log(np.asarray(pres, np.float64)),
               np.asarray(tgrid, np.float64), np.asarray(tref, np.float64),
               np.asarray(kdata, np.float64))
        return m

    def _set(self, wave, lnp, tgrid, tref, kdata):
        nw, npr, nt = len(wave), len(lnp), len(tgrid)
        if kdata.shape != (nw, npr, nt):
            raise RuntimeError(f"RFM: table shape {kdata.shape} != {(nw, npr, nt)}")
        if len(tref) != npr:
            raise RuntimeError("RFM: reference temperature must have one value per pressure")
        self.kshape = (nw, npr, nt)
        self.kaxis = torch.as_tensor(np.concatenate([wave, lnp, tgrid]))
        self.kdata = torch.as_tensor(np.ascontiguousarray(kdata))
        self.krefatm = torch.as_tensor(np.stack([lnp, tref]))
        self._dev_tables = {}

    def reset(self):
        from .ncread import open_netcdf
        path = find_resource(self.options.opacity_files()[0])
        nc = open_netcdf(path)  # rfm.cpp:39 nc_open(..., NC_NETCDF4, ...); classic too
        nw, npr, nt = (nc.dim_len("Wavenumber"), nc.dim_len("Pressure"),
                       nc.dim_len("TempGrid"))
        name = self.options.species_names()[self.options.species_ids()[0]]
        kd = nc.var(name).reshape(nw, npr, nt)
        self._set(nc.var("Wavenumber").reshape(nw), np.log(nc.var("Pressure").reshape(npr)),
                  nc.var("TempGrid").reshape(nt), nc.var("Temperature").reshape(npr), kd)

    def _tables(self, dev):
        key = str(dev)
        if key not in self._dev_tables:
            nw, npr, nt = self.kshape
            ax = _f64(self.kaxis, dev)
            self._dev_tables[key] = (ax, _f64(self.krefatm[self.ITM], dev), _f64(self.kdata, dev))
        return self._dev_tables[key]

    def hd_struct(self, dev) -> _lib.HdRfmTable:
        nw, npr, nt = self.kshape
        ax, tref, kd = self._tables(dev)
        p = ax.data_ptr()
        return _lib.HdRfmTable(nwave=nw, npres=npr, ntemp=nt, wave=p, lnp=p + 8 * nw,
                               tgrid=p + 8 * (nw + npr), tref=tref.data_ptr(),
                               kdata=kd.data_ptr(), species=int(self.options.species_ids()[0]))

    def forward(self, conc: torch.Tensor, kwargs: Dict[str, torch.Tensor]) -> torch.Tensor:
        if "pres" not in kwargs:
            raise RuntimeError("pres is required in kwargs")
        if "temp" not in kwargs:
            raise RuntimeError("temp is required in kwargs")
        dev = _device(conc, kwargs["pres"], kwargs["temp"])
        c = _f64(conc, dev)
        if c.dim() != 3:
            raise RuntimeError("conc must be (ncol, nlyr, nspecies)")
        ncol, nlyr, nsp = c.shape
        p = _f64(kwargs["pres"], dev).expand(ncol, nlyr).contiguous()
        t = _f64(kwargs["temp"], dev).expand(ncol, nlyr).contiguous()
        out = torch.empty((self.kshape[0], ncol, nlyr, 1), dtype=torch.float64, device=dev)
        tab = self.hd_struct(dev)
        lib = _lib.load()
        with torch.cuda.device(dev):
            _lib.check(lib.hd_rfm_attenuate(ctypes.byref(tab), c.data_ptr(), ncol, nlyr, nsp,
                                            p.data_ptr(), t.data_ptr(), out.data_ptr(),
                                            torch.cuda.current_stream(dev).cuda_stream))
        return out if conc.device.type == "cuda" else out.to(conc.device)

    __call__ = forward


def read_weights_rfm(filename: str) -> torch.Tensor:
    """src/utils/read_weights.cpp:18-46: the ``weights`` variable of an RFM ck file."""
    from .ncread import open_netcdf
    nc = open_netcdf(find_resource(filename))
    n = nc.dim_len("weights")
    return torch.as_tensor(nc.var("weights").reshape(n).copy())
