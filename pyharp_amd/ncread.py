"""Readers of the netCDF files the RFM attenuator and ``read_weights_rfm`` load
(``src/opacity/rfm.cpp:34-120``, ``src/utils/read_weights.cpp:18-46``: the
``nc_open / nc_inq_dimid / nc_inq_dimlen / nc_inq_varid / nc_get_var_double``
calls).  The netCDF library is not in this image; this is host-side file parsing:

* ``NetCDFClassic`` -- classic files (CDF-1, CDF-2 64-bit offset, CDF-5), pure
  Python (big-endian header + contiguous variables, per the classic format
  specification);
* ``NetCDF4`` -- netCDF-4 files (HDF5 containers, what rfm.cpp:39 opens with
  ``NC_NETCDF4``), through the C-ABI of ``include/hdnc.h`` over the HDF5-format
  walker of ``include/harp_amd/nc4read.hpp`` (in libhdisort.so);
* ``open_netcdf`` -- either, by the file's signature (as ``nc_open`` does).
"""

from __future__ import annotations

import struct
from typing import Dict, List, Tuple

import numpy as np

_NC_DIMENSION, _NC_VARIABLE, _NC_ATTRIBUTE = 0x0A, 0x0B, 0x0C
_TYPES = {1: (">i1", 1), 2: ("S1", 1), 3: (">i2", 2), 4: (">i4", 4), 5: (">f4", 4),
          6: (">f8", 8), 7: (">u1", 1), 8: (">u2", 2), 9: (">u4", 4), 10: (">i8", 8),
          11: (">u8", 8)}


class NetCDFClassic:
    """Parsed header of a classic netCDF file; variables read on demand."""

    def __init__(self, path: str):
        self.path = path
        with open(path, "rb") as f:
            head = f.read(8)
            if head[:4] == b"\x89HDF":
                raise RuntimeError(f"{path}: netCDF-4/HDF5 file; NetCDFClassic takes classic "
                                   "netCDF only (open_netcdf / NetCDF4 read it)")
            if head[:3] != b"CDF" or head[3] not in (1, 2, 5):
                raise RuntimeError(f"{path}: not a netCDF classic file")
            self.version = head[3]
            f.seek(0)
            self._buf = f.read()
        self._pos = 4
        self._nn = 8 if self.version == 5 else 4          # NON_NEG width
        self._off = 4 if self.version == 1 else 8         # OFFSET width
        self.numrecs = self._nonneg()
        self.dims: List[Tuple[str, int]] = self._dim_list()
        self.gatts = self._att_list()
        self.vars: Dict[str, dict] = {}
        self._var_list()
        rec = [v for v in self.vars.values() if v["record"]]
        self.recsize = sum(v["vsize"] for v in rec) if len(rec) > 1 else \
            (rec[0]["vsize"] if rec else 0)

    # ---- header primitives -------------------------------------------------
    def _u(self, fmt, n):
        v = struct.unpack_from(fmt, self._buf, self._pos)[0]
        self._pos += n
        return v

    def _nonneg(self):
        return self._u(">Q", 8) if self._nn == 8 else self._u(">I", 4)

    def _name(self):
        n = self._nonneg()
        s = self._buf[self._pos:self._pos + n].decode("utf-8")
        self._pos += (n + 3) & ~3
        return s

    def _tag_list(self, tag):
        t = self._u(">I", 4)
        n = self._nonneg()
        if t == 0 and n == 0:
            return 0
        if t != tag:
            raise RuntimeError(f"{self.path}: corrupt header (tag {t:#x})")
        return n

    def _dim_list(self):
        return [(self._name(), self._nonneg()) for _ in range(self._tag_list(_NC_DIMENSION))]

    def _att_list(self):
        atts = {}
        for _ in range(self._tag_list(_NC_ATTRIBUTE)):
            name = self._name()
            typ = self._u(">I", 4)
            n = self._nonneg()
            dt, sz = _TYPES[typ]
            raw = self._buf[self._pos:self._pos + n * sz]
            self._pos += (n * sz + 3) & ~3
            atts[name] = raw.decode("utf-8", "replace") if typ == 2 else \
                np.frombuffer(raw, dtype=dt).copy()
        return atts

    def _var_list(self):
        for _ in range(self._tag_list(_NC_VARIABLE)):
            name = self._name()
            nd = self._nonneg()
            dimids = [self._nonneg() for _ in range(nd)]
            atts = self._att_list()
            typ = self._u(">I", 4)
            vsize = self._nonneg()
            begin = self._u(">Q", 8) if self._off == 8 else self._u(">I", 4)
            shape = [self.dims[d][1] for d in dimids]
            record = bool(dimids) and self.dims[dimids[0]][1] == 0
            self.vars[name] = dict(dimids=dimids, shape=shape, type=typ, vsize=vsize,
                                   begin=begin, atts=atts, record=record)

    # ---- nc_inq_* / nc_get_var_double analogues -----------------------------
    def dim_len(self, name: str) -> int:
        for n, l in self.dims:
            if n == name:
                return self.numrecs if l == 0 else l
        raise RuntimeError(f"{self.path}: NetCDF: Invalid dimension ID or name ({name})")

    def var(self, name: str) -> np.ndarray:
        """nc_get_var_double: the whole variable as float64, C order."""
        if name not in self.vars:
            raise RuntimeError(f"{self.path}: NetCDF: Variable not found ({name})")
        v = self.vars[name]
        dt, sz = _TYPES[v["type"]]
        if v["type"] == 2:
            raise RuntimeError(f"{self.path}: variable {name} is a char array")
        if not v["record"]:
            count = int(np.prod(v["shape"])) if v["shape"] else 1
            a = np.frombuffer(self._buf, dtype=dt, count=count, offset=v["begin"])
            return a.astype(np.float64).reshape(v["shape"])
        per = int(np.prod(v["shape"][1:])) if len(v["shape"]) > 1 else 1
        rows = [np.frombuffer(self._buf, dtype=dt, count=per,
                              offset=v["begin"] + r * self.recsize)
                for r in range(self.numrecs)]
        return np.stack(rows).astype(np.float64).reshape([self.numrecs] + v["shape"][1:])


class NetCDF4:
    """A netCDF-4 (HDF5) file read through libhdisort.so's hdnc.h: ``dim_len`` is the
    extent of the dataset of that name (the coordinate variable or netCDF's
    dimension scale), ``var`` the whole variable as float64 in C order."""

    def __init__(self, path: str):
        import ctypes
        from . import _lib
        self.path = path
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        is4 = ctypes.c_int(0)
        _lib.check(self._lib.hd_nc_open(path.encode(), ctypes.byref(h), ctypes.byref(is4)))
        self._h = h
        if not is4.value:
            self.close()
            raise RuntimeError(f"{path}: not a netCDF-4/HDF5 file (use NetCDFClassic)")

    def close(self):
        if getattr(self, "_h", None):
            self._lib.hd_nc_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, name):
        from . import _lib
        if rc != _lib.HD_OK:
            msg = _lib.last_error()
            raise RuntimeError(msg or f"{self.path}: {name}")

    def dim_len(self, name: str) -> int:
        import ctypes
        n = ctypes.c_long(0)
        self._check(self._lib.hd_nc_dim_len(self._h, name.encode(), ctypes.byref(n)), name)
        return int(n.value)

    def var(self, name: str) -> np.ndarray:
        """nc_get_var_double: the whole variable as float64, C order (flat when the
        file's shape is not needed; see ``shape``)."""
        import ctypes
        n = ctypes.c_long(0)
        self._check(self._lib.hd_nc_var_size(self._h, name.encode(), ctypes.byref(n)), name)
        out = np.empty(int(n.value), dtype=np.float64)
        self._check(self._lib.hd_nc_get_var_double(
            self._h, name.encode(), out.ctypes.data_as(ctypes.c_void_p), n), name)
        return out


def open_netcdf(path: str):
    """nc_open: NetCDF4 for an HDF5 container, else NetCDFClassic."""
    with open(path, "rb") as f:
        head = f.read(8)
    if head == b"\x89HDF\r\n\x1a\n":
        return NetCDF4(path)
    return NetCDFClassic(path)
