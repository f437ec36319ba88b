"""netCDF-4 (HDF5) reader: include/harp_amd/nc4read.hpp, through the C++ checker
(g++) and through libhdisort.so's hdnc.h from Python (pyharp_amd.ncread), and
the RFM / read_weights_rfm loading of netCDF-4 tables (src/opacity/rfm.cpp:34-120
opens them with nc_open(..., NC_NETCDF4, ...); src/utils/read_weights.cpp:18-46).

The fixtures under tests/golden/nc4/ were written by tests/golden/nc4/make_nc4.c
with the HDF5 library in this image (libhdf5 1.10.6, /opt/conda) -- the real
HDF5 encoder, following the netCDF-4 conventions (creation-order-indexed links,
dimension scales, _Netcdf4Dimid, _NCProperties) -- so the reader is pinned to
the file format as libhdf5 lays it out: superblocks v0 and v3, v1/v2 object
headers, symbol-table, compact and dense (fractal heap, v2 B-tree of depth 0
and 1) groups, contiguous / compact / chunked (v1 B-tree, fixed array, single
chunk, implicit) storage, shuffle + deflate, f32 / f64 / i32, both byte orders.
Values: v(var, i) = sin(0.37 i + var) 10^((i mod 7) - 3) + var (make_nc4.c).
"""

import math
import os
import subprocess

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "nc4")
NW, NP, NT = 37, 11, 5
FILES = ["rfm_nc4.nc", "rfm_nc4_dense.nc", "rfm_nc4_many.nc", "rfm_latest.nc", "rfm_v0.nc"]
VARS = {"Wavenumber": (1, (NW,), "f8"), "Pressure": (2, (NP,), "f8"),
        "TempGrid": (3, (NT,), "f8"), "Temperature": (4, (NP,), "f8"),
        "CO2": (5, (NW, NP, NT), "f8"), "H2O": (6, (NW, NP, NT), "f4"),
        "O3": (7, (NW, NP, NT), "f8")}
EXTRA = {"rfm_nc4.nc": 0, "rfm_nc4_dense.nc": 10, "rfm_nc4_many.nc": 60, "rfm_latest.nc": 0,
         "rfm_v0.nc": 0}


def expected(var, shape, kind):
    n = int(np.prod(shape))
    # math.sin / math.pow: the C library's, as make_nc4.c computed them
    if var == 2:  # Pressure: positive and decreasing (RFM.reset takes its log)
        v = np.array([math.pow(10.0, 5.0 - 0.4 * i) * (1.0 + 0.05 * math.sin(0.37 * i + var))
                      for i in range(n)])
    else:
        v = np.array([math.sin(0.37 * i + var) * math.pow(10.0, (i % 7) - 3.0) + var
                      for i in range(n)])
    if kind == "f4":
        v = v.astype(np.float32).astype(np.float64)
    elif kind == "i4":
        v = np.trunc(v)
    return v.reshape(shape)


def all_vars(fname):
    out = dict(VARS)
    for x in range(EXTRA[fname]):
        out[f"X{x:02d}"] = (100 + x, (3 + x % 5,), "i4" if x % 2 else "f8")
    if fname == "rfm_latest.nc":
        out["N2O"] = (8, (NW, NP, NT), "f8")
    return out


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("nc4") / "ncread_check")
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "ncread_check.cpp"), "-o", exe, "-lz"],
                   check=True)
    return exe


def run_checker(exe, path, names):
    out = subprocess.run([exe, path] + names, capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    vals = {}
    for line in out.stdout.splitlines():
        parts = line.split()
        if parts[0].startswith("dim:"):
            vals[parts[0]] = int(parts[1])
        else:
            vals.setdefault(parts[0], []).append(float(parts[2]))
    return vals


@pytest.mark.parametrize("fname", FILES)
def test_cpp_reader_reads_every_variable(checker, fname):
    vs = all_vars(fname)
    got = run_checker(checker, os.path.join(FIX, fname),
                      ["dim:Wavenumber", "dim:Pressure", "dim:TempGrid"] + sorted(vs))
    assert (got["dim:Wavenumber"], got["dim:Pressure"], got["dim:TempGrid"]) == (NW, NP, NT)
    for name, (var, shape, kind) in vs.items():
        np.testing.assert_array_equal(np.array(got[name]).reshape(shape),
                                      expected(var, shape, kind), err_msg=f"{fname}:{name}")


@pytest.mark.parametrize("fname", FILES)
def test_python_reader_reads_every_variable(fname):
    from pyharp_amd.ncread import NetCDF4, open_netcdf
    nc = open_netcdf(os.path.join(FIX, fname))
    assert isinstance(nc, NetCDF4)
    assert [nc.dim_len(d) for d in ("Wavenumber", "Pressure", "TempGrid")] == [NW, NP, NT]
    for name, (var, shape, kind) in all_vars(fname).items():
        np.testing.assert_array_equal(nc.var(name).reshape(shape), expected(var, shape, kind),
                                      err_msg=f"{fname}:{name}")
    with pytest.raises(RuntimeError, match="not found"):
        nc.var("nope")
    with pytest.raises(RuntimeError, match="dimension"):
        nc.dim_len("nope")


def test_weights_file():
    from pyharp_amd.ncread import open_netcdf
    nc = open_netcdf(os.path.join(FIX, "weights_nc4.nc"))
    assert nc.dim_len("weights") == 16
    np.testing.assert_array_equal(nc.var("weights"), expected(9, (16,), "f8"))


def test_not_hdf5_and_truncated(tmp_path):
    from pyharp_amd.ncread import NetCDF4
    bad = tmp_path / "t.nc"
    data = open(os.path.join(FIX, "rfm_nc4.nc"), "rb").read()
    bad.write_bytes(data[:600])
    with pytest.raises(RuntimeError):
        NetCDF4(str(bad)).var("CO2")
    bad.write_bytes(b"CDF\x01" + b"\0" * 28)
    with pytest.raises(RuntimeError):
        NetCDF4(str(bad))


@pytest.mark.parametrize("fname", ["rfm_nc4.nc", "rfm_nc4_many.nc", "rfm_v0.nc"])
def test_rfm_reset_on_netcdf4_tables(tmp_path, fname):
    """RFM.reset and read_weights_rfm on a netCDF-4 table give exactly what they give
    on the same table written as classic netCDF (scipy)."""
    import shutil
    from scipy.io import netcdf_file
    from pyharp_amd.opacity import RFM, AttenuatorOptions, add_resource_directory
    d4 = tmp_path / "nc4"
    dc = tmp_path / "classic"
    d4.mkdir()
    dc.mkdir()
    shutil.copy(os.path.join(FIX, fname), d4 / "ck.nc")
    f = netcdf_file(str(dc / "ck.nc"), "w", version=2)
    for dname, n in (("Wavenumber", NW), ("Pressure", NP), ("TempGrid", NT)):
        f.createDimension(dname, n)
    for name, (var, shape, kind) in VARS.items():
        dims = {1: ("Wavenumber",), 2: ("Pressure",), 3: ("TempGrid",),
                4: ("Pressure",)}.get(var, ("Wavenumber", "Pressure", "TempGrid"))
        v = f.createVariable(name, "d", dims)
        v[:] = expected(var, shape, kind)
    f.close()
    tabs = {}
    for tag, d in (("nc4", d4), ("classic", dc)):
        add_resource_directory(str(d))
        op = AttenuatorOptions().species_names(["CO2", "H2O", "O3"]) \
            .species_weights([44e-3, 18e-3, 48e-3])
        tabs[tag] = [RFM(op.copy().species_ids([k]).opacity_files(["ck.nc"])) for k in range(3)]
    for a, b in zip(tabs["nc4"], tabs["classic"]):
        assert a.kshape == b.kshape == (NW, NP, NT)
        assert bool(torch.isfinite(a.kaxis).all())  # ln p of a positive pressure axis
        for attr in ("kdata", "kaxis", "krefatm"):
            np.testing.assert_array_equal(getattr(a, attr).numpy(), getattr(b, attr).numpy())


def test_read_weights_rfm_netcdf4(tmp_path):
    import shutil
    from pyharp_amd.opacity import add_resource_directory, read_weights_rfm
    shutil.copy(os.path.join(FIX, "weights_nc4.nc"), tmp_path / "w.nc")
    add_resource_directory(str(tmp_path))
    np.testing.assert_array_equal(read_weights_rfm("w.nc").numpy(), expected(9, (16,), "f8"))


@pytest.mark.parametrize("fname", ["rfm_nc4.nc", "rfm_nc4_dense.nc", "rfm_v0.nc"])
def test_corrupted_files_fail_cleanly(checker, tmp_path, fname):
    """Byte-corrupted fixtures (deterministic offsets across the superblock, object
    headers, B-trees, heaps and chunk data) either read or raise -- the reader's
    structural bounds (continuation-block and B-tree depth caps, chunk rank/zero
    checks, shuffle element size) keep a hostile file from crashing or hanging it."""
    data = bytearray(open(os.path.join(FIX, fname), "rb").read())
    rng = np.random.default_rng(len(data))
    offs = np.unique(np.concatenate([np.arange(0, min(len(data), 512), 7),
                                     rng.integers(0, len(data), 96)]))
    bad = tmp_path / "c.nc"
    for off in offs:
        for val in (0x00, 0xFF, data[off] ^ 0x5A):
            d = bytearray(data)
            d[off] = val
            bad.write_bytes(bytes(d))
            out = subprocess.run([checker, str(bad), "CO2", "dim:Pressure"], capture_output=True,
                                 text=True, timeout=20)
            assert out.returncode in (0, 2), (off, val, out.returncode, out.stdout[-200:])
