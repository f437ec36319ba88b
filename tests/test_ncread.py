"""Classic-netCDF reader (pyharp_amd/ncread.py) and the RFM table loading on
CPU: files written by scipy.io.netcdf_file (CDF-1 and CDF-2) read back exactly."""

import numpy as np
import pytest

from rfm_fixture import write_rfm_table


@pytest.mark.parametrize("version", [1, 2])
def test_roundtrip_types_and_records(tmp_path, version):
    from scipy.io import netcdf_file
    from pyharp_amd.ncread import NetCDFClassic
    p = str(tmp_path / "t.nc")
    f = netcdf_file(p, "w", version=version)
    f.createDimension("t", None)
    f.createDimension("x", 3)
    f.createDimension("y", 4)
    a = f.createVariable("a", "d", ("x", "y"))
    a[:] = np.arange(12.0).reshape(3, 4) / 7
    b = f.createVariable("b", "f", ("y",))
    b[:] = [1.5, 2.5, -3.25, 4.0]
    c = f.createVariable("c", "i", ("x",))
    c[:] = [7, -8, 9]
    c.units = "count"
    r1 = f.createVariable("r1", "d", ("t", "x"))
    r2 = f.createVariable("r2", "i", ("t",))
    for k in range(5):
        r1[k] = np.arange(3.0) + 10 * k
        r2[k] = k * k
    f.history = "written by the test"
    f.close()
    nc = NetCDFClassic(p)
    assert nc.version == version
    assert nc.dim_len("x") == 3 and nc.dim_len("t") == 5
    np.testing.assert_array_equal(nc.var("a"), np.arange(12.0).reshape(3, 4) / 7)
    np.testing.assert_array_equal(nc.var("b"), [1.5, 2.5, -3.25, 4.0])
    np.testing.assert_array_equal(nc.var("c"), [7, -8, 9])
    np.testing.assert_array_equal(nc.var("r1"), np.arange(3.0)[None] + 10 * np.arange(5)[:, None])
    np.testing.assert_array_equal(nc.var("r2"), np.arange(5) ** 2)
    assert nc.vars["c"]["atts"]["units"] == "count"
    assert "history" in nc.gatts
    with pytest.raises(RuntimeError):
        nc.var("nope")
    with pytest.raises(RuntimeError):
        nc.dim_len("nope")


def test_hdf5_and_garbage_refused(tmp_path):
    from pyharp_amd.ncread import NetCDFClassic
    p = tmp_path / "h.nc"
    p.write_bytes(b"\x89HDF\r\n\x1a\n" + b"\0" * 64)
    with pytest.raises(RuntimeError, match="HDF5"):
        NetCDFClassic(str(p))
    p.write_bytes(b"hello world")
    with pytest.raises(RuntimeError):
        NetCDFClassic(str(p))


def test_rfm_reset_reads_the_tables(tmp_path):
    from pyharp_amd.opacity import RFM, AttenuatorOptions, add_resource_directory, \
        read_weights_rfm
    fx = write_rfm_table(str(tmp_path / "ck.nc"))
    add_resource_directory(str(tmp_path))
    op = AttenuatorOptions().species_names(["CO2", "H2O"]).species_weights([44e-3, 18e-3])
    h2o = RFM(op.copy().species_ids([1]).opacity_files(["ck.nc"]))
    nw, npr, nt = h2o.kshape
    assert (nw, npr, nt) == (16, 12, 5)
    np.testing.assert_array_equal(h2o.kdata.numpy(), fx["tables"]["H2O"])
    np.testing.assert_array_equal(h2o.kaxis[:nw].numpy(), fx["wave"])
    np.testing.assert_allclose(h2o.kaxis[nw:nw + npr].numpy(), np.log(fx["pres"]), rtol=0,
                               atol=0)
    np.testing.assert_array_equal(h2o.krefatm[1].numpy(), fx["tref"])
    np.testing.assert_array_equal(read_weights_rfm("ck.nc").numpy(), fx["weights"])
    with pytest.raises(RuntimeError):
        RFM(op.copy().species_ids([0, 1]).opacity_files(["ck.nc"]))


def test_interpn_oracle_is_multilinear():
    """interpn reproduces a multilinear function inside the grid and clamps outside"""
    from oracle import harp_np as H
    ax = [np.array([1.0, 2.0, 4.0]), np.array([-1.0, 0.5, 2.0, 3.0]), np.array([10.0, 20.0])]
    f = lambda a, b, c: 2 * a - 3 * b + 0.5 * c + 1  # noqa: E731
    data = np.array([[[f(a, b, c) for c in ax[2]] for b in ax[1]] for a in ax[0]])
    for pt in ([1.5, 0.0, 12.0], [3.9, 2.9, 19.0], [2.0, 0.5, 10.0]):
        assert abs(H.interpn(pt, data, ax) - f(*pt)) < 1e-12
    assert abs(H.interpn([0.0, -5.0, 30.0], data, ax) - f(1.0, -1.0, 20.0)) < 1e-12


def test_cpp_reader_matches(tmp_path):
    """include/harp_amd/ncread.hpp (compiled with g++ here) reads the same values"""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "ncread_check")
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(root, "include"),
                    os.path.join(root, "tests", "cpp", "ncread_check.cpp"), "-o", exe, "-lz"],
                   check=True)
    fx = write_rfm_table(str(tmp_path / "ck.nc"), version=1)
    out = subprocess.run([exe, str(tmp_path / "ck.nc"), "dim:Pressure", "Pressure", "H2O",
                          "weights"], capture_output=True, text=True, check=True).stdout.split("\n")
    vals = {}
    for l in out:
        if not l:
            continue
        parts = l.split()
        if parts[0].startswith("dim:"):
            vals[parts[0]] = int(parts[1])
        else:
            vals.setdefault(parts[0], []).append(float(parts[2]))
    assert vals["dim:Pressure"] == 12
    np.testing.assert_array_equal(vals["Pressure"], fx["pres"])
    np.testing.assert_array_equal(np.array(vals["H2O"]).reshape(16, 12, 5), fx["tables"]["H2O"])
    np.testing.assert_array_equal(vals["weights"], fx["weights"])
    bad = tmp_path / "h.nc"
    bad.write_bytes(b"\x89HDF\r\n\x1a\n" + b"\0" * 32)
    r = subprocess.run([exe, "--classic", str(bad), "x"], capture_output=True, text=True)
    assert r.returncode == 2 and "HDF5" in r.stdout
