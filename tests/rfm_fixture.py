"""Synthetic RFM ck table in classic netCDF (written with scipy.io.netcdf_file),
laid out as harp's RFM reader expects (src/opacity/rfm.cpp:30-120,
src/utils/read_weights.cpp:18-46): dims Wavenumber, Pressure, TempGrid, weights;
variables Wavenumber, Pressure [Pa], TempGrid [K anomaly], Temperature [K]
(reference profile), one ln(m^2/kmol) table per species, weights.  The real
amarsw-ck-B1.nc is git-ignored upstream; this stands in for it in tests."""

import numpy as np


def write_rfm_table(path, nwave=16, npres=12, ntemp=5, species=("CO2", "H2O"), seed=3,
                    version=2):
    from scipy.io import netcdf_file
    rng = np.random.default_rng(seed)
    f = netcdf_file(path, "w", version=version)
    f.createDimension("Wavenumber", nwave)
    f.createDimension("Pressure", npres)
    f.createDimension("TempGrid", ntemp)
    f.createDimension("weights", nwave)
    wave = f.createVariable("Wavenumber", "d", ("Wavenumber",))
    wave[:] = np.linspace(1.0, 150.0, nwave)
    pres = f.createVariable("Pressure", "d", ("Pressure",))
    pres[:] = np.logspace(7, 2, npres)                    # descending, like a profile
    tg = f.createVariable("TempGrid", "d", ("TempGrid",))
    tg[:] = np.linspace(-40.0, 40.0, ntemp)
    tr = f.createVariable("Temperature", "d", ("Pressure",))
    tr[:] = np.linspace(320.0, 150.0, npres)
    tables = {}
    for sp in species:
        v = f.createVariable(sp, "d", ("Wavenumber", "Pressure", "TempGrid"))
        t = rng.uniform(-8.0, 4.0, (nwave, npres, ntemp))
        v[:] = t
        tables[sp] = t
    w = f.createVariable("weights", "d", ("weights",))
    x, gw = np.polynomial.legendre.leggauss(nwave)
    w[:] = 0.5 * gw
    w.units = "1"
    f.title = "synthetic RFM ck table"
    f.close()
    return dict(wave=np.linspace(1.0, 150.0, nwave), pres=np.logspace(7, 2, npres),
                tgrid=np.linspace(-40.0, 40.0, ntemp), tref=np.linspace(320.0, 150.0, npres),
                tables=tables, weights=0.5 * gw)
