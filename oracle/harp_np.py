"""CPU restatement (numpy, TEST INFRASTRUCTURE ONLY) of the harp-side steps on
either side of the DISORT solve, for the parity tests of include/hdharp.h.

Nothing in pyharp_amd/ imports this module; it is the checker, never the
thing measured or shipped.  Each function cites the reference code it follows
(/root/reference at the survey snapshot).

Parity status: the reference's tests for these steps (tests/test_attenuator.cpp)
print without asserting, and the reference sources need the CMake-generated
configure.h, so they are not built here.  The restatement is pinned by
closed-form properties in tests/test_harp_oracle.py (exact table values at the
nodes, linearity between them, clamping outside, constant-spacing band sums)
and by the amars_sw example's own quantitative statement that the integrated
TOA downward flux is within 2 W/m^2 of 410 W/m^2 (examples/amars_sw.cpp:75-77).
"""

from __future__ import annotations

import numpy as np


def locate(xx, x):
    """src/math/locate.h:15-42 (Numerical Recipes locate), zero-offset result:
    j with xx[j] <= x < xx[j+1]; -1 below, n-1 at/above the last node."""
    n = len(xx)
    jl, ju = 0, n + 1
    ascnd = xx[n - 1] >= xx[0]
    while ju - jl > 1:
        jm = (ju + jl) >> 1
        if (x >= xx[jm - 1]) == ascnd:
            jl = jm
        else:
            ju = jm
    if x == xx[0]:
        j = 1
    elif x == xx[n - 1]:
        j = n
    else:
        j = jl
    return j - 1


def interp1(x, axis, data):
    """src/math/interpn.h:34-76 with ndim = 1: data (rows, nval) -> (nval,)."""
    n = len(axis)
    i1 = locate(axis, x)
    if i1 == -1:
        i1 = i2 = 0
    elif i1 == n - 1:
        i2 = n - 1
    else:
        i2 = i1 + 1
    x1, x2 = axis[i1], axis[i2]
    v1, v2 = data[i1], data[i2]
    if x2 != x1:
        return ((x - x1) * v2 + (x2 - x) * v1) / (x2 - x1)
    return (v1 + v2) / 2.0


def read_table(path):
    """src/utils/fileio.cpp decomment_file + the 2-pass read of s8_fuller.cpp:29-62."""
    rows = []
    with open(path) as f:
        for line in f:
            line = line.split("#", 1)[0].strip()
            if line:
                rows.append([float(v) for v in line.split()])
    return np.asarray(rows, dtype=np.float64)


def load_attenuator(path, species_weight):
    """(kwave [um], kdata (rows, 2)) after reset(): k_ext *= species weight
    (s8_fuller.cpp:64-66)."""
    t = read_table(path)
    kdata = t[:, 1:].copy()
    kdata[:, 0] *= species_weight
    return t[:, 0].copy(), kdata


def attenuate(kwave, kdata, species, conc, wavenumber=None, wavelength=None):
    """S8FullerImpl::forward (s8_fuller.cpp:72-117): (nwave, ncol, nlyr, 2)."""
    coord = 1.0e4 / np.asarray(wavenumber) if wavelength is None else np.asarray(wavelength)
    ncol, nlyr, _ = conc.shape
    out = np.zeros((len(coord), ncol, nlyr, 2))
    c = conc[:, :, species]
    for w, x in enumerate(coord):
        k, s = interp1(x, kwave, kdata)
        kc = k * c
        out[w, :, :, 0] = kc
        out[w, :, :, 1] = s * kc
    return out


def band_optics(tables, conc, dz, nprop=2, wavenumber=None, wavelength=None):
    """examples/amars_sw.cpp:261-271: prop = sum_a attenuate_a; prop *= dz;
    prop[...,1] /= prop[...,0] (0 where tau = 0).  tables: [(kwave, kdata, species)]."""
    ncol, nlyr, _ = conc.shape
    dz = np.broadcast_to(np.asarray(dz, np.float64).reshape(-1, nlyr), (ncol, nlyr))
    tot = None
    for kwave, kdata, sp in tables:
        a = attenuate(kwave, kdata, sp, conc, wavenumber, wavelength)
        tot = a if tot is None else tot + a
    tot = tot * dz[None, :, :, None]
    prop = np.zeros(tot.shape[:3] + (nprop,))
    prop[..., 0] = tot[..., 0]
    with np.errstate(invalid="ignore", divide="ignore"):
        prop[..., 1] = np.where(tot[..., 0] != 0.0, tot[..., 1] / tot[..., 0], 0.0)
    return prop


def hg_table(kwave, g):
    """A Henyey-Greenstein asymmetry per table row: scalar g -> filled, else as given."""
    return np.broadcast_to(np.asarray(g, np.float64), (len(kwave),)).copy()


def band_loop_optics(tables, conc, dz, nmom, wavenumber=None, wavelength=None, ext0=None):
    """RadiationBandImpl::forward's mixing (src/radiation/radiation_band.cpp:86-116) in
    the reference's operation order, on the layout the solver reads:
    (nwave, ncol, nlyr, 2 + nmom).

    tables: [(kwave, kdata (rows, 2) = (k_ext [m^2/mol], ssa), species, g (rows,) or None)];
    attenuator a's kdata = [k_a c_a, ssa_a, g_a^1 .. g_a^nmom] (HG moments when g is
    given; g^l as repeated products), all three interpolated by interp1.  Per element:
      ext = ext0 + sum_a k_a c_a;  sca = sum_a ssa_a * (k_a c_a);
      m_l = sum_a (chi_al * ssa_a) * (k_a c_a);
      prop[2+l] = m_l / (sca + 1e-10);  prop[1] = sca / (ext + 1e-10);  prop[0] = ext * dz.
    ext0: (nwave, ncol, nlyr) extinction of nprop = 1 attenuators (RFM), added first.
    The reference's latent bugs (prop without the wave axis, :83-84; aerosol slot 1
    already ssa*k*c, s8_fuller.cpp:113-114) are not reproduced (include/hdharp.h)."""
    coord = 1.0e4 / np.asarray(wavenumber) if wavelength is None else np.asarray(wavelength)
    ncol, nlyr, _ = conc.shape
    nwave = len(coord)
    dz = np.broadcast_to(np.asarray(dz, np.float64).reshape(-1, nlyr), (ncol, nlyr))
    ext = np.zeros((nwave, ncol, nlyr))
    sca = np.zeros((nwave, ncol, nlyr))
    mom = np.zeros((nwave, ncol, nlyr, nmom))
    if ext0 is not None:
        ext = ext + np.asarray(ext0, np.float64).reshape(nwave, ncol, nlyr)
    for kwave, kdata, sp, g in tables:
        cols = [kdata[:, 0], kdata[:, 1], np.zeros(len(kwave)) if g is None else g]
        k3 = np.stack(cols, axis=1)
        c = conc[:, :, sp]
        for w, x in enumerate(coord):
            k, s, gw = interp1(x, kwave, k3)
            kc = k * c
            ext[w] = ext[w] + kc
            sca[w] = sca[w] + s * kc
            if g is not None:
                chi = gw
                for l in range(nmom):
                    if l:
                        chi = chi * gw
                    mom[w, :, :, l] = mom[w, :, :, l] + (chi * s) * kc
    prop = np.zeros((nwave, ncol, nlyr, 2 + nmom))
    prop[..., 2:] = mom / (sca + 1e-10)[..., None]
    prop[..., 1] = sca / (ext + 1e-10)
    prop[..., 0] = ext * dz[None]
    return prop


def band_flux(flux, weight):
    """sum_w weight_w F_w in w order (amars_lw.cpp:84-88)."""
    out = np.zeros(flux.shape[1:])
    for w in range(flux.shape[0]):
        out = weight[w] * flux[w] + out
    return out


def heating_rate(bflux, dz, rho, cp):
    """examples/amars_sw.cpp:291-302: dT/dt[k] = -(1/(rho_k cp)) (dF[k+1]-dF[k])/dz_k,
    dF = F_up - F_dn, level 0 = bottom.  bflux (ncol, nlyr+1, 2)."""
    df = bflux[..., 0] - bflux[..., 1]
    ncol, nlev = df.shape
    dz = np.broadcast_to(dz, (ncol, nlev - 1))
    rho = np.broadcast_to(rho, (ncol, nlev - 1))
    return -(1.0 / (rho * cp)) * (df[:, 1:] - df[:, :-1]) / dz


def spherical_flux_correction(bflux, x1f, area, vol):
    """src/utils/spherical_flux_correction.cpp:3-17 along the level axis of the
    harp band flux (ncol, nlev, 2); returns a corrected copy."""
    f = np.array(bflux, dtype=np.float64, copy=True)
    nlev = f.shape[1]
    fiu = f[:, nlev - 1, :].copy()
    for i in range(nlev - 2, -1, -1):
        dx1f = x1f[i + 1] - x1f[i]
        fi = f[:, i, :].copy()
        volh = (fiu - fi) / dx1f * vol[i]
        fiu = fi
        f[:, i, :] = (f[:, i + 1, :] * area[i + 1] - volh) / area[i]
    return f


# ---- the amars_sw example's own helpers (examples/amars_sw.cpp) -------------

def short_wavenumber_grid(nwave):
    """amars_sw.cpp:70-76."""
    return np.linspace(2000.0, 50000.0, nwave)


def bb_toa_flux(wave, ncol, temp, fscale):
    """amars_sw.cpp:84-102: scaled blackbody TOA flux [W/(m^2 cm^-1)]."""
    c1 = 1.19144e-5 * 1e-3
    c2 = 1.4388
    sr_sun = 2.92842e-5
    f = fscale * sr_sun * c1 * wave ** 3 / (np.exp(c2 * wave / temp) - 1.0)
    return np.repeat(f[:, None], ncol, axis=1)


def read_aerosol_profile(path):
    """amars_sw.cpp:104-126 + 228-239: p [Pa], T [K], mixing ratios (2, n)."""
    t = read_table(path)
    return t[:, 0] * 1e5, t[:, 1].copy(), np.stack([t[:, 2], t[:, 3]])


def regrid_ptx(nlyr, p, T, mr):
    """amars_sw.cpp:128-152: uniform p and T grids (top first), mixing ratios
    interpolated in p with interp1 (interpolate_mixing_ratios, :24-36)."""
    p_min, p_max = p.min(), p.max()
    T_min, T_max = T.min(), T.max()
    p_step = (p_max - p_min) / (nlyr - 1)
    T_step = (T_max - T_min) / (nlyr - 1)
    new_p = np.zeros(nlyr)
    new_T = np.zeros(nlyr)
    for i in range(nlyr):
        new_p[nlyr - 1 - i] = p_min + i * p_step
        new_T[nlyr - 1 - i] = T_min + i * T_step
    new_mr = np.zeros((mr.shape[0], nlyr))
    for j in range(mr.shape[0]):
        for i in range(nlyr):
            new_mr[j, i] = interp1(new_p[i], p, mr[j][:, None])[0]
    return new_p, new_T, new_mr


def calc_dz(nlyr, new_p, new_rho, g):
    """amars_sw.cpp:154-170 (the last layer is twice the one below it)."""
    dz = np.ones(nlyr)
    for i in range(nlyr - 1):
        dz[i] *= (new_p[i] - new_p[i + 1]) / (g * new_rho[i])
    dz[nlyr - 1] *= 2 * dz[nlyr - 2]
    return dz


def amars_sw_atmosphere(profile_path, nlyr=40, g=3.711, mean_mol_weight=0.044, R=8.314472):
    """conc (1, nlyr, 2) [mol/m^3] (S8 = species 0, H2SO4 = 1), rho, dz, p
    (amars_sw.cpp:228-258)."""
    p, T, mr = read_aerosol_profile(profile_path)
    new_p, new_T, new_mr = regrid_ptx(nlyr, p, T, mr)
    conc = np.ones((1, nlyr, 2))
    new_rho = np.zeros(nlyr)
    for k in range(nlyr):
        conc[0, k, 0] = (new_mr[1, k] * new_p[k]) / (R * new_T[k])
        conc[0, k, 1] = (new_mr[0, k] * new_p[k]) / (R * new_T[k])
        new_rho[k] = (new_p[k] * mean_mol_weight) / (R * new_T[k])
    dz = calc_dz(nlyr, new_p, new_rho, g)
    return conc, new_rho, dz, new_p


def interpn(coor, data, axes):
    """src/math/interpn.h:34-76 for any ndim (nval = 1): data has shape
    tuple(len(a) for a in axes); the recursion and arithmetic order of the
    reference (lerp of the two sub-interpolations along the leading axis)."""
    axis = axes[0]
    n = len(axis)
    x = coor[0]
    i1 = locate(axis, x)
    if i1 == -1:
        i1 = i2 = 0
    elif i1 == n - 1:
        i2 = n - 1
    else:
        i2 = i1 + 1
    if len(axes) == 1:
        v1, v2 = data[i1], data[i2]
    else:
        v1 = interpn(coor[1:], data[i1], axes[1:])
        v2 = interpn(coor[1:], data[i2], axes[1:])
    x1, x2 = axis[i1], axis[i2]
    if x2 != x1:
        return ((x - x1) * v2 + (x2 - x) * v1) / (x2 - x1)
    return (v1 + v2) / 2.0


def rfm_forward(wave, lnp_axis, temp_axis, ref_temp, kdata, conc, pres, temp, species):
    """harp::RFMImpl::forward (src/opacity/rfm.cpp:122-197) + get_reftemp
    (:199-225): tempa = T - interp1(ln p; ln p_ref, T_ref); k = interpn over
    (wave, ln p, tempa) of ln(m^2/kmol); prop = 1e-3 exp(k) conc[..., species].
    Returns (nwave, ncol, nlyr, 1)."""
    conc = np.asarray(conc, np.float64)
    ncol, nlyr = conc.shape[:2]
    nwave = len(wave)
    out = np.zeros((nwave, ncol, nlyr, 1))
    lnp = np.log(np.asarray(pres, np.float64))
    tref = np.zeros((ncol, nlyr))
    for c in range(ncol):
        for l in range(nlyr):
            tref[c, l] = interpn([lnp[c, l]], np.asarray(ref_temp), [lnp_axis])
    tempa = np.asarray(temp, np.float64) - tref
    for w in range(nwave):
        for c in range(ncol):
            for l in range(nlyr):
                v = interpn([wave[w], lnp[c, l], tempa[c, l]], kdata,
                            [wave, lnp_axis, temp_axis])
                out[w, c, l, 0] = 1.0e-3 * np.exp(v) * conc[c, l, species]
    return out
