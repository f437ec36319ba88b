"""Numpy FP64 restatement of the flux-only DISORT solve (azimuthal mode m=0).

TEST INFRASTRUCTURE ONLY.  Nothing in ``pyharp_amd`` imports this module; only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may use it, and only as the checker.

What this follows
-----------------
The reference (franciscospauldingastudillo/pyharp @ 2025-02-17) does not contain
the solver arithmetic: it links ``pydisort`` @ ``afee3ec897f``
(``cmake/pydisort.cmake:9-11``), which wraps cdisort 2.1.3
(``src/rtsolver/rtsolver.hpp:16``).  Neither is present in the container and
there is no network, so this module restates the *published* DISORT method
(Stamnes, Tsay, Wiscombe & Jayaweera 1988; DISORT 2.0 report) with the same
stage structure as cdisort:

=============  ==============================================================
cdisort stage  here
=============  ==============================================================
c_qgausn       :func:`double_gauss`    (Gauss-Legendre on (0,1), nstr/2 nodes)
c_setdis       :func:`setdis`          (dither, delta-M, scaled optical depth)
c_soleig       :func:`soleig`          (eig of (alpha-beta)(alpha+beta), nstr/2)
c_upbeam       :func:`upbeam`          (dense nstr x nstr solve)
c_upisot       :func:`upisot`          (two dense nstr x nstr solves)
c_setmtx/solve0 :func:`solve_bc`       (banded system, half-bandwidth 3*nstr/2-1,
                                        LAPACK gbsv = LINPACK SGBFA/SGBSL)
c_fluxes       :func:`fluxes`
c_planck_func1 :func:`plkavg`          (DISORT PLKAVG series, same truncation)
=============  ==============================================================

harp-side conventions (``disort_forward``) follow the call sites:
``prop`` is ``(nwave, ncol, nlyr, nprop)`` with layer 0 at the **bottom**
(``examples/amars_sw.cpp:141-146``, ``src/radiation/radiation_band.cpp:116``),
slots ``IEX=0`` (optical thickness), ``ISS=1`` (single-scattering albedo),
``IPM=2..`` phase moments chi_1..chi_nmom (``src/index.h:12-18``; chi_0 = 1
implicit, as ``tests/test_disort.cpp:31-40`` allocates ``2+nstr`` slots for
``nmom = nstr``).  The solver works top->bottom and the output flux
``(nwave, ncol, nlyr+1, 2)`` has level 0 at the surface, ``[...,0]`` = upward,
``[...,1]`` = rfldir + rfldn (``src/rtsolver/rt_solver_disort.cpp_:172-181``).

Parity status: **parity unpinned** against cdisort itself (absent).  The
module is pinned by (i) the DISOTEST problem-1 published fluxes restated in
``tests/golden/disotest1.json`` and (ii) analytic known answers (direct beam,
omega=0 slab on the same quadrature, conservative-scattering flux
conservation) in ``tests/test_oracle.py``.
"""

from __future__ import annotations

import math

import numpy as np
import scipy.linalg

# DISORT 2.0 dither: ssalb == 1 is replaced by 1 - DITHER, where
# DITHER = 10*eps, enlarged to sqrt() on 14+ digit machines.
DITHER = math.sqrt(10.0 * np.finfo(np.float64).eps)

# PLKAVG constants (DISORT 2.0).
PLK_C2 = 1.438786
PLK_SIGMA = 5.67032e-8
PLK_VCUT = 1.5
PLK_VCP = (10.25, 5.7, 3.9, 2.9, 2.3, 1.9, 0.0)


# --------------------------------------------------------------------------- #
# quadrature / Legendre
# --------------------------------------------------------------------------- #
def double_gauss(nn: int):
    """nn-point Gauss-Legendre nodes/weights on (0, 1) (c_qgausn); sum(w)=1."""
    x, w = np.polynomial.legendre.leggauss(nn)
    return 0.5 * (x + 1.0), 0.5 * w


def legendre_table(lmax: int, mu) -> np.ndarray:
    """P_l(mu) for l = 0..lmax-1, shape (lmax, len(mu))."""
    mu = np.atleast_1d(np.asarray(mu, dtype=np.float64))
    p = np.zeros((lmax, mu.size))
    p[0] = 1.0
    if lmax > 1:
        p[1] = mu
    for l in range(2, lmax):
        p[l] = ((2 * l - 1) * mu * p[l - 1] - (l - 1) * p[l - 2]) / l
    return p


# --------------------------------------------------------------------------- #
# Planck
# --------------------------------------------------------------------------- #
def _plkf(x):
    return x ** 3 / math.expm1(x)


def plkavg(wnumlo: float, wnumhi: float, t: float) -> float:
    """Planck radiance integrated over [wnumlo, wnumhi] cm^-1 at T [W m^-2 sr^-1].

    Restatement of DISORT 2.0 PLKAVG (c_planck_func1): power series below
    v = 1.5, the exponential series truncated by the VCP table above, and an
    iterated Simpson rule when the interval is narrow (< 1 % relative).
    """
    if t < 0.0 or wnumhi <= wnumlo or wnumlo < 0.0:
        raise ValueError("plkavg: bad temperature or wavenumbers")
    if t < 1.0e-4:
        return 0.0
    sigdpi = PLK_SIGMA / math.pi
    conc = 15.0 / math.pi ** 4
    v = [PLK_C2 * wnumlo / t, PLK_C2 * wnumhi / t]
    vmax = math.log(np.finfo(np.float64).max)
    epsil = np.finfo(np.float64).eps
    if v[0] > epsil and v[1] < vmax and (wnumhi - wnumlo) / wnumhi < 1.0e-2:
        hh = v[1] - v[0]
        oldval = 0.0
        val0 = _plkf(v[0]) + _plkf(v[1])
        val = val0
        for n in range(1, 11):
            dl = hh / (2 * n)
            val = val0
            for k in range(1, 2 * n):
                val += 2 * (1 + k % 2) * _plkf(v[0] + k * dl)
            val = dl / 3.0 * val
            if abs((val - oldval) / val) <= 1.0e-6:
                break
            oldval = val
        return sigdpi * t ** 4 * conc * val

    a = (1.0 / 3.0, -1.0 / 8.0, 1.0 / 60.0, -1.0 / 5040.0,
         1.0 / 272160.0, -1.0 / 13305600.0, 1.0 / 622702080.0)
    p = [0.0, 0.0]
    d = [0.0, 0.0]
    smallv = 0
    for i in range(2):
        vi = v[i]
        if vi < PLK_VCUT:
            smallv += 1
            vsq = vi * vi
            p[i] = conc * vsq * vi * (a[0] + vi * (a[1] + vi * (a[2] + vsq * (
                a[3] + vsq * (a[4] + vsq * (a[5] + vsq * a[6]))))))
        else:
            mmax = 0
            while True:
                mmax += 1
                if not vi < PLK_VCP[mmax - 1]:
                    break
            ex = math.exp(-vi)
            exm = 1.0
            di = 0.0
            for m in range(1, mmax + 1):
                mv = m * vi
                exm *= ex
                di += exm * (6.0 + mv * (6.0 + mv * (3.0 + mv))) / m ** 4
            d[i] = conc * di
    if smallv == 2:
        val = p[1] - p[0]
    elif smallv == 1:
        val = 1.0 - p[0] - d[1]
    else:
        val = d[0] - d[1]
    return sigdpi * t ** 4 * val


# --------------------------------------------------------------------------- #
# per-solve stages
# --------------------------------------------------------------------------- #
def setdis(dtauc, ssalb, pmom, nstr):
    """Dither, delta-M scaling, cumulative scaled optical depth (c_setdis).

    pmom: (nlyr, nmom+1) with pmom[:,0] = 1.
    Returns dtaucp, taucpr (nlyr+1), tauc (nlyr+1), oprim, gl (nlyr, nstr).
    """
    dtauc = np.asarray(dtauc, np.float64)
    ssalb = np.where(np.asarray(ssalb, np.float64) == 1.0, 1.0 - DITHER, ssalb)
    nlyr = dtauc.size
    nmom = pmom.shape[1] - 1
    f = pmom[:, nstr] if nmom >= nstr else np.zeros(nlyr)
    dtaucp = (1.0 - ssalb * f) * dtauc
    oprim = ssalb * (1.0 - f) / (1.0 - ssalb * f)
    gl = np.zeros((nlyr, nstr))
    kmax = min(nstr, nmom + 1)
    for k in range(kmax):
        gl[:, k] = (2 * k + 1) * oprim * (pmom[:, k] - f) / (1.0 - f)
    for k in range(kmax, nstr):
        gl[:, k] = (2 * k + 1) * oprim * (0.0 - f) / (1.0 - f)
    taucpr = np.concatenate([[0.0], np.cumsum(dtaucp)])
    tauc = np.concatenate([[0.0], np.cumsum(dtauc)])
    return dtaucp, taucpr, tauc, oprim, gl


def _cc_matrix(gl_lc, cmu_full, cwt_full, ylm):
    """CC(i,j) = 1/2 sum_l GL_l P_l(mu_i) P_l(mu_j) w_j over all 2nn streams."""
    return 0.5 * (ylm.T * gl_lc) @ ylm * cwt_full[None, :]


def soleig(cc, cmu):
    """Homogeneous solution of one layer (c_soleig / c_asymtx).

    Returns kk (nn, positive), gplus, gminus (nn x nn; columns = modes) such
    that [gplus[:,j]; gminus[:,j]] * exp(-kk_j tau) solves the RTE and the
    swapped pair is the exp(+kk_j tau) solution.
    """
    nn = cmu.size
    cpp = cc[:nn, :nn]
    cpm = cc[:nn, nn:]
    alpha = (cpp - np.eye(nn)) / cmu[:, None]
    beta = cpm / cmu[:, None]
    apb = alpha + beta
    amb = alpha - beta
    evals, evecs = np.linalg.eig(amb @ apb)
    if np.max(np.abs(evals.imag)) > 1e-8 * max(1.0, np.max(np.abs(evals.real))):
        raise ArithmeticError("soleig: complex eigenvalues")
    k2 = evals.real
    x = evecs.real
    if np.any(k2 <= 0.0):
        raise ArithmeticError("soleig: non-positive eigenvalue")
    kk = np.sqrt(k2)
    y = (apb @ x) / kk[None, :]
    gplus = 0.5 * (x + y)
    gminus = 0.5 * (x - y)
    return kk, gplus, gminus


def upbeam(cc, cmu_full, gl_lc, ylm_full, umu0, fbeam):
    """Beam particular solution Z with I_p(tau) = Z exp(-tau/umu0) (c_upbeam)."""
    nstr = cmu_full.size
    p0 = legendre_table(nstr, [-umu0])[:, 0]
    x0 = fbeam / (4.0 * math.pi) * (ylm_full.T @ (gl_lc * p0))
    a = np.diag(1.0 + cmu_full / umu0) - cc
    return np.linalg.solve(a, x0)


def upisot(cc, cmu_full, oprim_lc, xr0, xr1):
    """Thermal particular solution Z0 + Z1 tau (c_upisot)."""
    nstr = cmu_full.size
    a = np.eye(nstr) - cc
    z1 = np.linalg.solve(a, np.full(nstr, (1.0 - oprim_lc) * xr1))
    z0 = np.linalg.solve(a, (1.0 - oprim_lc) * xr0 + cmu_full * z1)
    return z0, z1


def disort_column(dtauc, ssalb, pmom, nstr, *, umu0=1.0, fbeam=0.0,
                  albedo=0.0, fisot=0.0, planck=False, temper=None,
                  btemp=0.0, ttemp=0.0, temis=0.0, wvnmlo=0.0, wvnmhi=0.0,
                  return_all=False):
    """One flux-only DISORT solve, cdisort conventions (layers top->bottom).

    Returns dict with rfldir, rfldn, flup (each nlyr+1, at layer boundaries,
    top->bottom) and fdn = rfldir + rfldn.
    """
    dtauc = np.atleast_1d(np.asarray(dtauc, np.float64))
    nlyr = dtauc.size
    if nstr < 2 or nstr % 2:
        raise ValueError("nstr must be even and >= 2")
    nn = nstr // 2
    pmom = np.asarray(pmom, np.float64).reshape(nlyr, -1)
    cmu, cwt = double_gauss(nn)
    cmu_full = np.concatenate([cmu, -cmu])
    cwt_full = np.concatenate([cwt, cwt])
    ylm = legendre_table(nstr, cmu_full)  # (nstr, 2nn)

    dtaucp, taucpr, tauc, oprim, gl = setdis(dtauc, ssalb, pmom, nstr)

    if fbeam > 0.0 and not (0.0 < umu0 <= 1.0):
        # cdisort's input check (c_chekin): a beam needs 0 < umu0 <= 1
        raise ValueError(f"umu0 = {umu0} outside (0, 1] with fbeam > 0")
    beam = fbeam > 0.0
    if planck:
        pkag = np.array([plkavg(wvnmlo, wvnmhi, t) for t in temper])
        bplanck = plkavg(wvnmlo, wvnmhi, btemp)
        tplanck = plkavg(wvnmlo, wvnmhi, ttemp) * temis
    else:
        pkag = np.zeros(nlyr + 1)
        bplanck = tplanck = 0.0

    kk = np.zeros((nlyr, nn))
    gc = np.zeros((nlyr, nstr, nstr))  # columns: nn "+k" modes then nn "-k" modes
    zbeam = np.zeros((nlyr, nstr))
    z0 = np.zeros((nlyr, nstr))
    z1 = np.zeros((nlyr, nstr))
    for lc in range(nlyr):
        cc = _cc_matrix(gl[lc], cmu_full, cwt_full, ylm)
        k, gp, gm = soleig(cc, cmu)
        kk[lc] = k
        gc[lc, :nn, :nn] = gp
        gc[lc, nn:, :nn] = gm
        gc[lc, :nn, nn:] = gm
        gc[lc, nn:, nn:] = gp
        if beam:
            zbeam[lc] = upbeam(cc, cmu_full, gl[lc], ylm, umu0, fbeam)
        if planck:
            xr1 = (pkag[lc + 1] - pkag[lc]) / dtaucp[lc] if dtaucp[lc] > 0 else 0.0
            xr0 = pkag[lc] - xr1 * taucpr[lc]
            z0[lc], z1[lc] = upisot(cc, cmu_full, oprim[lc], xr0, xr1)

    def zpart(lc, tau):
        v = z0[lc] + z1[lc] * tau
        if beam:
            v = v + zbeam[lc] * math.exp(-tau / umu0)
        return v

    ee = np.exp(-kk * dtaucp[:, None])  # (nlyr, nn)

    # --- banded boundary-condition system (c_setmtx), unknowns LL(j, lc) --- #
    ncol = nstr * nlyr
    a = np.zeros((ncol, ncol))
    b = np.zeros(ncol)

    def top_cols(lc):  # intensity at the layer top = gc * [1, e]
        return gc[lc] * np.concatenate([np.ones(nn), ee[lc]])[None, :]

    def bot_cols(lc):  # intensity at the layer bottom = gc * [e, 1]
        return gc[lc] * np.concatenate([ee[lc], np.ones(nn)])[None, :]

    # TOA: downward intensities = fisot + temis*B(ttemp)
    t0 = top_cols(0)
    a[:nn, :nstr] = t0[nn:, :]
    b[:nn] = fisot + tplanck - zpart(0, 0.0)[nn:]
    # interfaces
    for lc in range(nlyr - 1):
        r0 = nn + lc * nstr
        a[r0:r0 + nstr, lc * nstr:(lc + 1) * nstr] = bot_cols(lc)
        a[r0:r0 + nstr, (lc + 1) * nstr:(lc + 2) * nstr] = -top_cols(lc + 1)
        tau = taucpr[lc + 1]
        b[r0:r0 + nstr] = zpart(lc + 1, tau) - zpart(lc, tau)
    # surface (Lambertian)
    r0 = nn + (nlyr - 1) * nstr
    lb = bot_cols(nlyr - 1)
    refl = 2.0 * albedo * (cwt * cmu)  # acts on downward intensities
    a[r0:r0 + nn, (nlyr - 1) * nstr:] = lb[:nn, :] - refl[None, :] @ lb[nn:, :]
    zb = zpart(nlyr - 1, taucpr[nlyr])
    rhs = np.full(nn, (1.0 - albedo) * bplanck)
    if beam:
        rhs += albedo * umu0 * fbeam * math.exp(-taucpr[nlyr] / umu0) / math.pi
    b[r0:r0 + nn] = rhs - (zb[:nn] - refl @ zb[nn:])

    bw = 3 * nn - 1
    ab = np.zeros((2 * bw + 1, ncol))
    for j in range(ncol):
        lo = max(0, j - bw)
        hi = min(ncol, j + bw + 1)
        ab[bw + lo - j:bw + hi - j, j] = a[lo:hi, j]
    ll = scipy.linalg.solve_banded((bw, bw), ab, b)
    ll = ll.reshape(nlyr, nstr)

    # --- fluxes at the nlyr+1 layer boundaries (c_fluxes) --- #
    uu = np.zeros((nlyr + 1, nstr))
    uu[0] = top_cols(0) @ ll[0] + zpart(0, 0.0)
    for lc in range(nlyr):
        uu[lc + 1] = bot_cols(lc) @ ll[lc] + zpart(lc, taucpr[lc + 1])
    wmu = cwt * cmu
    flup = 2.0 * math.pi * uu[:, :nn] @ wmu
    dfdn = 2.0 * math.pi * uu[:, nn:] @ wmu
    if beam:
        rfldir = umu0 * fbeam * np.exp(-tauc / umu0)
        fdntot = dfdn + umu0 * fbeam * np.exp(-taucpr / umu0)
    else:
        rfldir = np.zeros(nlyr + 1)
        fdntot = dfdn
    out = {"rfldir": rfldir, "rfldn": fdntot - rfldir, "flup": flup,
           "fdn": fdntot}
    if return_all:
        out.update(uu=uu, kk=kk, taucpr=taucpr, gl=gl, oprim=oprim)
    return out


# --------------------------------------------------------------------------- #
# harp-level driver (pydisort DisortImpl::forward contract)
# --------------------------------------------------------------------------- #
def disort_forward(prop, bc, temf=None, *, nstr, nmom=None, planck=False,
                   wave_lower=None, wave_upper=None):
    """Batch driver with harp's layout: prop (W, C, L, nprop), layer 0 = bottom.

    bc: dict of (W, C) arrays; keys fbeam, umu0, albedo, btemp, ttemp, temis,
    fisot (missing -> 0, umu0 -> 1).  temf: (C, L+1) bottom->top.
    Returns flux (W, C, L+1, 2), level 0 = surface.
    """
    prop = np.asarray(prop, np.float64)
    nwave, ncol, nlyr, nprop = prop.shape
    if nmom is None:
        nmom = nstr
    nm = max(0, min(nmom, nprop - 2))

    def bcv(key, default):
        if key in bc and bc[key] is not None:
            return np.broadcast_to(np.asarray(bc[key], np.float64), (nwave, ncol))
        return np.full((nwave, ncol), default)

    fbeam, umu0, albedo = bcv("fbeam", 0.0), bcv("umu0", 1.0), bcv("albedo", 0.0)
    btemp, ttemp = bcv("btemp", 0.0), bcv("ttemp", 0.0)
    temis, fisot = bcv("temis", 0.0), bcv("fisot", 0.0)
    flux = np.zeros((nwave, ncol, nlyr + 1, 2))
    for w in range(nwave):
        for c in range(ncol):
            p = prop[w, c, ::-1]  # top -> bottom
            pm = np.zeros((nlyr, nm + 1))
            pm[:, 0] = 1.0
            if nm:
                pm[:, 1:] = p[:, 2:2 + nm]
            ssa = p[:, 1] if nprop > 1 else np.zeros(nlyr)
            kw = {}
            if planck:
                kw = dict(planck=True, temper=np.asarray(temf)[c, ::-1],
                          btemp=btemp[w, c], ttemp=ttemp[w, c],
                          temis=temis[w, c], wvnmlo=wave_lower[w],
                          wvnmhi=wave_upper[w])
            r = disort_column(p[:, 0], ssa, pm, nstr, umu0=umu0[w, c],
                              fbeam=fbeam[w, c], albedo=albedo[w, c],
                              fisot=fisot[w, c], **kw)
            flux[w, c, :, 0] = r["flup"][::-1]
            flux[w, c, :, 1] = r["fdn"][::-1]
    return flux


def layer2level(var, order=4, blower="extrapolate", bupper="constant"):
    """Layer -> level interpolation (src/utils/layer2level.cpp:7-79, interp.hpp:7-21)."""
    var = np.asarray(var, np.float64)
    nlyr = var.shape[-1]
    out = np.zeros(var.shape[:-1] + (nlyr + 1,))
    if nlyr == 1:
        out[..., 0] = var[..., 0]
        out[..., 1] = var[..., 0]
        return out
    out[..., 0] = (3.0 * var[..., 0] - var[..., 1]) / 2.0 if blower == "extrapolate" else var[..., 0]
    if order == 4:
        out[..., 1] = (var[..., 0] + var[..., 1]) / 2.0
        if nlyr > 2:
            out[..., nlyr - 1] = (var[..., nlyr - 1] + var[..., nlyr - 2]) / 2.0
        if nlyr > 3:
            cm = np.array([-1.0 / 12.0, 7.0 / 12.0, 7.0 / 12.0, -1.0 / 12.0])
            for i in range(2, nlyr - 1):
                out[..., i] = var[..., i - 2:i + 2] @ cm
    else:
        out[..., 1:nlyr] = (var[..., :-1] + var[..., 1:]) / 2.0
    out[..., nlyr] = (3.0 * var[..., -1] - var[..., -2]) / 2.0 if bupper == "extrapolate" else var[..., -1]
    return out
