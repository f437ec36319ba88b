"""Numpy model of the HIP kernels' *formulation* (test-side only).

This mirrors, step by step, what ``pyharp_amd/csrc/hd_kernels.hip`` computes so
that a formulation error can be separated from a kernel-coding error.  It is
NOT the oracle (``oracle/disort_np.py`` is, with DISORT's own structure) and is
never imported by the product.

Formulation:
  * homogeneous solution from the symmetrised eigenproblem
      L L^T = D^1/2 (W^-1 - S-) D^1/2,   Sym = L^T D^1/2 (W^-1 - S+) D^1/2 L
    (S+/- = even/odd Legendre parts of the phase matrix, D = W M^-1),
    k^2 = eig(Sym), X = W^-1 D^1/2 L V, Y = -k W^-1 D^1/2 L^-T V
  * layer operators  Q- = X m D-^-1, Q+ = Y m D+^-1,
      D+ = X(1+e) - Y m,  D- = X m - Y(1+e),   R = Q- + Q+,  T = I - Q- + Q+
  * sources from the beam/thermal particular solutions
  * adding sweep top->bottom (R_above, S_down), scalar Lambert surface,
    back-substitution bottom->top.
"""

import math

import numpy as np

from oracle.disort_np import DITHER, double_gauss, legendre_table, plkavg


def layer_ops(dtau, ssa, chi, nstr, umu0, fbeam, b_top, b_bot, tauc_top):
    nn = nstr // 2
    mu, w = double_gauss(nn)
    if ssa == 1.0:
        ssa = 1.0 - DITHER
    nmom = len(chi)
    f = chi[nstr - 1] if nmom >= nstr else 0.0
    taup = (1.0 - ssa * f) * dtau
    om = ssa * (1.0 - f) / (1.0 - ssa * f)
    gl = np.array([(2 * l + 1) * om * ((1.0 if l == 0 else (chi[l - 1] if l - 1 < nmom else 0.0)) - f) / (1.0 - f)
                   for l in range(nstr)])
    pt = legendre_table(nstr, mu)  # (nstr, nn)
    ev = np.arange(nstr) % 2 == 0
    splus = (pt[ev].T * gl[ev]) @ pt[ev]
    sminus = (pt[~ev].T * gl[~ev]) @ pt[~ev]
    d = w / mu
    sd = np.sqrt(d)
    am = np.diag(1.0 / mu) - sd[:, None] * sminus * sd[None, :]
    ap = np.diag(1.0 / mu) - sd[:, None] * splus * sd[None, :]
    lch = np.linalg.cholesky(am)
    sym = lch.T @ ap @ lch
    k2, v = np.linalg.eigh(sym)
    k = np.sqrt(k2)
    lv = lch @ v
    x = (sd / w)[:, None] * lv
    y = -(sd / w)[:, None] * np.linalg.solve(lch.T, v) * k[None, :]
    e = np.exp(-k * taup)
    m = -np.expm1(-k * taup)
    dp = x * (1 + e) - y * m
    dm = x * m - y * (1 + e)
    qm = np.linalg.solve(dm.T, (x * m).T).T
    qp = np.linalg.solve(dp.T, (y * m).T).T
    r = qm + qp
    t = np.eye(nn) - qm + qp

    def linv(vec):   # W^-1 D^1/2 L^-T L^-1 D^1/2 vec
        z = np.linalg.solve(lch, sd * vec)
        z = np.linalg.solve(lch.T, z)
        return sd * z / w

    splus_src = np.zeros(nn)
    sminus_src = np.zeros(nn)
    e0 = 1.0
    if fbeam > 0 and umu0 > 0:
        e0 = math.exp(-taup / umu0)
        p0 = legendre_table(nstr, [umu0])[:, 0]
        xs = fbeam / (2 * math.pi) * (pt[ev].T @ (gl[ev] * p0[ev]))
        xd = -fbeam / (2 * math.pi) * (pt[~ev].T @ (gl[~ev] * p0[~ev]))
        # r = (alpha-beta) M^-1 xs + M^-1 xd / mu0 ; (alpha-beta)M^-1 = -M^-1 D^-1/2 L L^T D^1/2
        rv = -(1.0 / (mu * sd)) * (lch @ (lch.T @ (sd * xs))) + xd / (mu * umu0)
        # X^-1 = V^T L^-1 D^-1/2 W
        tt = v.T @ np.linalg.solve(lch, (w / sd) * rv)
        tt = tt / (1.0 / umu0 ** 2 - k2)
        s = x @ tt
        dd = linv(xd - mu * s / umu0)
        zp = 0.5 * (s + dd)
        zm = 0.5 * (s - dd)
        att = math.exp(-tauc_top / umu0)
        zp *= att
        zm *= att
        splus_src += zp - r @ zm - t @ (zp * e0)
        sminus_src += zm * e0 - t @ zm - r @ (zp * e0)
    if b_top != 0.0 or b_bot != 0.0:
        h = linv(mu)
        qmh = qm @ h
        one = np.ones(nn)
        if taup > 0:
            gfac = (b_bot - b_top) * (2.0 / taup) * qmh
        else:
            gfac = np.zeros(nn)
        splus_src += b_top * (one - r @ one) - b_bot * (t @ one) + gfac
        sminus_src += b_bot * (one - r @ one) - b_top * (t @ one) - gfac
    return dict(r=r, t=t, sp=splus_src, sm=sminus_src, taup=taup)


def solve_column(dtauc, ssalb, chis, nstr, umu0=1.0, fbeam=0.0, albedo=0.0,
                 fisot=0.0, planck=False, temper=None, btemp=0.0, wvnmlo=0.0,
                 wvnmhi=0.0):
    """Layers top->bottom; returns (flup, fdn) at nlyr+1 levels top->bottom."""
    nn = nstr // 2
    mu, w = double_gauss(nn)
    nlyr = len(dtauc)
    beam = fbeam > 0 and umu0 > 0
    pk = [plkavg(wvnmlo, wvnmhi, tt) for tt in temper] if planck else [0.0] * (nlyr + 1)
    ops = []
    tauc = 0.0
    for lc in range(nlyr):
        o = layer_ops(dtauc[lc], ssalb[lc], chis[lc], nstr, umu0, fbeam if beam else 0.0,
                      pk[lc], pk[lc + 1], tauc)
        o["tauc_top"] = tauc
        tauc += o["taup"]
        ops.append(o)
    c = 2 * math.pi * w * mu
    ra = np.zeros((nn, nn))
    sd = np.full(nn, fisot)
    store = []
    for o in ops:
        w1 = np.eye(nn) - o["r"] @ ra
        zt = np.linalg.solve(w1, o["t"])
        t_ = np.linalg.solve(w1, o["r"] @ sd + o["sp"])
        store.append((zt, t_, ra.T @ c, c @ sd))
        u = ra @ t_ + sd
        p = ra @ zt
        ra = o["r"] + o["t"] @ p
        sd = o["t"] @ u + o["sm"]
    e_surf = 0.0
    if beam:
        e_surf += albedo * umu0 * fbeam * math.exp(-tauc / umu0) / math.pi
    if planck:
        e_surf += (1 - albedo) * plkavg(wvnmlo, wvnmhi, btemp)
    wm = w * mu
    xs = (2 * albedo * wm @ sd + e_surf) / (1 - 2 * albedo * wm @ (ra @ np.ones(nn)))
    ip = np.full(nn, xs)
    flup = np.zeros(nlyr + 1)
    fdn = np.zeros(nlyr + 1)
    dirb = (lambda tt: umu0 * fbeam * math.exp(-tt / umu0)) if beam else (lambda tt: 0.0)
    flup[nlyr] = c @ ip
    fdn[nlyr] = c @ (ra @ ip + sd) + dirb(tauc)
    for lc in range(nlyr - 1, -1, -1):
        zt, t_, rc, cs = store[lc]
        ip = zt @ ip + t_
        flup[lc] = c @ ip
        fdn[lc] = rc @ ip + cs + dirb(ops[lc]["tauc_top"])
    return flup, fdn
