"""Numpy model of the HIP kernels' *formulation* (test-side only).

This mirrors, step by step, what ``pyharp_amd/csrc/hd_kernels.hip`` computes so
that a formulation error can be separated from a kernel-coding error.  It is
NOT the oracle (``oracle/disort_np.py`` is, with DISORT's own structure) and is
never imported by the product.

Formulation:
  * homogeneous solution from the symmetrised eigenproblem
      L L^T = D^1/2 (W^-1 - S-) D^1/2,   C C^T = D^1/2 (W^-1 - S+) D^1/2,
      Sym = L^T C C^T L = X X^T with X = L^T C;  the kernel's one-sided
    Jacobi rotates X's columns into B = X W (orthogonal columns), so
    k^2 = |b_j|^2, V = B K^-1 and U = L V (here V comes from eigh of X X^T)
  * layer operators in the flux-weighted basis, Omega = U Delta^1/2,
    Psi^T = L^-T V Gamma^1/2, and by Woodbury
      A- = (I + Omega Omega^T)^-1, A+ = (I + Psi^T Psi)^-1,
      R~ = A+ - A-,  T~ = A- + A+ - I,  Q~- = I - A-,  Q~+ = A+ - I
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
    # one-sided Jacobi view (hd_layer_kernel): C C^T = -A+, X = L^T C, Sym = X X^T;
    # the rotations give B = X W with k^2 = |b_j|^2, V = B K^-1 and U = L V
    cch = np.linalg.cholesky(ap)
    x = lch.T @ cch
    _, wv = np.linalg.eigh(x.T @ x)
    bcols = x @ wv
    k2 = np.sum(bcols * bcols, axis=0)
    k = np.sqrt(k2)
    u = lch @ (bcols / k[None, :])            # U = L V = L B K^-1
    # ---- layer operators in the flux-weighted basis (g = sqrt(w mu)) ----
    e = np.exp(-k * taup)
    m = -np.expm1(-k * taup)
    th = m / (1.0 + e)                        # tanh(k tau'/2)
    delta = np.where(k * taup > 1e-8, th / np.where(k > 0, k, 1.0), 0.5 * taup)
    gamma = k * th
    omega = u * np.sqrt(delta)[None, :]       # Omega = U Delta^1/2
    vv = np.linalg.solve(lch, u)              # V = L^-1 U
    psit = np.linalg.solve(lch.T, vv) * np.sqrt(gamma)[None, :]   # Psi^T = L^-T V Gamma^1/2
    # Woodbury: Q~- = I - A-, Q~+ = A+ - I with A- = (I + Omega Omega^T)^-1,
    # A+ = (I + Psi^T Psi)^-1 (two SPD inverses from Cholesky factors)
    aminus = np.linalg.inv(np.eye(nn) + omega @ omega.T)
    aplus = np.linalg.inv(np.eye(nn) + psit @ psit.T)
    qtm = np.eye(nn) - aminus
    qtp = aplus - np.eye(nn)
    g = np.sqrt(w * mu)
    rt = aplus - aminus                       # R~ (symmetric)
    tt_ = aminus + aplus - np.eye(nn)         # T~ (symmetric)

    def linv(vec):   # W^-1 D^1/2 L^-T L^-1 D^1/2 vec
        z = np.linalg.solve(lch, sd * vec)
        z = np.linalg.solve(lch.T, z)
        return sd * z / w

    zp = np.zeros(nn)
    zm = np.zeros(nn)
    e0 = 1.0
    if fbeam > 0 and umu0 > 0:
        e0 = math.exp(-taup / umu0)
        p0 = legendre_table(nstr, [umu0])[:, 0]
        xs = fbeam / (2 * math.pi) * (pt[ev].T @ (gl[ev] * p0[ev]))
        xd = -fbeam / (2 * math.pi) * (pt[~ev].T @ (gl[~ev] * p0[~ev]))
        rv = -(1.0 / (mu * sd)) * (lch @ (lch.T @ (sd * xs))) + xd / (mu * umu0)
        ttv = u.T @ np.linalg.solve(lch.T, np.linalg.solve(lch, (w / sd) * rv))   # V^T y2 = U^T L^-T y2
        ttv = ttv / (1.0 / umu0 ** 2 - k2)
        svec = (sd / w) * (u @ ttv)           # X tt, X = W^-1 D^1/2 L V = W^-1 D^1/2 U
        dd = linv(xd - mu * svec / umu0)
        att = math.exp(-tauc_top / umu0)
        zp = 0.5 * (svec + dd) * att
        zm = 0.5 * (svec - dd) * att
    db = b_bot - b_top
    bsum = b_top + b_bot
    if b_top != 0.0 or b_bot != 0.0:
        b1 = db / taup if taup > 0 else 0.0
        cvec = db + 2.0 * b1 * linv(mu)
    else:
        cvec = np.zeros(nn)
    avec = zm - zp * e0
    bvec = zm + zp * e0
    pv = qtm @ (g * (cvec - avec))
    qv = qtp @ (g * (bvec + bsum))
    splus_src = g * (zp * (1 - e0) - db) + pv - qv
    sminus_src = g * (-zm * (1 - e0) + db) - pv - qv
    # back to the unscaled basis for the sweep in this model
    r = rt * (1 / g)[:, None] * g[None, :]
    t = tt_ * (1 / g)[:, None] * g[None, :]
    splus_src = splus_src / g
    sminus_src = sminus_src / g
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
