"""Numpy model of the radiance kernels' formulation (test-side only).

Mirrors ``pyharp_amd/csrc/hd_rad.hip`` step by step so that a formulation
error can be told apart from a kernel-coding error; checked against the
radiance oracle (``oracle/disort_rad_np.py``) in ``tests/test_kernel_model.py``.
Never imported by the product.

Per azimuthal mode m:
  * the flux kernels' symmetric eigenproblem and flux-weighted R~/T~/S~ with
    the mode-m Legendre table Y_l^m(mu_i), parity split by (l + m), beam source
    scaled by (2 - delta_m0), thermal source only at m = 0;
  * adding sweep + back-substitution that keeps the quadrature intensities
    I+ and I- = R_above I+ + S_down at every level (Lambert surface and top
    emission only at m = 0);
  * layer constants from the level intensities, pivot-free:
      X^-1 = V^T L^-1 diag(g),  Y^-1 = -K^-1 V^T L^T diag(g)   (g = sqrt(w mu))
      C+ = (X^-1 s_top + Y^-1 d_top)/2,  C- = (X^-1 s_bot - Y^-1 d_bot)/2
    with s, d the sum/difference of I+ and I- minus the particular solution;
  * radiance at a user angle by integrating the source function through each
    layer: mode scattering H(+/-k) = c_e . X +/- c_o . Y with
    c_e/o = w * Cu_e/o (the even/odd parts of the mode-m phase row at mu_u).
"""

import math

import numpy as np

from oracle.disort_np import DITHER, double_gauss, plkavg
from oracle.disort_rad_np import lepoly


def layer_rad(dtau, ssa, chi, nstr, m, umu0, fbeam, b_top, b_bot, tauc_top):
    nn = nstr // 2
    mu, w = double_gauss(nn)
    if ssa == 1.0:
        ssa = 1.0 - DITHER
    nmom = len(chi)
    f = chi[nstr - 1] if nmom >= nstr else 0.0
    taup = (1.0 - ssa * f) * dtau
    om = ssa * (1.0 - f) / (1.0 - ssa * f)
    gl = np.array([(2 * l + 1) * om * ((1.0 if l == 0 else (chi[l - 1] if l - 1 < nmom else 0.0))
                                        - f) / (1.0 - f) for l in range(nstr)])
    pt = lepoly(nstr, m, mu)                       # (nstr, nn)
    ev = (np.arange(nstr) + m) % 2 == 0
    splus = (pt[ev].T * gl[ev]) @ pt[ev]
    sminus = (pt[~ev].T * gl[~ev]) @ pt[~ev]
    sd = np.sqrt(w / mu)
    g = np.sqrt(w * mu)
    am = np.diag(1.0 / mu) - sd[:, None] * sminus * sd[None, :]
    ap = np.diag(1.0 / mu) - sd[:, None] * splus * sd[None, :]
    lch = np.linalg.cholesky(am)
    sym = lch.T @ ap @ lch
    k2, v = np.linalg.eigh(sym)
    k = np.sqrt(k2)
    e = np.exp(-k * taup)
    mm = -np.expm1(-k * taup)
    th = mm / (1.0 + e)
    delta = np.where(k * taup > 1e-8, th / np.where(k > 0, k, 1.0), 0.5 * taup)
    gamma = k * th
    omega = (lch @ v) * np.sqrt(delta)[None, :]
    psit = np.linalg.solve(lch.T, v) * np.sqrt(gamma)[None, :]
    jm = np.linalg.cholesky(np.eye(nn) + omega.T @ omega)
    phi = np.linalg.solve(jm, omega.T).T
    qtm = phi @ phi.T
    jp = np.linalg.cholesky(np.eye(nn) + psit.T @ psit)
    xi = np.linalg.solve(jp, psit.T)
    qtp = -(xi.T @ xi)

    def linv(vec):
        z = np.linalg.solve(lch, sd * vec)
        z = np.linalg.solve(lch.T, z)
        return sd * z / w

    zp = np.zeros(nn)
    zm = np.zeros(nn)
    e0 = 1.0
    if fbeam > 0 and umu0 > 0:
        fac = 2.0 - (m == 0)
        e0 = math.exp(-taup / umu0)
        p0 = lepoly(nstr, m, [umu0])[:, 0]
        xs = fac * fbeam / (2 * math.pi) * (pt[ev].T @ (gl[ev] * p0[ev]))
        xd = -fac * fbeam / (2 * math.pi) * (pt[~ev].T @ (gl[~ev] * p0[~ev]))
        rv = -(1.0 / (mu * sd)) * (lch @ (lch.T @ (sd * xs))) + xd / (mu * umu0)
        ttv = v.T @ np.linalg.solve(lch, (w / sd) * rv)
        ttv = ttv / (1.0 / umu0 ** 2 - k2)
        svec = (sd / w) * (lch @ (v @ ttv))
        dd = linv(xd - mu * svec / umu0)
        att = math.exp(-tauc_top / umu0)
        zp = 0.5 * (svec + dd) * att
        zm = 0.5 * (svec - dd) * att
    thermal = m == 0 and (b_top != 0.0 or b_bot != 0.0)
    if thermal:
        bb = b_bot if taup > 0 else b_top
        db = bb - b_top
        slope = db / taup if taup > 0 else 0.0
        hvec = linv(mu)
        cvec = db + 2.0 * slope * hvec
    else:
        db, slope, hvec, cvec = 0.0, 0.0, np.zeros(nn), np.zeros(nn)
        bb = b_top = 0.0
    bsum = b_top + bb
    avec = zm - zp * e0
    bvec = zm + zp * e0
    pv = qtm @ (g * (cvec - avec))
    qv = qtp @ (g * (bvec + bsum))
    sp = g * (zp * (1 - e0) - db) + pv - qv
    sm = g * (-zm * (1 - e0) + db) - pv - qv
    rt = qtm + qtp
    tt = np.eye(nn) - qtm + qtp
    return dict(r=rt * (1 / g)[:, None] * g[None, :], t=tt * (1 / g)[:, None] * g[None, :],
                sp=sp / g, sm=sm / g, taup=taup, om=om, gl=gl, lch=lch, v=v, k=k, zp=zp, zm=zm,
                hvec=hvec, bt=b_top, slope=slope, tau=dtau)


def _part(o, t, umu0, beam):
    """particular solution (I+ , I-) at local depth t of a layer"""
    eb = math.exp(-t / umu0) if beam else 0.0
    b = o["bt"] + o["slope"] * t
    return o["zp"] * eb + b + o["slope"] * o["hvec"], o["zm"] * eb + b - o["slope"] * o["hvec"]


def solve_mode(dtauc, ssalb, chis, nstr, m, umu0=1.0, fbeam=0.0, albedo=0.0, fisot=0.0,
               pk=None, bsurf=0.0, btop=0.0):
    """Layers top->bottom.  Returns (ops, ip (L+1, nn), im (L+1, nn), C+ (L, nn), C- (L, nn))."""
    nn = nstr // 2
    mu, w = double_gauss(nn)
    g = np.sqrt(w * mu)
    nlyr = len(dtauc)
    beam = fbeam > 0 and umu0 > 0
    pk = np.zeros(nlyr + 1) if pk is None else pk
    ops = []
    tauc = 0.0
    for lc in range(nlyr):
        o = layer_rad(dtauc[lc], ssalb[lc], chis[lc], nstr, m, umu0, fbeam if beam else 0.0,
                      pk[lc], pk[lc + 1], tauc)
        o["tauc_top"] = tauc
        tauc += o["taup"]
        ops.append(o)
    alb = albedo if m == 0 else 0.0
    top = (fisot + btop) if m == 0 else 0.0
    ra = np.zeros((nn, nn))
    sd = np.full(nn, top)
    store = []
    for o in ops:
        w1 = np.eye(nn) - o["r"] @ ra
        zt = np.linalg.solve(w1, o["t"])
        t_ = np.linalg.solve(w1, o["r"] @ sd + o["sp"])
        store.append((zt, t_, ra.copy(), sd.copy()))
        u = ra @ t_ + sd
        ra = o["r"] + o["t"] @ (ra @ zt)
        sd = o["t"] @ u + o["sm"]
    esurf = 0.0
    if m == 0:
        if beam:
            esurf += alb * umu0 * fbeam * math.exp(-tauc / umu0) / math.pi
        esurf += (1 - alb) * bsurf
    wm = w * mu
    x = (2 * alb * wm @ sd + esurf) / (1 - 2 * alb * wm @ (ra @ np.ones(nn)))
    ip = np.zeros((nlyr + 1, nn))
    im = np.zeros((nlyr + 1, nn))
    ip[nlyr] = x
    im[nlyr] = ra @ ip[nlyr] + sd
    for lc in range(nlyr - 1, -1, -1):
        zt, t_, ra_l, sd_l = store[lc]
        ip[lc] = zt @ ip[lc + 1] + t_
        im[lc] = ra_l @ ip[lc] + sd_l
    cp = np.zeros((nlyr, nn))
    cm = np.zeros((nlyr, nn))
    for lc, o in enumerate(ops):
        lch, v, k = o["lch"], o["v"], o["k"]
        xinv = lambda s: v.T @ np.linalg.solve(lch, g * s)            # noqa: E731
        yinv = lambda d: -(v.T @ (lch.T @ (g * d))) / k                # noqa: E731
        pp, pm_ = _part(o, 0.0, umu0, beam)
        st, dt = ip[lc] + im[lc] - (pp + pm_), ip[lc] - im[lc] - (pp - pm_)
        pp, pm_ = _part(o, o["taup"], umu0, beam)
        sb, db = ip[lc + 1] + im[lc + 1] - (pp + pm_), ip[lc + 1] - im[lc + 1] - (pp - pm_)
        cp[lc] = 0.5 * (xinv(st) + yinv(dt))
        cm[lc] = 0.5 * (xinv(sb) - yinv(db))
    return ops, ip, im, cp, cm


def _seg_exp(a, c, t1, t2, tref, mu):
    """int_{t1}^{t2} a e^{-c (t - tref)} e^{-(t - t1)/mu} dt/mu, t1 = evaluation point"""
    p1 = math.exp(-c * (t1 - tref))
    den = 1.0 + c * mu
    x = den * (t2 - t1) / mu
    if abs(x) < 0.5:
        ph = 1.0 if x == 0.0 else -math.expm1(-x) / x
        return a * p1 * (t2 - t1) / mu * ph
    p2 = math.exp(-c * (t2 - tref) - (t2 - t1) / mu)
    return a * (p1 - p2) / den


def user_radiance(ops, ip, im, cp, cm, nstr, m, umu_u, utau, umu0=1.0, fbeam=0.0, albedo=0.0,
                  fisot=0.0, bsurf=0.0, btop=0.0):
    """Mode-m radiance at user cosine umu_u for each user depth (unscaled,
    ascending): the march the user-angle kernel does."""
    nn = nstr // 2
    mu, w = double_gauss(nn)
    g = np.sqrt(w * mu)
    sdv = np.sqrt(w / mu)
    nlyr = len(ops)
    beam = fbeam > 0 and umu0 > 0
    fac = 2.0 - (m == 0)
    yu = lepoly(nstr, m, [umu_u])[:, 0]
    y0 = lepoly(nstr, m, [umu0])[:, 0] * np.where((np.arange(nstr) + m) % 2 == 0, 1.0, -1.0)
    ptab = lepoly(nstr, m, mu)
    ev = (np.arange(nstr) + m) % 2 == 0
    taus = np.concatenate([[0.0], np.cumsum([o["tau"] for o in ops])])
    out = np.zeros(len(utau))

    def layer_terms(o, lc):
        cue = 0.5 * (ptab[ev].T @ (o["gl"][ev] * yu[ev]))   # (nn,)
        cuo = 0.5 * (ptab[~ev].T @ (o["gl"][~ev] * yu[~ev]))
        ce = v_t(o, o["lch"].T @ (sdv * cue))
        co = -o["k"] * v_t(o, np.linalg.solve(o["lch"], sdv * cuo))
        hp, hm = ce + co, ce - co
        terms = []
        for j in range(nn):
            terms.append(("exp", cp[lc, j] * hp[j], o["k"][j], 0.0))
            terms.append(("exp", cm[lc, j] * hm[j], -o["k"][j], o["taup"]))
        if beam:
            zs, zd = o["zp"] + o["zm"], o["zp"] - o["zm"]
            x0 = fac * fbeam / (4 * math.pi) * (o["gl"] @ (yu * y0)) * \
                math.exp(-o["tauc_top"] / umu0)
            terms.append(("exp", x0 + w @ (cue * zs + cuo * zd), 1.0 / umu0, 0.0))
        if m == 0 and (o["bt"] != 0.0 or o["slope"] != 0.0):
            ce0 = (1.0 - o["om"]) + 2.0 * (w @ cue)
            a1 = o["slope"] * ce0
            a0 = o["bt"] * ce0 + 2.0 * o["slope"] * (w @ (cuo * o["hvec"]))
            terms.append(("lin", a0, a1, 0.0))
        return terms

    def v_t(o, x):
        return o["v"].T @ x

    def integrate(terms, t1, t2, mu_):
        s = 0.0
        for kind, a, c, tref in terms:
            if kind == "exp":
                s += _seg_exp(a, c, t1, t2, tref, mu_)
            else:
                e2 = math.exp(-(t2 - t1) / mu_)
                s += (a + c * t1 + c * mu_) - (a + c * t2 + c * mu_) * e2
        return s

    if umu_u > 0:
        if m == 0:
            dirb = umu0 * fbeam * math.exp(-sum(o["taup"] for o in ops) / umu0) if beam else 0.0
            fdn = 2 * math.pi * (w * mu) @ im[nlyr]
            cur = albedo / math.pi * (fdn + dirb) + (1 - albedo) * bsurf
        else:
            cur = 0.0
        k = len(utau) - 1
        for lc in range(nlyr - 1, -1, -1):
            o = ops[lc]
            terms = layer_terms(o, lc)
            scale = o["taup"] / o["tau"] if o["tau"] > 0 else 0.0
            while k >= 0 and utau[k] >= taus[lc]:
                t = (utau[k] - taus[lc]) * scale
                out[k] = cur * math.exp(-(o["taup"] - t) / umu_u) + \
                    integrate(terms, t, o["taup"], umu_u)
                k -= 1
            cur = cur * math.exp(-o["taup"] / umu_u) + integrate(terms, 0.0, o["taup"], umu_u)
    else:
        cur = (fisot + btop) if m == 0 else 0.0
        k = 0
        for lc in range(nlyr):
            o = ops[lc]
            terms = layer_terms(o, lc)
            scale = o["taup"] / o["tau"] if o["tau"] > 0 else 0.0
            while k < len(utau) and utau[k] <= taus[lc + 1]:
                t = (utau[k] - taus[lc]) * scale
                out[k] = cur * math.exp(t / umu_u) + integrate(terms, t, 0.0, umu_u)
                k += 1
            cur = cur * math.exp(o["taup"] / umu_u) + integrate(terms, o["taup"], 0.0, umu_u)
    return out
