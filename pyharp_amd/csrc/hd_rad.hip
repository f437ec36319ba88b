// hd_rad.hip -- gfx950 kernels of the intensity path: every azimuthal mode,
// fluxes at user optical depths (usrtau) and radiances at user angles
// (usrang), nstr <= 32.  One lane owns one (solve, mode m) problem ("unit");
// units are mode-major inside a chunk (u = m*ns + sl), so a wave's lanes share
// m and the mode-m Legendre tables are uniform loads.
//
//   hd_rad_taus_kernel       unscaled depth of every level (cumsum from the top)
//   hd_rad_layer_kernel<NN>  per (unit, layer): the flux kernel's layer setup
//                            with the mode-m table Y_l^m(mu_i), parity split by
//                            (l+m), beam source x (2 - delta_m0), thermal only at
//                            m = 0; also keeps L, V, k and the particular
//                            solution for the radiance kernels  [c_soleig,
//                            c_upbeam, c_upisot per mode]
//   hd_rad_sweep_kernel<NN>  per unit: adding sweep (Lambert surface and top
//                            emission only at m = 0) and back-substitution that
//                            keeps I+ and I- at every level   [c_setmtx, c_solve0]
//   hd_rad_const_kernel<NN>  per (unit, layer): the layer's homogeneous
//                            constants from its level intensities, pivot-free
//   hd_rad_flux_kernel<NN>   per (solve, user depth): fluxes from the m = 0
//                            field inside the layer                 [c_fluxes]
//   hd_rad_user_kernel<NN>   per (unit, user angle): source-function integration
//                            along the ray through every layer       [c_usrint]
//   hd_rad_azimuth_kernel    uu = sum_m I_m cos(m (phi - phi0))
//
// Formulation: DESIGN.md section 3b, mirrored in numpy by
// tests/kernel_model_rad.py; oracle: oracle/disort_rad_np.py.
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "hd_rad.hpp"

namespace hd {
#ifdef HD_RAD_WIDE
namespace wide {
#endif

namespace {

constexpr int kLayerBlockR = 256;
// the layer kernel's records (operators for the sweep, radiance records for the const,
// flux and user kernels): whole-line stores, read a kernel later -- nontemporal
#ifndef HD_RAD_NT
#define HD_RAD_NT 1
#endif
constexpr bool kRadNt = HD_RAD_NT != 0;
constexpr int kLayersPerBlockR = kLayerBlockR / 64;

// nstr <= 16 (NN <= 8, this translation unit): every NN-loop fully unrolled,
// the matrices in registers.  nstr 18..32 (NN 9..16): hd_rad_wide.hip compiles
// this same file with the NN-loops rolled (HD_RUNROLL = nounroll), so the
// per-lane matrices live in private memory -- the coverage path of the
// intensity kernels at large nstr (the flux path has the team kernels)
#ifndef HD_RUNROLL
#define HD_RUNROLL _Pragma("unroll")
#endif
// rrd addressing in the const / flux / user kernels: [layer][element][unit] (unit
// fastest: the one-lane kernels' coalesced layout) at nstr <= 16; at nstr 18..32 the
// team kernels (hd_team_mfma.hip) write and read it, and it is [layer][unit][element]
// (a team's accesses to one unit's record share lines)
#ifdef HD_RAD_WIDE
#define HD_RREC(lc, u) (A.rrd + ((size_t)(lc) * nu + (u)) * rad_rec_doubles(NN))
#define HD_RS ((size_t)1)
#else
#define HD_RREC(lc, u) (A.rrd + (size_t)(lc) * rad_rec_doubles(NN) * nu + (u))
#define HD_RS nu
#endif

template <int NN>
struct RadTab {
  double lam[2 * NN][2 * NN][NN];  // Y_l^m(mu_i): [m][l][i]
};

struct RadConst {
  Quad<1> q1;
  Quad<2> q2;
  Quad<3> q3;
  Quad<4> q4;
  Quad<5> q5;
  Quad<6> q6;
  Quad<7> q7;
  Quad<8> q8;
  RadTab<1> t1;
  RadTab<2> t2;
  RadTab<3> t3;
  RadTab<4> t4;
  RadTab<5> t5;
  RadTab<6> t6;
  RadTab<7> t7;
  RadTab<8> t8;
  double seed[2 * kRadMaxNN];                // prod_{i<=m} sqrt((2i-1)/(2i))
  double ra[2 * kRadMaxNN][2 * kRadMaxNN];   // [m][l] (2l-1)/sqrt(l^2-m^2), l > m
  double rb[2 * kRadMaxNN][2 * kRadMaxNN];   // [m][l] sqrt((l-1)^2-m^2)/sqrt(l^2-m^2)
};
__constant__ RadConst c_rad;

#ifdef HD_RAD_WIDE
struct RadConstWide {
  Quad<9> q9;
  Quad<10> q10;
  Quad<11> q11;
  Quad<12> q12;
  Quad<13> q13;
  Quad<14> q14;
  Quad<15> q15;
  Quad<16> q16;
  RadTab<9> t9;
  RadTab<10> t10;
  RadTab<11> t11;
  RadTab<12> t12;
  RadTab<13> t13;
  RadTab<14> t14;
  RadTab<15> t15;
  RadTab<16> t16;
};
__constant__ RadConstWide c_radw;
#endif

template <int NN>
__device__ __forceinline__ const Quad<NN>& quad_r() {
  if constexpr (NN == 1) return c_rad.q1;
  else if constexpr (NN == 2) return c_rad.q2;
  else if constexpr (NN == 3) return c_rad.q3;
  else if constexpr (NN == 4) return c_rad.q4;
  else if constexpr (NN == 5) return c_rad.q5;
  else if constexpr (NN == 6) return c_rad.q6;
  else if constexpr (NN == 7) return c_rad.q7;
  else if constexpr (NN == 8) return c_rad.q8;
#ifdef HD_RAD_WIDE
  else if constexpr (NN == 9) return c_radw.q9;
  else if constexpr (NN == 10) return c_radw.q10;
  else if constexpr (NN == 11) return c_radw.q11;
  else if constexpr (NN == 12) return c_radw.q12;
  else if constexpr (NN == 13) return c_radw.q13;
  else if constexpr (NN == 14) return c_radw.q14;
  else if constexpr (NN == 15) return c_radw.q15;
  else return c_radw.q16;
#endif
}
template <int NN>
__device__ __forceinline__ const RadTab<NN>& tab_r() {
  if constexpr (NN == 1) return c_rad.t1;
  else if constexpr (NN == 2) return c_rad.t2;
  else if constexpr (NN == 3) return c_rad.t3;
  else if constexpr (NN == 4) return c_rad.t4;
  else if constexpr (NN == 5) return c_rad.t5;
  else if constexpr (NN == 6) return c_rad.t6;
  else if constexpr (NN == 7) return c_rad.t7;
  else if constexpr (NN == 8) return c_rad.t8;
#ifdef HD_RAD_WIDE
  else if constexpr (NN == 9) return c_radw.t9;
  else if constexpr (NN == 10) return c_radw.t10;
  else if constexpr (NN == 11) return c_radw.t11;
  else if constexpr (NN == 12) return c_radw.t12;
  else if constexpr (NN == 13) return c_radw.t13;
  else if constexpr (NN == 14) return c_radw.t14;
  else if constexpr (NN == 15) return c_radw.t15;
  else return c_radw.t16;
#endif
}

// Y_m^m(x) = seed_m (1 - x^2)^(m/2)
__device__ __forceinline__ double ylm_seed(int m, double x) {
  const double s = sqrt(fmax(0.0, 1.0 - x * x));
  double p = c_rad.seed[m];
  for (int i = 0; i < m; ++i) p *= s;
  return p;
}

// Y_l^m(x), l < N (compile-time l, runtime m)
template <int N>
__device__ __forceinline__ void ylm_row(int m, double x, double (&y)[N]) {
  const double seed = ylm_seed(m, x);
  double y1 = 0.0, y2 = 0.0;
#pragma unroll
  for (int l = 0; l < N; ++l) {
    const double v =
        l < m ? 0.0 : (l == m ? seed : fma(c_rad.ra[m][l] * x, y1, -c_rad.rb[m][l] * y2));
    y[l] = v;
    y2 = y1;
    y1 = v;
  }
}

__device__ __forceinline__ void flag(const RadArgs& A, long s, int st) {
  if (st) {
    atomicOr(&A.status[s], st);
    if (st & 0x0F) atomicOr(A.anyerr, 1);
  }
}


}  // namespace

// ============================================================================
// unscaled depth of every level, solver order (0 = top)
// ============================================================================
__global__ __launch_bounds__(256) void hd_rad_taus_kernel(RadArgs A) {
  const int sl = blockIdx.x * blockDim.x + threadIdx.x;
  if (sl >= A.ns) return;
  const long s = A.s0 + sl;
  const int L = A.nlyr, np = A.nprop;
  const double* p = A.prop + (size_t)s * L * np;
  double t = 0.0;
  A.taus[sl] = 0.0;
  for (int lc = 0; lc < L; ++lc) {
    t += p[(size_t)(L - 1 - lc) * np];
    A.taus[(size_t)(lc + 1) * A.ns + sl] = t;
  }
  if (A.utau && A.ntau > 0 && A.utau[A.ntau - 1] > t * (1.0 + 1e-12) + 1e-300)
    flag(A, s, kStBadInput);  // user depth below the bottom
}

// ============================================================================
// per-(unit, layer) setup (hd_layer_kernel generalised to mode m)
// ============================================================================
template <int NN>
__global__ __launch_bounds__(kLayerBlockR) void hd_rad_layer_kernel(RadArgs A) {
  constexpr int N = 2 * NN;
  constexpr int kPsi = NN > 1 ? NN * NN : 1;
  constexpr int nsym = NN * (NN + 1) / 2;
  __shared__ double psi_lds[NN <= 8 ? kPsi * kLayerBlockR : 1];
  double psi_priv[NN <= 8 ? 1 : kPsi];  // NN > 8: private memory, like the matrices
  auto psi_at = [&](int e) -> double& {
    if constexpr (NN <= 8) return psi_lds[e * kLayerBlockR + threadIdx.x];
    else return psi_priv[e];
  };
  const Quad<NN>& Qc = quad_r<NN>();
  const int lt = threadIdx.x;
  const int ntile = (A.nu + 63) / 64;
  const int ts = blockIdx.x % ntile;
  const int tl = blockIdx.x / ntile;
  const int u = ts * 64 + (lt & 63);
  const int lc = tl * kLayersPerBlockR + (lt >> 6);
  const int L = A.nlyr;
  if (u >= A.nu || lc >= L) return;
  const int m = u / A.ns;
  const int sl = u - m * A.ns;
  const long s = A.s0 + sl;
  const size_t nu = A.nu;
  const int nm = A.nmom;
  const int np = A.nprop;
  int st = 0;

  const double* q = A.prop + ((size_t)s * L + (L - 1 - lc)) * np;
  const double tau = q[0];
  double ssa = np > 1 ? q[1] : 0.0;
  if (!(tau >= 0.0) || !(ssa >= 0.0) || !(ssa <= 1.0)) st |= kStBadInput;
  if (ssa == 1.0) ssa = 1.0 - kDither;
  const double f = nm >= N ? q[1 + N] : 0.0;
  if (!(f < 1.0)) st |= kStBadInput;
  const double taup = (1.0 - ssa * f) * tau;
  const double om = ssa * (1.0 - f) / (1.0 - ssa * f);
  const double rf = om / (1.0 - f);

  const double mu0 = A.umu0 ? A.umu0[s] : 1.0;
  const double fb = A.fbeam ? A.fbeam[s] : 0.0;
  const bool beam = fb > 0.0 && mu0 > 0.0;
  if (fb > 0.0 && !(mu0 > 0.0 && mu0 <= 1.0)) st |= kStBadInput;  // cdisort c_chekin
  const double rmu0 = beam ? 1.0 / mu0 : 0.0;
  const double mub = beam ? mu0 : 0.0;
  const bool therm = A.planck && m == 0;

  // ---- mode-m phase matrix even/odd parts (parity of l+m) + beam vectors ----
  double lch[NN][NN], ap[NN][NN], xs[NN], xd[NN];
HD_RUNROLL
  for (int i = 0; i < NN; ++i) {
    xs[i] = xd[i] = 0.0;
HD_RUNROLL
    for (int j = i; j < NN; ++j) lch[i][j] = ap[i][j] = 0.0;
  }
  {
    const int mp = m & 1;
    const double* lam = &tab_r<NN>().lam[m][0][0];
    const double seed = ylm_seed(m, mub);
    double y1 = 0.0, y2 = 0.0;  // Y_{l-1}^m(mu0), Y_{l-2}^m(mu0)
    // Y_l^m = 0 for l < m (tables and recurrence): the pairs below m/2 add exact zeros
#pragma nounroll
    for (int l2 = m >> 1; l2 < NN; ++l2) {
      const int la = 2 * l2, lb = la + 1;
      const double ya =
          la < m ? 0.0 : (la == m ? seed : fma(c_rad.ra[m][la] * mub, y1, -c_rad.rb[m][la] * y2));
      y2 = y1;
      y1 = ya;
      const double yb =
          lb < m ? 0.0 : (lb == m ? seed : fma(c_rad.ra[m][lb] * mub, y1, -c_rad.rb[m][lb] * y2));
      y2 = y1;
      y1 = yb;
      const int le = mp ? lb : la, lo = mp ? la : lb;
      const double pe0 = mp ? yb : ya, po0 = mp ? ya : yb;
      const double che = le == 0 ? 1.0 : (le <= nm ? q[1 + le] : 0.0);
      const double cho = lo == 0 ? 1.0 : (lo <= nm ? q[1 + lo] : 0.0);
      const double ge = (2 * le + 1) * (che - f) * rf;
      const double go = (2 * lo + 1) * (cho - f) * rf;
      const double* te = lam + le * NN;
      const double* to = lam + lo * NN;
      double ue[NN], uo[NN];
HD_RUNROLL
      for (int i = 0; i < NN; ++i) {
        ue[i] = ge * te[i];
        uo[i] = go * to[i];
        xs[i] = fma(ue[i], pe0, xs[i]);
        xd[i] = fma(uo[i], po0, xd[i]);
      }
HD_RUNROLL
      for (int i = 0; i < NN; ++i)
HD_RUNROLL
        for (int j = i; j < NN; ++j) {
          ap[i][j] = fma(ue[i], te[j], ap[i][j]);
          lch[i][j] = fma(uo[i], to[j], lch[i][j]);
        }
    }
  }
HD_RUNROLL
  for (int i = 0; i < NN; ++i)
HD_RUNROLL
    for (int j = i; j < NN; ++j) {
      const double diag = (i == j) ? Qc.rmu[i] : 0.0;
      const double sij = Qc.sd[i] * Qc.sd[j];
      lch[i][j] = fma(-sij, lch[i][j], diag);
      ap[i][j] = fma(-sij, ap[i][j], diag);
    }
  double rdl[NN];
  if (!chol_inplace<NN>(lch, rdl)) st |= kStEigen;

  double* rr = A.rrd + (size_t)lc * rad_rec_doubles(NN) * nu + u;
  constexpr int oV = nsym, oK = nsym + NN * NN, oZp = oK + NN, oZm = oZp + NN, oH = oZm + NN;
  constexpr int oBt = oH + NN, oSl = oBt + 1, oTp = oSl + 1, oOm = oTp + 1, oEk = oOm + 1;
  constexpr int oE0 = oEk + NN;

  double y2[NN], lxd[NN];
  const double fb2 = fb * ((m == 0 ? 0.5 : 1.0) / kPi);
  if (beam) {
    double y[NN], z[NN];
HD_RUNROLL
    for (int i = 0; i < NN; ++i) y[i] = Qc.sd[i] * (fb2 * xs[i]);
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
      double t = 0.0;
HD_RUNROLL
      for (int k = i; k < NN; ++k) t = fma(lch[k][i], y[k], t);
      z[i] = t;
    }
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
      double t = 0.0;
HD_RUNROLL
      for (int k = 0; k <= i; ++k) t = fma(lch[i][k], z[k], t);
      y[i] = t;
    }
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
      const double xdi = -fb2 * xd[i];
      const double rv = fma(-y[i], Qc.rg[i], xdi * rmu0 * Qc.rmu[i]);
      y2[i] = Qc.g[i] * rv;
      lxd[i] = Qc.sd[i] * xdi;
    }
    lower_solve<NN>(lch, rdl, y2);  // V^T y2 below
    lower_solve<NN>(lch, rdl, lxd);
    lower_t_solve<NN>(lch, rdl, lxd);
  } else {
HD_RUNROLL
    for (int i = 0; i < NN; ++i) y2[i] = lxd[i] = 0.0;
  }
  // thermal (m = 0): cvec = dB + 2 (dB/tau') h,  h = W^-1 D^1/2 L^-T L^-1 D^1/2 mu
  double cvec[NN];
  double db = 0.0, bsum = 0.0;
  if (therm) {
    const double bt = A.planckv[(size_t)(L - lc) * A.ns + sl];
    const double bb = taup > 0.0 ? A.planckv[(size_t)(L - lc - 1) * A.ns + sl] : bt;
    db = bb - bt;
    bsum = bt + bb;
    const double b1 = taup > 0.0 ? 2.0 * db / taup : 0.0;
HD_RUNROLL
    for (int i = 0; i < NN; ++i) cvec[i] = Qc.sd[i] * Qc.mu[i];
    lower_solve<NN>(lch, rdl, cvec);
    lower_t_solve<NN>(lch, rdl, cvec);
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
      rec_st<kRadNt>(&rr[(oH + i) * nu], Qc.rg[i] * cvec[i]);
      cvec[i] = fma(b1 * Qc.rg[i], cvec[i], db);
    }
    rec_st<kRadNt>(&rr[oBt * nu], bt);
    rec_st<kRadNt>(&rr[oSl * nu], 0.5 * b1);
  } else {
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
      cvec[i] = 0.0;
      rec_st<kRadNt>(&rr[(oH + i) * nu], 0.0);
    }
    rec_st<kRadNt>(&rr[oBt * nu], 0.0);
    rec_st<kRadNt>(&rr[oSl * nu], 0.0);
  }
  rec_st<kRadNt>(&rr[oTp * nu], taup);
  rec_st<kRadNt>(&rr[oOm * nu], om);
  {  // L (packed lower, row-major)
    int e = 0;
HD_RUNROLL
    for (int i = 0; i < NN; ++i)
HD_RUNROLL
      for (int k = 0; k <= i; ++k) rec_st<kRadNt>(&rr[(e++) * nu], lch[i][k]);
  }

  // ---- eigenpairs (hd_layer_kernel's form): C C^T = -A+, X = L^T C, Sym = X X^T;
  // the one-sided Jacobi on X's columns gives B = X W with k_j = |b_j| and
  // V = B K^-1 (stored for the later kernels), U = L V ----
  double rdc[NN];
  if (!chol_inplace<NN>(ap, rdc)) st |= kStEigen;  // lower ap <- C
  double v[NN][NN];  // X, then B, then V, then Omega = L V Delta^1/2
HD_RUNROLL
  for (int i = 0; i < NN; ++i)
HD_RUNROLL
    for (int j = 0; j < NN; ++j) {  // X_ij = sum_{k >= max(i,j)} L_ki C_kj
      double t = 0.0;
HD_RUNROLL
      for (int k = (i > j ? i : j); k < NN; ++k) t = fma(lch[k][i], ap[k][j], t);
      v[i][j] = t;
    }
  if (!jacobi_os<NN>(v, A.max_sweeps)) st |= kStEigen;
  jacobi_os_polish<NN>(v, beam && near_resonance<NN>(v, rmu0 * rmu0, kResPolish));
  double kk[NN];
HD_RUNROLL
  for (int j = 0; j < NN; ++j) {
    double k2 = 0.0;
HD_RUNROLL
    for (int i = 0; i < NN; ++i) k2 = fma(v[i][j], v[i][j], k2);
    if (!(k2 > 0.0)) st |= kStEigen;
    const double rk = k2 > 0.0 ? rsq_nr(k2) : 0.0;
    kk[j] = k2 * rk;
    rec_st<kRadNt>(&rr[(oK + j) * nu], kk[j]);
HD_RUNROLL
    for (int i = 0; i < NN; ++i) v[i][j] *= rk;  // V = B K^-1
  }

  // ---- beam particular solution at the layer top ----
  double zp[NN], zm[NN];
  double e0 = 0.0;
  if (beam) {
    double tt[NN];
    const double r2 = rmu0 * rmu0;
HD_RUNROLL
    for (int j = 0; j < NN; ++j) {  // tt = V^T y2 / (1/mu0^2 - k^2)
      double t = 0.0;
HD_RUNROLL
      for (int i = 0; i < NN; ++i) t = fma(v[i][j], y2[i], t);
      double den = fma(-kk[j], kk[j], r2);
      if (fabs(den) < 1.0e-9 * r2) {
        st |= kStResonance;
        den = den < 0.0 ? -1.0e-9 * r2 : 1.0e-9 * r2;
      }
      tt[j] = t / den;
    }
    double sv[NN], y[NN];
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {  // V tt
      double t = 0.0;
HD_RUNROLL
      for (int j = 0; j < NN; ++j) t = fma(v[i][j], tt[j], t);
      y[i] = t;
    }
HD_RUNROLL
    for (int i = NN - 1; i >= 0; --i) {  // s = W^-1 D^1/2 L V tt
      double t = 0.0;
HD_RUNROLL
      for (int k = 0; k <= i; ++k) t = fma(lch[i][k], y[k], t);
      sv[i] = Qc.rg[i] * t;
    }
HD_RUNROLL
    for (int i = 0; i < NN; ++i) y[i] = Qc.sd[i] * Qc.mu[i] * sv[i];
    lower_solve<NN>(lch, rdl, y);
    lower_t_solve<NN>(lch, rdl, y);
    const double tauc = A.tauc[(size_t)lc * A.ns + sl];
    const double att = 0.5 * exp(-tauc * rmu0);
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
      const double dd = Qc.rg[i] * fma(-y[i], rmu0, lxd[i]);
      zp[i] = (sv[i] + dd) * att;
      zm[i] = (sv[i] - dd) * att;
    }
    e0 = exp(-taup * rmu0);
  } else {
HD_RUNROLL
    for (int i = 0; i < NN; ++i) zp[i] = zm[i] = 0.0;
  }
HD_RUNROLL
  for (int i = 0; i < NN; ++i) {
    rec_st<kRadNt>(&rr[(oZp + i) * nu], zp[i]);
    rec_st<kRadNt>(&rr[(oZm + i) * nu], zm[i]);
  }

  // ---- layer operators in the flux-weighted basis (as hd_layer_kernel) ----
  double dsq[NN], gsq[NN];
HD_RUNROLL
  for (int j = 0; j < NN; ++j) {
    const double x = kk[j] * taup;
    const double mm = -expm1(-x);
    const double th = mm * rcp_nr(2.0 - mm);
    const double delta = x > 1.0e-8 ? th * rcp_nr(kk[j] > 0.0 ? kk[j] : 1.0) : 0.5 * taup;
    dsq[j] = sqrt(delta);
    gsq[j] = sqrt(kk[j] * th);
    rec_st<kRadNt>(&rr[(oEk + j) * nu], 1.0 - mm);  // exp(-k tau') for the user-angle kernel
  }
  rec_st<kRadNt>(&rr[oE0 * nu], e0);
HD_RUNROLL
  for (int j = 0; j < NN; ++j) {  // V (stored), Psi^T = L^-T V Gamma^1/2 -> LDS
    double x[NN];
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
      rec_st<kRadNt>(&rr[(oV + i * NN + j) * nu], v[i][j]);
      x[i] = v[i][j] * gsq[j];
    }
    lower_t_solve<NN>(lch, rdl, x);
HD_RUNROLL
    for (int i = 0; i < NN; ++i) psi_at(i * NN + j) = x[i];
  }
HD_RUNROLL
  for (int j = 0; j < NN; ++j)  // Omega = L V Delta^1/2, in place (rows bottom-up)
HD_RUNROLL
    for (int i = 0; i < NN; ++i) v[i][j] *= dsq[j];
HD_RUNROLL
  for (int i = NN - 1; i >= 0; --i)
HD_RUNROLL
    for (int j = 0; j < NN; ++j) {
      double t = 0.0;
HD_RUNROLL
      for (int k = 0; k <= i; ++k) t = fma(lch[i][k], v[k][j], t);
      v[i][j] = t;
    }

  double* out = A.rsw + (size_t)lc * ne1<NN>() * nu + u;
  double ga[NN], gb[NN];
HD_RUNROLL
  for (int i = 0; i < NN; ++i) {
    ga[i] = Qc.g[i] * (cvec[i] - fma(-zp[i], e0, zm[i]));
    gb[i] = Qc.g[i] * (fma(zp[i], e0, zm[i]) + bsum);
  }
  // Woodbury (as hd_layer_kernel): Q~- = I - A-, Q~+ = A+ - I with
  // A- = (I + Omega Omega^T)^-1, A+ = (I + Psi^T Psi)^-1; R~ = A+ - A-, T~ = A- + A+ - I
  double pvec[NN], am_[NN][NN];
  {
HD_RUNROLL
    for (int i = 0; i < NN; ++i)
HD_RUNROLL
      for (int j = i; j < NN; ++j) {
        double t = (i == j) ? 1.0 : 0.0;
HD_RUNROLL
        for (int k = 0; k < NN; ++k) t = fma(v[i][k], v[j][k], t);
        am_[i][j] = t;
      }
    double rdh[NN];
    if (!chol_inplace<NN>(am_, rdh)) st |= kStEigen;
    spd_inverse_upper<NN>(am_, rdh);
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {  // p = Q~- ga = ga - A- ga
      double t = ga[i];
HD_RUNROLL
      for (int j = 0; j < NN; ++j) t = fma(-HD_SYM(am_, i, j), ga[j], t);
      pvec[i] = t;
    }
  }
  double ap_[NN][NN], qvec[NN];
  {
    double pt_[NN][NN];  // pt_[i][j] = Psi^T[i][j]
HD_RUNROLL
    for (int i = 0; i < NN; ++i)
HD_RUNROLL
      for (int j = 0; j < NN; ++j) pt_[i][j] = psi_at(i * NN + j);
HD_RUNROLL
    for (int i = 0; i < NN; ++i)
HD_RUNROLL
      for (int j = i; j < NN; ++j) {
        double t = (i == j) ? 1.0 : 0.0;
HD_RUNROLL
        for (int k = 0; k < NN; ++k) t = fma(pt_[i][k], pt_[j][k], t);
        ap_[i][j] = t;
      }
    double rdh[NN];
    if (!chol_inplace<NN>(ap_, rdh)) st |= kStEigen;
    spd_inverse_upper<NN>(ap_, rdh);
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {  // q = Q~+ gb = A+ gb - gb
      double t = -gb[i];
HD_RUNROLL
      for (int j = 0; j < NN; ++j) t = fma(HD_SYM(ap_, i, j), gb[j], t);
      qvec[i] = t;
    }
  }
  double chk = 0.0;
  {
    int e = 0;
HD_RUNROLL
    for (int i = 0; i < NN; ++i)
HD_RUNROLL
      for (int j = i; j < NN; ++j) {
        const double r = ap_[i][j] - am_[i][j];
        const double t = (am_[i][j] + ap_[i][j]) - ((i == j) ? 1.0 : 0.0);
        rec_st<kRadNt>(&out[e * nu], r);
        rec_st<kRadNt>(&out[(nsym + e) * nu], t);
        chk += r + t;
        ++e;
      }
  }
HD_RUNROLL
  for (int i = 0; i < NN; ++i) {
    const double sp = Qc.g[i] * (zp[i] * (1.0 - e0) - db) + pvec[i] - qvec[i];
    const double sm = Qc.g[i] * (-zm[i] * (1.0 - e0) + db) - pvec[i] - qvec[i];
    rec_st<kRadNt>(&out[(2 * nsym + i) * nu], sp);
    rec_st<kRadNt>(&out[(2 * nsym + NN + i) * nu], sm);
    chk += sp + sm;
  }
  rec_st<kRadNt>(&out[(2 * nsym + 2 * NN) * nu], taup);
  if (!isfinite(chk + taup)) st |= kStNonFinite;
  flag(A, s, st);
}

// ============================================================================
// per-unit adding sweep + back-substitution keeping I+/I- at every level
// ============================================================================
template <int NN>
#ifndef HD_RAD_SWEEP_WAVES
#define HD_RAD_SWEEP_WAVES 1
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(HD_RAD_SWEEP_WAVES)))
void hd_rad_sweep_kernel(RadArgs A) {
  const Quad<NN>& Qc = quad_r<NN>();
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= A.nu) return;
  const int m = u / A.ns;
  const int sl = u - m * A.ns;
  const long s = A.s0 + sl;
  const int L = A.nlyr;
  const size_t nu = A.nu;
  constexpr int nsym = NN * (NN + 1) / 2;
  constexpr int NB = rad_bsub_doubles(NN);
  int st = 0;

  const double mu0 = A.umu0 ? A.umu0[s] : 1.0;
  const double fb = A.fbeam ? A.fbeam[s] : 0.0;
  const bool beam = fb > 0.0 && mu0 > 0.0;
  double alb = A.albedo ? A.albedo[s] : 0.0;
  if (!(alb >= 0.0) || !(alb <= 1.0)) st |= kStBadInput;
  double top = A.fisot ? A.fisot[s] : 0.0;
  double bsurf = 0.0;
  if (A.planck) {
    bsurf = A.planckv[(size_t)(L + 1) * A.ns + sl];
    top += A.planckv[(size_t)(L + 2) * A.ns + sl];
  }
  if (m > 0) alb = top = bsurf = 0.0;  // Lambert surface, isotropic top: mode 0 only
  const double rmu0 = beam ? 1.0 / mu0 : 0.0;
  const double f0mu0 = (beam && m == 0) ? fb * mu0 : 0.0;

  double ra[NN][NN];
  double sd[NN];
HD_RUNROLL
  for (int i = 0; i < NN; ++i) {
    sd[i] = Qc.g[i] * top;
HD_RUNROLL
    for (int j = i; j < NN; ++j) ra[i][j] = 0.0;
  }
  double tauc = 0.0;
  for (int lc = 0; lc < L; ++lc) {
    const double* lp = A.rsw + (size_t)lc * ne1<NN>() * nu + u;
    double* bp = A.bsub + (size_t)lc * NB * nu + u;
    {  // stack above this layer: R_above (packed upper) and S_down
      int e = 0;
HD_RUNROLL
      for (int i = 0; i < NN; ++i)
HD_RUNROLL
        for (int j = i; j < NN; ++j) bp[(NN * NN + NN + (e++)) * nu] = ra[i][j];
HD_RUNROLL
      for (int i = 0; i < NN; ++i) bp[(NN * NN + NN + nsym + i) * nu] = sd[i];
    }
    double rl[NN][NN], spl[NN];
    {
      int e = 0;
HD_RUNROLL
      for (int i = 0; i < NN; ++i)
HD_RUNROLL
        for (int j = i; j < NN; ++j) rl[i][j] = lp[(size_t)(e++) * nu];
HD_RUNROLL
      for (int i = 0; i < NN; ++i) spl[i] = lp[(size_t)(2 * nsym + i) * nu];
    }
    double am[NN][NN], w1[NN][NN], t1[NN];
HD_RUNROLL
    for (int i = 0; i < NN; ++i)
HD_RUNROLL
      for (int j = 0; j < NN; ++j) am[i][j] = HD_SYM(ra, i, j);
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
HD_RUNROLL
      for (int j = 0; j < NN; ++j) {
        double t = (i == j) ? 1.0 : 0.0;
HD_RUNROLL
        for (int k = 0; k < NN; ++k) t = fma(-HD_SYM(rl, i, k), am[k][j], t);
        w1[i][j] = t;
      }
      double t = spl[i];
HD_RUNROLL
      for (int k = 0; k < NN; ++k) t = fma(HD_SYM(rl, i, k), sd[k], t);
      t1[i] = t;
    }
HD_RUNROLL
    for (int k = 0; k < NN; ++k) {
      const double piv = w1[k][k];
      if (!(fabs(piv) > 1.0e-12)) st |= kStPivot;
      const double rp = rcp_nr(piv);
      w1[k][k] = rp;
HD_RUNROLL
      for (int i = k + 1; i < NN; ++i) {
        const double l = w1[i][k] * rp;
        w1[i][k] = l;
HD_RUNROLL
        for (int j = k + 1; j < NN; ++j) w1[i][j] = fma(-l, w1[k][j], w1[i][j]);
      }
    }
HD_RUNROLL
    for (int i = 0; i < NN; ++i)
HD_RUNROLL
      for (int k = 0; k < i; ++k) t1[i] = fma(-w1[i][k], t1[k], t1[i]);
HD_RUNROLL
    for (int i = NN - 1; i >= 0; --i) {
HD_RUNROLL
      for (int k = i + 1; k < NN; ++k) t1[i] = fma(-w1[i][k], t1[k], t1[i]);
      t1[i] *= w1[i][i];
    }
    double uvec[NN];
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
      double t = sd[i];
HD_RUNROLL
      for (int k = 0; k < NN; ++k) t = fma(am[i][k], t1[k], t);
      uvec[i] = t;
      bp[(size_t)(NN * NN + i) * nu] = t1[i];
    }
HD_RUNROLL
    for (int r = 0; r < NN; ++r) {
HD_RUNROLL
      for (int j = 0; j < NN; ++j) {
        double t = am[r][j];
HD_RUNROLL
        for (int k = 0; k < j; ++k) t = fma(-am[r][k], w1[k][j], t);
        am[r][j] = t * w1[j][j];
      }
HD_RUNROLL
      for (int j = NN - 1; j >= 0; --j) {
        double t = am[r][j];
HD_RUNROLL
        for (int k = j + 1; k < NN; ++k) t = fma(-am[r][k], w1[k][j], t);
        am[r][j] = t;
      }
    }
    double tl[NN][NN];
    {
      int e = nsym;
HD_RUNROLL
      for (int i = 0; i < NN; ++i)
HD_RUNROLL
        for (int j = i; j < NN; ++j) tl[i][j] = lp[(size_t)(e++) * nu];
    }
HD_RUNROLL
    for (int j = 0; j < NN; ++j) {
      double x[NN];
HD_RUNROLL
      for (int i = 0; i < NN; ++i) x[i] = HD_SYM(tl, i, j);
HD_RUNROLL
      for (int i = 0; i < NN; ++i)
HD_RUNROLL
        for (int k = 0; k < i; ++k) x[i] = fma(-w1[i][k], x[k], x[i]);
HD_RUNROLL
      for (int i = NN - 1; i >= 0; --i) {
HD_RUNROLL
        for (int k = i + 1; k < NN; ++k) x[i] = fma(-w1[i][k], x[k], x[i]);
        x[i] *= w1[i][i];
      }
HD_RUNROLL
      for (int i = 0; i < NN; ++i) bp[(size_t)(i * NN + j) * nu] = x[i];
    }
HD_RUNROLL
    for (int r = 0; r < NN; ++r) {
      double row[NN];
HD_RUNROLL
      for (int j = 0; j < NN; ++j) {
        double t = 0.0;
HD_RUNROLL
        for (int k = 0; k < NN; ++k) t = fma(am[r][k], HD_SYM(tl, k, j), t);
        row[j] = t;
      }
HD_RUNROLL
      for (int j = 0; j < NN; ++j) am[r][j] = row[j];
    }
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
HD_RUNROLL
      for (int j = i; j < NN; ++j) {
        double t = rl[i][j];
HD_RUNROLL
        for (int k = 0; k < NN; ++k) t = fma(HD_SYM(tl, i, k), am[k][j], t);
        ra[i][j] = t;
      }
      double t = lp[(size_t)(2 * nsym + NN + i) * nu];
HD_RUNROLL
      for (int k = 0; k < NN; ++k) t = fma(HD_SYM(tl, i, k), uvec[k], t);
      sd[i] = t;
    }
    tauc += lp[(size_t)(2 * nsym + 2 * NN) * nu];
  }

  // ---- Lambertian surface (mode 0): I+ = x for every stream ----
  double gsd = 0.0, grg = 0.0;
HD_RUNROLL
  for (int i = 0; i < NN; ++i) {
    gsd += Qc.g[i] * sd[i];
HD_RUNROLL
    for (int j = 0; j < NN; ++j) grg += Qc.g[i] * HD_SYM(ra, i, j) * Qc.g[j];
  }
  double esurf = (1.0 - alb) * bsurf;
  if (beam) esurf += alb * f0mu0 * exp(-tauc * rmu0) / kPi;
  const double x = (2.0 * alb * gsd + esurf) / (1.0 - 2.0 * alb * grg);
  double ip[NN];
  double chk = 0.0;
  {
    double* lv = A.lev + (size_t)L * 2 * NN * nu + u;
HD_RUNROLL
    for (int i = 0; i < NN; ++i) ip[i] = Qc.g[i] * x;
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
      double t = sd[i];
HD_RUNROLL
      for (int j = 0; j < NN; ++j) t = fma(HD_SYM(ra, i, j), ip[j], t);
      lv[i * nu] = x;
      lv[(NN + i) * nu] = t * Qc.rg[i];
      chk += t;
    }
  }
  // ---- back-substitution bottom -> top ----
  for (int lc = L - 1; lc >= 0; --lc) {
    const double* bp = A.bsub + (size_t)lc * NB * nu + u;
    double nip[NN];
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
      double t = bp[(size_t)(NN * NN + i) * nu];
HD_RUNROLL
      for (int j = 0; j < NN; ++j) t = fma(bp[(size_t)(i * NN + j) * nu], ip[j], t);
      nip[i] = t;
    }
    double* lv = A.lev + (size_t)lc * 2 * NN * nu + u;
HD_RUNROLL
    for (int i = 0; i < NN; ++i) ip[i] = nip[i];
    int e = 0;
    double dn[NN];
HD_RUNROLL
    for (int i = 0; i < NN; ++i) dn[i] = bp[(size_t)(NN * NN + NN + nsym + i) * nu];
HD_RUNROLL
    for (int i = 0; i < NN; ++i)
HD_RUNROLL
      for (int j = i; j < NN; ++j) {
        const double r = bp[(size_t)(NN * NN + NN + (e++)) * nu];
        dn[i] = fma(r, ip[j], dn[i]);
        if (j != i) dn[j] = fma(r, ip[i], dn[j]);
      }
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
      lv[i * nu] = ip[i] * Qc.rg[i];
      lv[(NN + i) * nu] = dn[i] * Qc.rg[i];
      chk += ip[i] + dn[i];
    }
  }
  if (!isfinite(chk)) st |= kStNonFinite;
  flag(A, s, st);
}

// ============================================================================
// per-(unit, layer) homogeneous constants from the level intensities
//   C+ = (X^-1 s_top + Y^-1 d_top)/2,  C- = (X^-1 s_bot - Y^-1 d_bot)/2
//   X^-1 = V^T L^-1 diag(g),  Y^-1 = -K^-1 V^T L^T diag(g)
// ============================================================================
template <int NN>
__device__ __forceinline__ void load_layer(const RadArgs& A, int lc, int u, double (&lch)[NN][NN],
                                           double (&rd)[NN], double (&v)[NN][NN],
                                           double (&kk)[NN]) {
  constexpr int nsym = NN * (NN + 1) / 2;
  const size_t nu = A.nu;
  const double* rr = HD_RREC(lc, u);
  int e = 0;
HD_RUNROLL
  for (int i = 0; i < NN; ++i)
HD_RUNROLL
    for (int k = 0; k <= i; ++k) lch[i][k] = rr[(e++) * HD_RS];
HD_RUNROLL
  for (int i = 0; i < NN; ++i) rd[i] = 1.0 / lch[i][i];
HD_RUNROLL
  for (int i = 0; i < NN; ++i)
HD_RUNROLL
    for (int j = 0; j < NN; ++j) v[i][j] = rr[(nsym + i * NN + j) * HD_RS];
HD_RUNROLL
  for (int j = 0; j < NN; ++j) kk[j] = rr[(nsym + NN * NN + j) * HD_RS];
}

template <int NN>
#ifndef HD_RAD_CONST_WAVES
#define HD_RAD_CONST_WAVES 1
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HD_RAD_CONST_WAVES)))
void hd_rad_const_kernel(RadArgs A) {
  const Quad<NN>& Qc = quad_r<NN>();
  // grid.y = mode (uniform per block: the mode-m tables of the maps are scalar loads)
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long)A.ns * A.nlyr) return;
  const int lc = (int)(id / A.ns);
  const int sl = (int)(id - (long)lc * A.ns);
  const int m = blockIdx.y;
  const int u = m * A.ns + sl;
  const long s = A.s0 + sl;
  const size_t nu = A.nu;
  constexpr int nsym = NN * (NN + 1) / 2;
  constexpr int oZp = nsym + NN * NN + NN, oZm = oZp + NN, oH = oZm + NN, oBt = oH + NN;
  double lch[NN][NN], rd[NN], v[NN][NN], kk[NN];
  load_layer<NN>(A, lc, u, lch, rd, v, kk);
  const double* rr = HD_RREC(lc, u);
  const double bt = rr[oBt * HD_RS], slope = rr[(oBt + 1) * HD_RS], taup = rr[(oBt + 2) * HD_RS];
  const double mu0 = A.umu0 ? A.umu0[s] : 1.0;
  const double fb = A.fbeam ? A.fbeam[s] : 0.0;
  const double rmu0 = (fb > 0.0 && mu0 > 0.0) ? 1.0 / mu0 : 0.0;
  double cp[NN], cm[NN];
HD_RUNROLL
  for (int side = 0; side < 2; ++side) {  // 0: layer top, 1: layer bottom
    const double t = side ? taup : 0.0;
    const double eb = exp(-t * rmu0);
    const double b2 = 2.0 * fma(slope, t, bt);
    const double* lv = A.lev + (size_t)(lc + side) * 2 * NN * nu + u;
    double xs[NN], yd[NN];
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
      const double ipl = lv[i * nu], imi = lv[(NN + i) * nu];
      const double zp = rr[(oZp + i) * HD_RS], zm = rr[(oZm + i) * HD_RS], h = rr[(oH + i) * HD_RS];
      xs[i] = Qc.g[i] * (ipl + imi - (zp + zm) * eb - b2);
      yd[i] = Qc.g[i] * (ipl - imi - (zp - zm) * eb - 2.0 * slope * h);
    }
    lower_solve<NN>(lch, rd, xs);
    double ly[NN];
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {  // L^T yd
      double a = 0.0;
HD_RUNROLL
      for (int k = i; k < NN; ++k) a = fma(lch[k][i], yd[k], a);
      ly[i] = a;
    }
HD_RUNROLL
    for (int j = 0; j < NN; ++j) {
      double a = 0.0, b = 0.0;
HD_RUNROLL
      for (int i = 0; i < NN; ++i) {
        a = fma(v[i][j], xs[i], a);
        b = fma(v[i][j], ly[i], b);
      }
      b = kk[j] > 0.0 ? -b / kk[j] : 0.0;
      if (side == 0) cp[j] = 0.5 * (a + b);
      else cm[j] = 0.5 * (a - b);
    }
  }
  double* co = A.cst + (size_t)lc * 2 * NN * nu + u;
HD_RUNROLL
  for (int j = 0; j < NN; ++j) {
    co[j * nu] = cp[j];
    co[(NN + j) * nu] = cm[j];
  }
#ifndef HD_RAD_WIDE
  if (A.umap) {
    // The user-angle integration's angle-independent part, per (unit, layer).  For a
    // user cosine mu with Y_l^m(mu) = yu_l, split by the parity of l + m into
    // ye (l = 2 l2 + par) and yo (l = 2 l2 + 1 - par), par = m & 1:
    //   ce = Me ye,  Me = V^T L^T D Lam_e^T G_e      (the even source projection)
    //   cx = Mo yo,  Mo = V^T L^-1 D Lam_o^T G_o     (the odd one)
    //   beam amplitude  ab = abe . ye + abo . yo,  thermal  we = tve . ye, wo = tvo . yo
    // with D = diag(sqrt(w/mu)), Lam[l][i] = Y_l^m(mu_i), G = diag(gl/2) -- what
    // hd_rad_user_kernel forms per (unit, angle) from L, V and the moments, regrouped so
    // that it is formed once per (unit, layer) and each angle pays 2 NN^2 FMAs.
    // Element e: rsw [layer][e][unit] for e < ne1 (Me row-major, abe, abo, tve), then
    // bsub [layer][e - ne1][unit] (Mo row-major, tvo).
    constexpr int N = 2 * NN;
    constexpr int NE1 = rad_layer_record_doubles(NN);
    constexpr int NB = rad_bsub_doubles(NN);
    static_assert(NN * NN + 3 * NN <= NE1 && NN * NN + NN <= NB, "map does not fit");
    double* m1 = A.rsw + (size_t)lc * NE1 * nu + u;
    double* m2 = A.bsub + (size_t)lc * NB * nu + u;
    const int L = A.nlyr, np = A.nprop, nmo = A.nmom;
    const double* q = A.prop + ((size_t)s * L + (L - 1 - lc)) * np;
    double ssa = np > 1 ? q[1] : 0.0;
    if (ssa == 1.0) ssa = 1.0 - kDither;
    const double f = nmo >= N ? q[1 + N] : 0.0;
    const double om = ssa * (1.0 - f) / (1.0 - ssa * f);
    const double rf = om / (1.0 - f);
    const bool beam = fb > 0.0 && mu0 > 0.0;
    double y0[N];
    ylm_row<N>(m, beam ? mu0 : 0.0, y0);
    const double fac = (m == 0 ? 1.0 : 2.0) * fb / (4.0 * kPi);
    const double eb = beam ? fac * exp(-A.tauc[(size_t)lc * A.ns + sl] * rmu0) : 0.0;
    const int par = m & 1;
    const double* lam = &tab_r<NN>().lam[m][0][0];
    double zs[NN], zd[NN], hh[NN];
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
      const double zp = rr[(oZp + i) * HD_RS], zm = rr[(oZm + i) * HD_RS];
      zs[i] = beam ? Qc.w[i] * (zp + zm) : 0.0;
      zd[i] = beam ? Qc.w[i] * (zp - zm) : 0.0;
      hh[i] = Qc.w[i] * rr[(oH + i) * HD_RS];
    }
#pragma nounroll
    for (int l2 = 0; l2 < NN; ++l2) {
HD_RUNROLL
      for (int half = 0; half < 2; ++half) {  // 0: even part, 1: odd part
        const int l = 2 * l2 + (half ? 1 - par : par);
        const double chi = l == 0 ? 1.0 : (l <= nmo ? q[1 + l] : 0.0);
        const double gl = (2 * l + 1) * (chi - f) * rf;
        const double gh = 0.5 * gl;
        const double yl0 = ((l + m) & 1) ? -y0[l] : y0[l];  // Y_l^m(-mu0)
        double x[NN], sb = 0.0, st = 0.0;
HD_RUNROLL
        for (int i = 0; i < NN; ++i) {
          const double lm = lam[l * NN + i];
          x[i] = Qc.sd[i] * (gh * lm);
          sb = fma(half ? zd[i] : zs[i], lm, sb);
          st = half ? fma(hh[i], lm, st) : fma(Qc.w[i], lm, st);
        }
        double y[NN];
        if (half == 0) {  // L^T x
HD_RUNROLL
          for (int k = 0; k < NN; ++k) {
            double a = 0.0;
HD_RUNROLL
            for (int i = k; i < NN; ++i) a = fma(lch[i][k], x[i], a);
            y[k] = a;
          }
        } else {  // L^-1 x
HD_RUNROLL
          for (int i = 0; i < NN; ++i) {
            double t = x[i];
HD_RUNROLL
            for (int k = 0; k < i; ++k) t = fma(-lch[i][k], y[k], t);
            y[i] = t * rd[i];
          }
        }
        double* mo = half ? m2 : m1;
HD_RUNROLL
        for (int j = 0; j < NN; ++j) {
          double a = 0.0;
HD_RUNROLL
          for (int i = 0; i < NN; ++i) a = fma(v[i][j], y[i], a);
          mo[(size_t)(j * NN + l2) * nu] = a;
        }
        const double abv = fma(eb * gl, yl0, gh * sb);
        m1[(size_t)(NN * NN + half * NN + l2) * nu] = abv;
        if (half == 0) m1[(size_t)(NN * NN + 2 * NN + l2) * nu] = gh * st;
        else m2[(size_t)(NN * NN + l2) * nu] = gh * st;
      }
    }
  }
#endif
}

// ============================================================================
// fluxes at the user depths from the m = 0 field (unit u = sl)
// ============================================================================
template <int NN>
__global__ __launch_bounds__(256) void hd_rad_flux_kernel(RadArgs A) {
  const Quad<NN>& Qc = quad_r<NN>();
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long)A.ns * A.ntau) return;
  const int lu = (int)(id / A.ns);
  const int sl = (int)(id - (long)lu * A.ns);
  const int u = sl;  // mode 0
  const long s = A.s0 + sl;
  const int L = A.nlyr;
  const size_t nu = A.nu;
  constexpr int nsym = NN * (NN + 1) / 2;
  constexpr int oZp = nsym + NN * NN + NN, oZm = oZp + NN, oH = oZm + NN, oBt = oH + NN;
  const double tu = user_tau(A, lu, sl);
  int lc = 0;
  while (lc < L - 1 && tu > A.taus[(size_t)(lc + 1) * A.ns + sl]) ++lc;
  const double ttop = A.taus[(size_t)lc * A.ns + sl];
  const double tau = A.taus[(size_t)(lc + 1) * A.ns + sl] - ttop;
  double lch[NN][NN], rd[NN], v[NN][NN], kk[NN];
  load_layer<NN>(A, lc, u, lch, rd, v, kk);
  const double* rr = HD_RREC(lc, u);
  const double bt = rr[oBt * HD_RS], slope = rr[(oBt + 1) * HD_RS], taup = rr[(oBt + 2) * HD_RS];
  const double scale = tau > 0.0 ? taup / tau : 0.0;
  const double t = fmin(fmax((tu - ttop) * scale, 0.0), taup);
  const double mu0 = A.umu0 ? A.umu0[s] : 1.0;
  const double fb = A.fbeam ? A.fbeam[s] : 0.0;
  const bool beam = fb > 0.0 && mu0 > 0.0;
  const double rmu0 = beam ? 1.0 / mu0 : 0.0;
  const double* co = A.cst + (size_t)lc * 2 * NN * nu + u;
  double al[NN], be[NN];
HD_RUNROLL
  for (int j = 0; j < NN; ++j) {
    const double a = co[j * nu] * exp(-kk[j] * t);
    const double b = co[(NN + j) * nu] * exp(-kk[j] * (taup - t));
    al[j] = a + b;
    be[j] = kk[j] * (a - b);
  }
  double gs[NN], gd[NN];
HD_RUNROLL
  for (int i = 0; i < NN; ++i) {  // V al, V (k be)
    double a = 0.0, b = 0.0;
HD_RUNROLL
    for (int j = 0; j < NN; ++j) {
      a = fma(v[i][j], al[j], a);
      b = fma(v[i][j], be[j], b);
    }
    gs[i] = a;
    gd[i] = b;
  }
HD_RUNROLL
  for (int i = NN - 1; i >= 0; --i) {  // gs <- L gs (rows bottom-up, in place)
    double a = 0.0;
HD_RUNROLL
    for (int k = 0; k <= i; ++k) a = fma(lch[i][k], gs[k], a);
    gs[i] = a;
  }
  lower_t_solve<NN>(lch, rd, gd);  // g (I+ - I-)_hom = -L^-T V K be
  const double eb = exp(-t * rmu0);
  const double bb = fma(slope, t, bt);
  double up = 0.0, dn = 0.0;
HD_RUNROLL
  for (int i = 0; i < NN; ++i) {
    const double zp = rr[(oZp + i) * HD_RS], zm = rr[(oZm + i) * HD_RS], h = rr[(oH + i) * HD_RS];
    const double ipl = 0.5 * (gs[i] - gd[i]) + Qc.g[i] * (zp * eb + bb + slope * h);
    const double imi = 0.5 * (gs[i] + gd[i]) + Qc.g[i] * (zm * eb + bb - slope * h);
    up = fma(Qc.g[i], ipl, up);
    dn = fma(Qc.g[i], imi, dn);
  }
  up *= 2.0 * kPi;
  dn *= 2.0 * kPi;
  if (beam) dn += fb * mu0 * exp(-(A.tauc[(size_t)lc * A.ns + sl] + t) * rmu0);
  double* fo = A.flux + ((size_t)s * A.ntau + (A.ntau - 1 - lu)) * 2;
  fo[0] = up;
  fo[1] = dn;
  if (!isfinite(up + dn)) flag(A, s, kStNonFinite);
}

// ============================================================================
// per-(unit, user angle) source-function integration along the ray
// ============================================================================
template <int NN>
// HD_RAD_USER_WAVES: waves per SIMD the one-lane user-angle kernel is compiled for
#ifndef HD_RAD_USER_WAVES
#define HD_RAD_USER_WAVES 1
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(HD_RAD_USER_WAVES)))
void hd_rad_user_kernel(RadArgs A) {
  constexpr int N = 2 * NN;
  constexpr int nsym = NN * (NN + 1) / 2;
  constexpr int oZp = nsym + NN * NN + NN, oZm = oZp + NN, oH = oZm + NN, oBt = oH + NN;
  constexpr int oEk = oBt + 4, oE0 = oEk + NN;
  const Quad<NN>& Qc = quad_r<NN>();
  // grid.y = mode (uniform per block: the mode-m tables are scalar loads);
  // user angle fastest inside a block: the lanes of one unit read the same
  // layer records (one cache segment per unit instead of one per angle)
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long)A.ns * A.numu) return;
  const int sl = (int)(id / A.numu);
  const int iu = (int)(id - (long)sl * A.numu);
  const int m = blockIdx.y;
  const int u = m * A.ns + sl;
  const long s = A.s0 + sl;
  const int L = A.nlyr, np = A.nprop, nm = A.nmom;
  const size_t nu = A.nu;
  const double muu = A.umu[iu];
  const double mu0 = A.umu0 ? A.umu0[s] : 1.0;
  const double fb = A.fbeam ? A.fbeam[s] : 0.0;
  const bool beam = fb > 0.0 && mu0 > 0.0;
  const double rmu0 = beam ? 1.0 / mu0 : 0.0;
  const bool therm = A.planck && m == 0;
  const double fac = (m == 0 ? 1.0 : 2.0) * fb / (4.0 * kPi);
  double yu[N], y0[N];
  ylm_row<N>(m, muu, yu);
  ylm_row<N>(m, beam ? mu0 : 0.0, y0);
HD_RUNROLL
  for (int l = 0; l < N; ++l) y0[l] = ((l + m) & 1) ? -y0[l] : y0[l];  // Y_l^m(-mu0)
  const double* lam = &tab_r<NN>().lam[m][0][0];
  const bool up = muu > 0.0;

  double cur;
  if (up) {
    cur = 0.0;
    if (m == 0) {
      const double* lv = A.lev + (size_t)L * 2 * NN * nu + u;
      double fdn = 0.0;
HD_RUNROLL
      for (int i = 0; i < NN; ++i) fdn = fma(Qc.g[i] * Qc.g[i], lv[(NN + i) * nu], fdn);
      fdn *= 2.0 * kPi;
      const double alb = A.albedo ? A.albedo[s] : 0.0;
      if (beam) {
        const double tb = A.tauc[(size_t)(L - 1) * A.ns + sl] +
                          HD_RREC(L - 1, u)[(oBt + 2) * HD_RS];
        fdn += fb * mu0 * exp(-tb * rmu0);
      }
      cur = alb / kPi * fdn + (A.planck ? (1.0 - alb) * A.planckv[(size_t)(L + 1) * A.ns + sl]
                                        : 0.0);
    }
  } else {
    cur = 0.0;
    if (m == 0) {
      cur = A.fisot ? A.fisot[s] : 0.0;
      if (A.planck) cur += A.planckv[(size_t)(L + 2) * A.ns + sl];
    }
  }
  int k = up ? A.ntau - 1 : 0;
  double chk = 0.0;
  for (int step = 0; step < L; ++step) {
    const int lc = up ? L - 1 - step : step;
    const double ttop = A.taus[(size_t)lc * A.ns + sl];
    const double tbot = A.taus[(size_t)(lc + 1) * A.ns + sl];
    // ---- delta-M moments of this layer, mode-m phase row at muu ----
    const double* q = A.prop + ((size_t)s * L + (L - 1 - lc)) * np;
    double ssa = np > 1 ? q[1] : 0.0;
    if (ssa == 1.0) ssa = 1.0 - kDither;
    const double f = nm >= N ? q[1 + N] : 0.0;
    const double om = ssa * (1.0 - f) / (1.0 - ssa * f);
    const double rf = om / (1.0 - f);
    double cue[NN], cuo[NN];
    double x0 = 0.0;
    double gy[N];
HD_RUNROLL
    for (int l = 0; l < N; ++l) {
      const double chi = l == 0 ? 1.0 : (l <= nm ? q[1 + l] : 0.0);
      const double gl = (2 * l + 1) * (chi - f) * rf;
      gy[l] = 0.5 * gl * yu[l];
      x0 = fma(gl * yu[l], y0[l], x0);
    }
    // even/odd parts in l + m: m is uniform per block, so is the branch
    auto lsum = [&](int par) {
HD_RUNROLL
      for (int i = 0; i < NN; ++i) {
        double e = 0.0, o = 0.0;
HD_RUNROLL
        for (int l2 = 0; l2 < NN; ++l2) {
          e = fma(gy[2 * l2 + par], lam[(2 * l2 + par) * NN + i], e);
          o = fma(gy[2 * l2 + 1 - par], lam[(2 * l2 + 1 - par) * NN + i], o);
        }
        cue[i] = e;
        cuo[i] = o;
      }
    };
    if (m & 1) lsum(1);
    else lsum(0);
    const double* rr = HD_RREC(lc, u);
    const double bt = rr[oBt * HD_RS], slope = rr[(oBt + 1) * HD_RS], taup = rr[(oBt + 2) * HD_RS];
    // ce = V^T L^T (sd cue), co = -k V^T L^-1 (sd cuo); L and V streamed from the
    // record (each element used once), not held in registers
    double a1[NN], b1[NN];
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {
      a1[i] = 0.0;
      b1[i] = Qc.sd[i] * cuo[i];
    }
HD_RUNROLL
    for (int i = 0; i < NN; ++i) {  // row i of L: a1 += L[i][:]^T (sd cue)_i ; b1 forward subst.
      const double* li = rr + (size_t)(i * (i + 1) / 2) * HD_RS;
      const double ce_i = Qc.sd[i] * cue[i];
      double t = b1[i];
HD_RUNROLL
      for (int k2 = 0; k2 < i; ++k2) {
        const double l = li[k2 * HD_RS];
        a1[k2] = fma(l, ce_i, a1[k2]);
        t = fma(-l, b1[k2], t);
      }
      const double d = li[i * HD_RS];
      a1[i] = fma(d, ce_i, a1[i]);
      b1[i] = t / d;
    }
    const double* co = A.cst + (size_t)lc * 2 * NN * nu + u;
    const double* vr = rr + (size_t)nsym * HD_RS;
    double kk[NN], hpl[NN], hmi[NN];
HD_RUNROLL
    for (int j = 0; j < NN; ++j) {
      hpl[j] = hmi[j] = 0.0;
      kk[j] = rr[(nsym + NN * NN + j) * HD_RS];
    }
HD_RUNROLL
    for (int i = 0; i < NN; ++i)
HD_RUNROLL
      for (int j = 0; j < NN; ++j) {
        const double vij = vr[(i * NN + j) * HD_RS];
        hpl[j] = fma(vij, a1[i], hpl[j]);  // ce
        hmi[j] = fma(vij, b1[i], hmi[j]);  // V^T b1
      }
HD_RUNROLL
    for (int j = 0; j < NN; ++j) {
      const double ce = hpl[j], cx = -kk[j] * hmi[j];
      hpl[j] = co[j * nu] * (ce + cx);
      hmi[j] = co[(NN + j) * nu] * (ce - cx);
    }
    double ab = 0.0, a0 = 0.0, a1t = 0.0;
    if (beam) {
      double sc = 0.0;
HD_RUNROLL
      for (int i = 0; i < NN; ++i) {
        const double zp = rr[(oZp + i) * HD_RS], zm = rr[(oZm + i) * HD_RS];
        sc = fma(Qc.w[i], fma(cue[i], zp + zm, cuo[i] * (zp - zm)), sc);
      }
      ab = fma(fac * x0, exp(-A.tauc[(size_t)lc * A.ns + sl] * rmu0), sc);
    }
    if (therm) {
      double we = 0.0, wo = 0.0;
HD_RUNROLL
      for (int i = 0; i < NN; ++i) {
        we = fma(Qc.w[i], cue[i], we);
        wo = fma(Qc.w[i] * cuo[i], rr[(oH + i) * HD_RS], wo);
      }
      const double ce0 = (1.0 - om) + 2.0 * we;
      a1t = slope * ce0;
      a0 = fma(bt, ce0, 2.0 * slope * wo);
    }
    // general segment [t1 (evaluation), t2 (far end)] for user depths inside the layer
    auto integ = [&](double t1, double t2) {
      double r = 0.0;
HD_RUNROLL
      for (int j = 0; j < NN; ++j) {
        r += seg_exp(hpl[j], kk[j], t1, t2, 0.0, muu);
        r += seg_exp(hmi[j], -kk[j], t1, t2, taup, muu);
      }
      if (beam) r += seg_exp(ab, rmu0, t1, t2, 0.0, muu);
      if (therm) {
        const double e2 = exp(-(t2 - t1) / muu);
        r += (a0 + a1t * t1 + a1t * muu) - (a0 + a1t * t2 + a1t * muu) * e2;
      }
      return r;
    };
    // whole layer, entry -> exit, from the stored exp(-k tau'), exp(-tau'/mu0)
    // and one exp(-tau'/|mu|): the +k terms decay along upward rays, the -k
    // terms along downward ones; the other family meets 1 - k|mu| -> 0 and goes
    // through dexp's (1 - e^-y)/y series
    const double anu = fabs(muu);
    const double lmu = taup / anu;
    const double emu = exp(-lmu);
    double lay = 0.0;
HD_RUNROLL
    for (int j = 0; j < NN; ++j) {
      const double ek = rr[(oEk + j) * HD_RS];
      const double reg = (1.0 - ek * emu) / fma(kk[j], anu, 1.0);
      const double sng = dexp(ek, emu, fma(-kk[j], anu, 1.0), lmu);
      lay = up ? fma(hpl[j], reg, fma(hmi[j], sng, lay)) : fma(hpl[j], sng, fma(hmi[j], reg, lay));
    }
    if (beam) {
      const double e0l = rr[oE0 * HD_RS];
      lay += up ? ab * (1.0 - e0l * emu) / fma(anu, rmu0, 1.0)
                : ab * dexp(e0l, emu, fma(-anu, rmu0, 1.0), lmu);
    }
    if (therm) {  // (a0 + a1 t1 + a1 mu) - (a0 + a1 t2 + a1 mu) e^{-(t2-t1)/mu}
      lay += up ? (a0 + a1t * muu) - (a0 + a1t * taup + a1t * muu) * emu
                : (a0 + a1t * taup + a1t * muu) - (a0 + a1t * muu) * emu;
    }
    const double cin = cur;                // at the entry boundary
    const double cout = fma(cin, emu, lay);  // at the exit boundary
    const double tau = tbot - ttop;
    const double scale = tau > 0.0 ? taup / tau : 0.0;
    // value at local depth t: boundaries from cin/cout, interior by integ
    auto at = [&](double t) {
      const double tin = up ? taup : 0.0;  // entry depth
      if (t == tin) return cin;
      if (t == taup - tin) return cout;
      return cin * exp(-fabs(tin - t) / anu) + integ(t, tin);
    };
    if (up) {
      while (k >= 0 && user_tau(A, k, sl) >= ttop) {
        const double t = fmin(fmax((user_tau(A, k, sl) - ttop) * scale, 0.0), taup);
        const double val = at(t);
        A.radm[((size_t)k * A.numu + iu) * nu + u] = val;
        chk += val;
        --k;
      }
    } else {
      while (k < A.ntau && user_tau(A, k, sl) <= tbot) {
        const double t = fmin(fmax((user_tau(A, k, sl) - ttop) * scale, 0.0), taup);
        const double val = at(t);
        A.radm[((size_t)k * A.numu + iu) * nu + u] = val;
        chk += val;
        ++k;
      }
    }
    cur = cout;
  }
  // user depths beyond the bottom (flagged by the taus kernel): bottom value
  for (; k < A.ntau && !up; ++k) A.radm[((size_t)k * A.numu + iu) * nu + u] = cur;
  if (!isfinite(chk)) flag(A, s, kStNonFinite);
}

#ifndef HD_RAD_WIDE
// ============================================================================
// per-(unit, user angle) source-function integration from the const kernel's maps
// (nstr <= 16): the layer's source projections are two NN x NN products with the
// angle's Y_l^m row (ce = Me ye, cx = Mo yo) instead of hd_rad_user_kernel's
// per-angle Legendre sums, triangular solve and V^T products; the beam and thermal
// amplitudes are dot products.  Everything after that -- the whole-layer terms,
// interior user depths, the scan over layers -- is hd_rad_user_kernel's.
// ============================================================================
#ifndef HD_RAD_UMAP_WAVES
#define HD_RAD_UMAP_WAVES 2
#endif
#ifndef HD_RAD_UMAP_UTAU_REG
#define HD_RAD_UMAP_UTAU_REG 1
#endif
constexpr bool kUmapUtauReg = HD_RAD_UMAP_UTAU_REG != 0;
template <int NN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(HD_RAD_UMAP_WAVES)))
void hd_rad_user_map_kernel(RadArgs A) {
  constexpr int N = 2 * NN;
  constexpr int nsym = NN * (NN + 1) / 2;
  constexpr int oZp = nsym + NN * NN + NN, oZm = oZp + NN, oH = oZm + NN, oBt = oH + NN;
  constexpr int oEk = oBt + 4, oE0 = oEk + NN;
  constexpr int NE1 = rad_layer_record_doubles(NN);
  constexpr int NB = rad_bsub_doubles(NN);
  const Quad<NN>& Qc = quad_r<NN>();
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long)A.ns * A.numu) return;
  const int sl = (int)(id / A.numu);
  const int iu = (int)(id - (long)sl * A.numu);
  const int m = blockIdx.y;
  const int u = m * A.ns + sl;
  const long s = A.s0 + sl;
  const int L = A.nlyr;
  const size_t nu = A.nu;
  const double muu = A.umu[iu];
  const double mu0 = A.umu0 ? A.umu0[s] : 1.0;
  const double fb = A.fbeam ? A.fbeam[s] : 0.0;
  const bool beam = fb > 0.0 && mu0 > 0.0;
  const double rmu0 = beam ? 1.0 / mu0 : 0.0;
  const bool therm = A.planck && m == 0;
  const int par = m & 1;
  double ye[NN], yo[NN];
  {
    double yu[N];
    ylm_row<N>(m, muu, yu);
HD_RUNROLL
    for (int l2 = 0; l2 < NN; ++l2) {
      ye[l2] = yu[2 * l2 + par];
      yo[l2] = yu[2 * l2 + 1 - par];
    }
  }
  const bool up = muu > 0.0;

  double cur = 0.0;
  if (up) {
    if (m == 0) {
      const double* lv = A.lev + (size_t)L * 2 * NN * nu + u;
      double fdn = 0.0;
HD_RUNROLL
      for (int i = 0; i < NN; ++i) fdn = fma(Qc.g[i] * Qc.g[i], lv[(NN + i) * nu], fdn);
      fdn *= 2.0 * kPi;
      const double alb = A.albedo ? A.albedo[s] : 0.0;
      if (beam) {
        const double tb = A.tauc[(size_t)(L - 1) * A.ns + sl] +
                          HD_RREC(L - 1, u)[(oBt + 2) * HD_RS];
        fdn += fb * mu0 * exp(-tb * rmu0);
      }
      cur = alb / kPi * fdn + (A.planck ? (1.0 - alb) * A.planckv[(size_t)(L + 1) * A.ns + sl]
                                        : 0.0);
    }
  } else if (m == 0) {
    cur = A.fisot ? A.fisot[s] : 0.0;
    if (A.planck) cur += A.planckv[(size_t)(L + 2) * A.ns + sl];
  }
  int k = up ? A.ntau - 1 : 0;
  // the next user depth in ray order, held in a register: reloaded only when a depth
  // is consumed, not on every layer's loop test (a dependent load per layer)
  auto utau_at = [&](int kk) { return kk >= 0 && kk < A.ntau ? user_tau(A, kk, sl) : 0.0; };
  double utk = kUmapUtauReg ? utau_at(k) : 0.0;
  double chk = 0.0;
  for (int step = 0; step < L; ++step) {
    const int lc = up ? L - 1 - step : step;
    const double ttop = A.taus[(size_t)lc * A.ns + sl];
    const double tbot = A.taus[(size_t)(lc + 1) * A.ns + sl];
    const double* rr = HD_RREC(lc, u);
    const double* m1 = A.rsw + (size_t)lc * NE1 * nu + u;
    const double* m2 = A.bsub + (size_t)lc * NB * nu + u;
    const double* co = A.cst + (size_t)lc * 2 * NN * nu + u;
    const double bt = rr[oBt * HD_RS], slope = rr[(oBt + 1) * HD_RS], taup = rr[(oBt + 2) * HD_RS];
    double kk[NN], hpl[NN], hmi[NN];
HD_RUNROLL
    for (int j = 0; j < NN; ++j) {
      double ce = 0.0, cx = 0.0;
HD_RUNROLL
      for (int l2 = 0; l2 < NN; ++l2) {
        ce = fma(m1[(size_t)(j * NN + l2) * nu], ye[l2], ce);
        cx = fma(m2[(size_t)(j * NN + l2) * nu], yo[l2], cx);
      }
      kk[j] = rr[(nsym + NN * NN + j) * HD_RS];
      cx *= -kk[j];
      hpl[j] = co[j * nu] * (ce + cx);
      hmi[j] = co[(NN + j) * nu] * (ce - cx);
      // one row of the maps in flight at a time, consumed before the next row's loads
      // (at two waves per SIMD the other wave covers the latency; with the products
      // sunk below all 128 loads the kernel needed 490 registers)
      asm volatile("" : "+v"(hpl[j]), "+v"(hmi[j])::"memory");
    }
    double ab = 0.0, a0 = 0.0, a1t = 0.0;
    if (beam) {
HD_RUNROLL
      for (int l2 = 0; l2 < NN; ++l2) {
        ab = fma(m1[(size_t)(NN * NN + l2) * nu], ye[l2], ab);
        ab = fma(m1[(size_t)(NN * NN + NN + l2) * nu], yo[l2], ab);
      }
    }
    if (therm) {
      double we = 0.0, wo = 0.0;
HD_RUNROLL
      for (int l2 = 0; l2 < NN; ++l2) {
        we = fma(m1[(size_t)(NN * NN + 2 * NN + l2) * nu], ye[l2], we);
        wo = fma(m2[(size_t)(NN * NN + l2) * nu], yo[l2], wo);
      }
      const double om = rr[(oBt + 3) * HD_RS];
      const double ce0 = (1.0 - om) + 2.0 * we;
      a1t = slope * ce0;
      a0 = fma(bt, ce0, 2.0 * slope * wo);
    }
    // general segment [t1 (evaluation), t2 (far end)] for user depths inside the layer
    auto integ = [&](double t1, double t2) {
      double r = 0.0;
HD_RUNROLL
      for (int j = 0; j < NN; ++j) {
        r += seg_exp(hpl[j], kk[j], t1, t2, 0.0, muu);
        r += seg_exp(hmi[j], -kk[j], t1, t2, taup, muu);
        asm volatile("" : "+v"(r));  // one eigen-term at a time
      }
      if (beam) r += seg_exp(ab, rmu0, t1, t2, 0.0, muu);
      if (therm) {
        const double e2 = exp(-(t2 - t1) / muu);
        r += (a0 + a1t * t1 + a1t * muu) - (a0 + a1t * t2 + a1t * muu) * e2;
      }
      return r;
    };
    const double anu = fabs(muu);
    const double lmu = taup / anu;
    const double emu = exp(-lmu);
    double lay = 0.0;
HD_RUNROLL
    for (int j = 0; j < NN; ++j) {
      const double ek = rr[(oEk + j) * HD_RS];
      const double reg = (1.0 - ek * emu) / fma(kk[j], anu, 1.0);
      const double sng = dexp(ek, emu, fma(-kk[j], anu, 1.0), lmu);
      lay = up ? fma(hpl[j], reg, fma(hmi[j], sng, lay)) : fma(hpl[j], sng, fma(hmi[j], reg, lay));
      asm volatile("" : "+v"(lay));  // one eigen-term's quotient and series at a time
    }
    if (beam) {
      const double e0l = rr[oE0 * HD_RS];
      lay += up ? ab * (1.0 - e0l * emu) / fma(anu, rmu0, 1.0)
                : ab * dexp(e0l, emu, fma(-anu, rmu0, 1.0), lmu);
    }
    if (therm) {
      lay += up ? (a0 + a1t * muu) - (a0 + a1t * taup + a1t * muu) * emu
                : (a0 + a1t * taup + a1t * muu) - (a0 + a1t * muu) * emu;
    }
    const double cin = cur;
    const double cout = fma(cin, emu, lay);
    const double tau = tbot - ttop;
    const double scale = tau > 0.0 ? taup / tau : 0.0;
    auto at = [&](double t) {
      const double tin = up ? taup : 0.0;
      if (t == tin) return cin;
      if (t == taup - tin) return cout;
      return cin * exp(-fabs(tin - t) / anu) + integ(t, tin);
    };
    // the user depths in this layer, in ray order (one copy of the interior integral)
    while (up ? (k >= 0 && (kUmapUtauReg ? utk : user_tau(A, k, sl)) >= ttop)
              : (k < A.ntau && (kUmapUtauReg ? utk : user_tau(A, k, sl)) <= tbot)) {
      const double t = fmin(fmax(((kUmapUtauReg ? utk : user_tau(A, k, sl)) - ttop) * scale, 0.0), taup);
      const double val = at(t);
      A.radm[((size_t)k * A.numu + iu) * nu + u] = val;
      chk += val;
      k += up ? -1 : 1;
      if (kUmapUtauReg) utk = utau_at(k);
    }
    cur = cout;
  }
  for (; k < A.ntau && !up; ++k) A.radm[((size_t)k * A.numu + iu) * nu + u] = cur;
  if (!isfinite(chk)) flag(A, s, kStNonFinite);
}
#endif

// ============================================================================
// uu[s][j][lu][iu] = sum_m I_m cos(m (phi_j - phi0))
// ============================================================================
__global__ __launch_bounds__(256) void hd_rad_azimuth_kernel(RadArgs A) {
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = (long)A.ns * A.nphi * A.ntau * A.numu;
  if (id >= n) return;
  const int sl = (int)(id % A.ns);
  long r = id / A.ns;
  const int iu = (int)(r % A.numu);
  r /= A.numu;
  const int lu = (int)(r % A.ntau);
  const int j = (int)(r / A.ntau);
  const long s = A.s0 + sl;
  const double ph0 = A.phi0 ? A.phi0[s] : 0.0;
  const double dphi = (A.phi[j] - ph0) * (kPi / 180.0);
  const double* src = A.radm + ((size_t)lu * A.numu + iu) * A.nu + sl;
  double acc = 0.0;
  for (int m = 0; m < A.nm; ++m) acc = fma(src[(size_t)m * A.ns], cos(m * dphi), acc);
  A.uu[(((size_t)s * A.nphi + j) * A.ntau + lu) * A.numu + iu] = acc;
}


// ============================================================================
// IMS step of the Nakajima-Tanaka correction (DISORT 2.0 SECSCA / XIFUNC, STWL
// eqs. A.13-A.16), without the F0/(4 pi) factor: secondary scattering through
// the truncated forward peak, which delta-M (and so the TMS step) treats as
// exactly forward.  The slab above the user depth tu (unscaled; the user's
// layer lu_l down to tu) is replaced by its omega- and f-weighted averages;
// the peak's phase function P'' has moments 1 below nstr and
// g_l = <omega chi_l>/<omega f> from nstr on, and PSPIKE = 2 P'' - P''*P''
// (moments 2 g - g^2).  Same arithmetic as oracle/disort_rad_np.py's
// ims_correction / xi_func.  mu1 = |mu| of a downward user direction.
// ============================================================================
__device__ double ims_term(const RadArgs& A, long s, int nstr, double ct, double mu1, double mu0,
                           double tu, int lu_l) {
  constexpr double kTiny = 1.0e-4;
  const int L = A.nlyr, np = A.nprop, nm = A.nmom;
  if (nm < nstr) return 0.0;  // no truncation: f = 0
  const double* q0 = A.prop + (size_t)s * L * np;
  // dtau of solver layer lc above tu (harp layer L-1-lc); ssalb dithered as in setdis
  auto slab = [&](int lc, double& ssa) {
    const double* q = q0 + (size_t)(L - 1 - lc) * np;
    ssa = np > 1 ? q[1] : 0.0;
    if (ssa == 1.0) ssa = 1.0 - kDither;
    if (lc < lu_l) return q[0];
    const double d = tu - A.taus[(size_t)lc * A.ns + (s - A.s0)];
    return d > 0.0 ? d : 0.0;
  };
  double wsum = 0.0, fsum = 0.0, stau = 0.0;
  for (int lc = 0; lc <= lu_l; ++lc) {
    double ssa;
    const double dt = slab(lc, ssa);
    const double wt = ssa * dt;
    wsum += wt;
    fsum = fma(wt, q0[(size_t)(L - 1 - lc) * np + 1 + nstr], fsum);
    stau += dt;
  }
  if (!(wsum > kTiny) || !(fsum > kTiny) || !(stau > kTiny)) return 0.0;
  const double fw = fsum / stau;  // f-bar omega-bar
  // PSPIKE by the Legendre recurrence at cos(Theta)
  double ps = 1.0, p1 = 1.0, p2 = 0.0;
  for (int k = 1; k <= nm; ++k) {
    const double pk = ((2 * k - 1) * ct * p1 - (k - 1) * p2) / k;
    p2 = p1;
    p1 = pk;
    double wk = 1.0;
    if (k >= nstr) {
      double gs = 0.0;
      for (int lc = 0; lc <= lu_l; ++lc) {
        double ssa;
        const double dt = slab(lc, ssa);
        gs = fma(ssa * dt, q0[(size_t)(L - 1 - lc) * np + 1 + k], gs);
      }
      const double g = gs / fsum;
      wk = g * (2.0 - g);
    }
    ps = fma((2 * k + 1) * wk, pk, ps);
  }
  // xi(mu1, mu2, tu), mu2 = mu0 / (1 - f w)
  const double mu2 = mu0 / (1.0 - fw);
  const double a = 1.0 / mu2 - 1.0 / mu1;
  const double x = a * tu;
  const double e1 = exp(-tu / mu1);
  double xi;
  if (fabs(x) < 0.5) {
    double h = 0.0, term = 1.0, fact = 2.0;  // sum_{k>=2} (-1)^k (k-1)/k! x^(k-2)
    for (int k = 2; k < 24; ++k) {
      h += (k - 1) / fact * term;
      term *= -x;
      fact *= k + 1;
    }
    xi = e1 * tu * tu / (mu1 * mu2) * h;
  } else {
    xi = (e1 - exp(-tu / mu2) * (1.0 + x)) / (a * a * mu1 * mu2);
  }
  return fw * fw / (1.0 - fw) * ps * xi;
}

// ============================================================================
// Nakajima-Tanaka correction (DISORT 2.0 INTCOR): the TMS step (STWL eq. 68),
// exact single scattering (full moment series, omega/(1 - f omega)) minus the
// delta-M one (truncated series, omega'), both on the scaled depths, and for
// downward directions minus the IMS term (ims_term); added to uu
// ============================================================================
__global__ __launch_bounds__(256) void hd_rad_tms_kernel(RadArgs A, int nstr) {
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = (long)A.ns * A.nphi * A.ntau * A.numu;
  if (id >= n) return;
  const int sl = (int)(id % A.ns);
  long r = id / A.ns;
  const int iu = (int)(r % A.numu);
  r /= A.numu;
  const int lu = (int)(r % A.ntau);
  const int j = (int)(r / A.ntau);
  const long s = A.s0 + sl;
  const double mu0 = A.umu0 ? A.umu0[s] : 1.0;
  const double fb = A.fbeam ? A.fbeam[s] : 0.0;
  if (!(fb > 0.0 && mu0 > 0.0)) return;
  const int L = A.nlyr, np = A.nprop, nm = A.nmom;
  const double mu = A.umu[iu];
  const double ph0 = A.phi0 ? A.phi0[s] : 0.0;
  const double ct = fma(-mu, mu0, sqrt(fmax(0.0, 1.0 - mu * mu)) *
                                      sqrt(fmax(0.0, 1.0 - mu0 * mu0)) *
                                      cos((A.phi[j] - ph0) * (kPi / 180.0)));
  // user depth -> layer and scaled depth
  const double tu = user_tau(A, lu, sl);
  int lu_l = 0;
  while (lu_l < L - 1 && tu > A.taus[(size_t)(lu_l + 1) * A.ns + sl]) ++lu_l;
  const double rmu0 = 1.0 / mu0;
  double acc = 0.0, tau_u = 0.0;
  for (int pass = 0; pass < 2; ++pass) {  // pass 0: scaled depth of the user level
    const int lo = pass == 0 ? lu_l : (mu > 0.0 ? lu_l : 0);
    const int hi = pass == 0 ? lu_l : (mu > 0.0 ? L - 1 : lu_l);
    for (int lc = lo; lc <= hi; ++lc) {
      const double* q = A.prop + ((size_t)s * L + (L - 1 - lc)) * np;
      const double tau = q[0];
      double ssa = np > 1 ? q[1] : 0.0;
      if (ssa == 1.0) ssa = 1.0 - kDither;
      const double f = nm >= nstr ? q[1 + nstr] : 0.0;
      const double taup = (1.0 - ssa * f) * tau;
      const double top = A.tauc[(size_t)lc * A.ns + sl];
      if (pass == 0) {
        const double ttop = A.taus[(size_t)lc * A.ns + sl];
        const double scale = tau > 0.0 ? taup / tau : 0.0;
        tau_u = top + fmin(fmax((tu - ttop) * scale, 0.0), taup);
        continue;
      }
      const double bot = top + taup;
      const double t1 = mu > 0.0 ? fmax(tau_u, top) : fmin(tau_u, bot);
      const double t2 = mu > 0.0 ? bot : top;
      // phase functions at cos(Theta): full series and delta-M truncated series
      double pa = 1.0, pm = 1.0;  // k = 0 terms: chi_0 = 1, (chi_0 - f)/(1 - f) = 1
      double p1 = 1.0, p2 = 0.0;
      const int kmax = nm > nstr - 1 ? nm : nstr - 1;
      for (int k = 1; k <= kmax; ++k) {
        const double pk = ((2 * k - 1) * ct * p1 - (k - 1) * p2) / k;
        p2 = p1;
        p1 = pk;
        const double chi = k <= nm ? q[1 + k] : 0.0;
        if (k <= nm) pa = fma((2 * k + 1) * chi, pk, pa);
        if (k < nstr) pm = fma((2 * k + 1) * (chi - f) / (1.0 - f), pk, pm);
      }
      const double om = ssa * (1.0 - f) / (1.0 - ssa * f);
      const double w = ssa * pa / (1.0 - f * ssa) - om * pm;
      // int_{t1}^{t2} e^{-t/mu0} e^{-(t - tau_u)/mu} dt/mu
      const double e1 = exp(-t1 * rmu0 - (t1 - tau_u) / mu);
      const double den = fma(rmu0, mu, 1.0);
      const double x = den * (t2 - t1) / mu;
      double seg;
      if (fabs(x) < 0.5) {
        const double phx = x == 0.0 ? 1.0 : -expm1(-x) / x;
        seg = e1 * (t2 - t1) / mu * phx;
      } else {
        seg = (e1 - exp(-t2 * rmu0 - (t2 - tau_u) / mu)) / den;
      }
      acc = fma(w, seg, acc);
    }
  }
  if (mu < 0.0 && fb > 1.0e-4) acc -= ims_term(A, s, nstr, ct, -mu, mu0, tu, lu_l);  // SECSCA: fbeam > tiny
  A.uu[(((size_t)s * A.nphi + j) * A.ntau + lu) * A.numu + iu] += fb / (4.0 * kPi) * acc;
}

// ============================================================================
// host side
// ============================================================================
template <int NN>
static void fill_rad(Quad<NN>& q, RadTab<NN>& t, const QuadHost& h) {
  for (int i = 0; i < NN; ++i) {
    q.mu[i] = h.mu[i];
    q.w[i] = h.w[i];
    q.sd[i] = h.sd[i];
    q.g[i] = h.g[i];
    q.rmu[i] = 1.0 / h.mu[i];
    q.rg[i] = 1.0 / h.g[i];
    for (int l = 0; l < 2 * NN; ++l) q.pt[l][i] = h.pt[l][i];
  }
  // Y_l^m(mu_i) by the same recurrence as ylm_row
  for (int m = 0; m < 2 * NN; ++m)
    for (int i = 0; i < NN; ++i) {
      const double x = h.mu[i];
      double seed = 1.0;
      for (int a = 1; a <= m; ++a) seed *= std::sqrt((2.0 * a - 1) / (2.0 * a));
      seed *= std::pow(std::sqrt(std::fmax(0.0, 1.0 - x * x)), m);
      double y1 = 0.0, y2 = 0.0;
      for (int l = 0; l < 2 * NN; ++l) {
        double v = 0.0;
        if (l == m) v = seed;
        else if (l > m)
          v = ((2.0 * l - 1) * x * y1 - std::sqrt((double)(l - 1) * (l - 1) - (double)m * m) * y2) /
              std::sqrt((double)l * l - (double)m * m);
        t.lam[m][l][i] = v;
        y2 = y1;
        y1 = v;
      }
    }
}

// called once per device, under hd_api.cpp's global table lock (ensure_rad_tables),
// so the function-static staging buffers below are never filled concurrently
hipError_t upload_rad_tables(const QuadHost* per_nn) {
  static RadConst c;  // ~60 KB: keep off the stack
  fill_rad<1>(c.q1, c.t1, per_nn[0]);
  fill_rad<2>(c.q2, c.t2, per_nn[1]);
  fill_rad<3>(c.q3, c.t3, per_nn[2]);
  fill_rad<4>(c.q4, c.t4, per_nn[3]);
  fill_rad<5>(c.q5, c.t5, per_nn[4]);
  fill_rad<6>(c.q6, c.t6, per_nn[5]);
  fill_rad<7>(c.q7, c.t7, per_nn[6]);
  fill_rad<8>(c.q8, c.t8, per_nn[7]);
#ifdef HD_RAD_WIDE
  static RadConstWide cw;  // ~560 KB
  fill_rad<9>(cw.q9, cw.t9, per_nn[8]);
  fill_rad<10>(cw.q10, cw.t10, per_nn[9]);
  fill_rad<11>(cw.q11, cw.t11, per_nn[10]);
  fill_rad<12>(cw.q12, cw.t12, per_nn[11]);
  fill_rad<13>(cw.q13, cw.t13, per_nn[12]);
  fill_rad<14>(cw.q14, cw.t14, per_nn[13]);
  fill_rad<15>(cw.q15, cw.t15, per_nn[14]);
  fill_rad<16>(cw.q16, cw.t16, per_nn[15]);
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_radw), &cw, sizeof(RadConstWide));
  if (e != hipSuccess) return e;
#else
  // the nstr 18..32 instantiations keep their own tables (hd_rad_wide.hip)
  hipError_t e = wide::upload_rad_tables(per_nn);
  if (e != hipSuccess) return e;
#endif
  for (int m = 0; m < 2 * kRadMaxNN; ++m) {
    double sd = 1.0;
    for (int a = 1; a <= m; ++a) sd *= std::sqrt((2.0 * a - 1) / (2.0 * a));
    c.seed[m] = sd;
    for (int l = 0; l < 2 * kRadMaxNN; ++l) {
      if (l > m) {
        const double den = std::sqrt((double)l * l - (double)m * m);
        c.ra[m][l] = (2.0 * l - 1) / den;
        c.rb[m][l] = std::sqrt((double)(l - 1) * (l - 1) - (double)m * m) / den;
      } else {
        c.ra[m][l] = c.rb[m][l] = 0.0;
      }
    }
  }
  return hipMemcpyToSymbol(HIP_SYMBOL(c_rad), &c, sizeof(RadConst));
}

// HD_RAD_USER=rolled: nstr 18..32 user angles by the one-lane-per-(unit, angle) kernel
static bool rad_user_rolled() {
  static const bool v = [] {
    const char* e = ab_env("HD_RAD_USER");
    return e && std::strcmp(e, "rolled") == 0;
  }();
  return v;
}

// HD_RAD_USER=direct: nstr <= 16 user angles by the per-angle hd_rad_user_kernel
static bool rad_user_direct() {
#if HD_AB_VARIANTS
  static const bool v = [] {
    const char* e = ab_env("HD_RAD_USER");
    return e && std::strcmp(e, "direct") == 0;
  }();
  return v;
#else
  return false;  // the per-angle kernel at nstr <= 16: A/B build only
#endif
}

template <int NN>
static void launch_rad(const RadArgs& a, bool radiances, hipStream_t st) {
  const unsigned ns_b = (unsigned)((a.ns + 255) / 256);
  hipLaunchKernelGGL(hd_rad_taus_kernel, dim3(ns_b), dim3(256), 0, st, a);
  const unsigned nb1 = (unsigned)(((a.nu + 63) / 64) *
                                  ((a.nlyr + kLayersPerBlockR - 1) / kLayersPerBlockR));
  if constexpr (NN > kMaxRegNN)
    (void)hd::launch_rad_team_layer(NN, a, st);  // team layout + MFMA (hd_team_mfma.hip)
  else
    hipLaunchKernelGGL(hd_rad_layer_kernel<NN>, dim3(nb1), dim3(kLayerBlockR), 0, st, a);
  if constexpr (NN > kMaxRegNN)
    (void)hd::launch_rad_team_sweep(NN, a, st);  // team layout + MFMA (hd_team_mfma.hip)
  else
    hipLaunchKernelGGL(hd_rad_sweep_kernel<NN>, dim3((unsigned)((a.nu + 63) / 64)), dim3(64), 0,
                       st, a);
  const bool rad = radiances && a.numu > 0 && a.nphi > 0;
  // nstr 18..32 with radiances: the team user-angle kernel also forms the layers'
  // homogeneous constants (hd_team_mfma.hip), so the const kernel does not run
  const bool team_user =
      NN > kMaxRegNN && rad && a.numu <= rad_layer_record_doubles(NN) && !rad_user_rolled();
  // nstr <= 16 with radiances: the const kernel writes the angle-independent maps and
  // the user angles run hd_rad_user_map_kernel (HD_AB=1 HD_RAD_USER=direct: the
  // per-angle hd_rad_user_kernel)
  const bool umap = NN <= kMaxRegNN && rad && !rad_user_direct();
  RadArgs ac = a;
  ac.umap = umap ? 1 : 0;
  if (team_user) {
    (void)hd::launch_rad_team_user(NN, a, st);
  } else {
    const long nc = (long)a.ns * a.nlyr;
    hipLaunchKernelGGL(hd_rad_const_kernel<NN>, dim3((unsigned)((nc + 255) / 256), (unsigned)a.nm),
                       dim3(256), 0, st, ac);
  }
  const long nf = (long)a.ns * a.ntau;
  hipLaunchKernelGGL(hd_rad_flux_kernel<NN>, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, st,
                     a);
  if (rad) {
    const long nr = (long)a.ns * a.numu;
#ifndef HD_RAD_WIDE
    if (umap)
      hipLaunchKernelGGL(hd_rad_user_map_kernel<NN>, dim3((unsigned)((nr + 63) / 64), (unsigned)a.nm),
                         dim3(64), 0, st, ac);
    else
#endif
    if constexpr (NN > kMaxRegNN || HD_AB_VARIANTS) {
      if (!team_user)
        hipLaunchKernelGGL(hd_rad_user_kernel<NN>, dim3((unsigned)((nr + 63) / 64), (unsigned)a.nm),
                           dim3(64), 0, st, a);
    }
    const long na = (long)a.ns * a.nphi * a.ntau * a.numu;
    hipLaunchKernelGGL(hd_rad_azimuth_kernel, dim3((unsigned)((na + 255) / 256)), dim3(256), 0,
                       st, a);
    if (a.corint && a.tauc)
      hipLaunchKernelGGL(hd_rad_tms_kernel, dim3((unsigned)((na + 255) / 256)), dim3(256), 0, st,
                         a, 2 * NN);
  }
}

hipError_t launch_rad_chunk(int nn, const RadArgs& a, bool radiances, hipStream_t stream) {
  switch (nn) {
#ifndef HD_RAD_WIDE
    case 1: launch_rad<1>(a, radiances, stream); break;
    case 2: launch_rad<2>(a, radiances, stream); break;
    case 3: launch_rad<3>(a, radiances, stream); break;
    case 4: launch_rad<4>(a, radiances, stream); break;
    case 5: launch_rad<5>(a, radiances, stream); break;
    case 6: launch_rad<6>(a, radiances, stream); break;
    case 7: launch_rad<7>(a, radiances, stream); break;
    case 8: launch_rad<8>(a, radiances, stream); break;
    default: return wide::launch_rad_chunk(nn, a, radiances, stream);
#else
    case 9: launch_rad<9>(a, radiances, stream); break;
    case 10: launch_rad<10>(a, radiances, stream); break;
    case 11: launch_rad<11>(a, radiances, stream); break;
    case 12: launch_rad<12>(a, radiances, stream); break;
    case 13: launch_rad<13>(a, radiances, stream); break;
    case 14: launch_rad<14>(a, radiances, stream); break;
    case 15: launch_rad<15>(a, radiances, stream); break;
    case 16: launch_rad<16>(a, radiances, stream); break;
    default: return hipErrorInvalidValue;
#endif
  }
  return hipGetLastError();
}

#ifndef HD_RAD_WIDE
size_t rad_scratch_doubles_per_unit(int nn, int nlyr) {
  const size_t ne1r = (size_t)rad_layer_record_doubles(nn);
  return (size_t)nlyr * (ne1r + rad_rec_doubles(nn) + rad_bsub_doubles(nn) + 4 * nn) +
         (size_t)2 * nn;
}
#endif

#ifdef HD_RAD_WIDE
}  // namespace wide
#endif
}  // namespace hd
