// hd_device.hpp -- device-side building blocks of the flux-only discrete-ordinate
// solve (gfx950, FP64).  Everything here works on per-thread register arrays
// with compile-time indices (NN = nstr/2 is a template parameter), so the
// matrices of one layer problem live in VGPRs: one lane = one problem.
//
// Method: the DISORT m=0 equations (Stamnes et al. 1988;
// the cdisort 2.1.3 stages c_setdis/c_soleig/c_upbeam/c_upisot that pydisort
// @ afee3ec897f calls, cmake/pydisort.cmake:9-11) are solved through the
// symmetric form of the half-range eigenproblem (Cholesky + cyclic Jacobi) and
// per-layer reflection/transmission operators in the flux-weighted basis,
// which are symmetric and need only SPD (pivot-free) factorizations.
#pragma once

#include <hip/hip_runtime.h>

// Jacobi rotation angles in FP32 with FP64-normalised c, s (jacobi_os_round,
// team_jacobi_round); 0: the all-FP64 angle formulas
#ifndef HD_JACOBI_F32_ANGLE
#define HD_JACOBI_F32_ANGLE 1
#endif

namespace hd {

constexpr double kPi = 3.14159265358979323846;
// DISORT 2.0: ssalb == 1 is dithered to 1 - sqrt(10*DBL_EPSILON)
constexpr double kDither = 4.712160915387242e-08;

// Beam cosine: taken as given, as pydisort's forward passes it to cdisort, whose
// input check rejects umu0 outside (0, 1] when fbeam > 0 (c_chekin): the layer
// kernels set HD_STATUS_BAD_INPUT for it (and the beam stays off), so the call
// fails with HD_ENUMERIC.  harp's legacy driver floored umu0 at 1e-3 on the
// caller's side before calling cdisort (rt_solver_disort.cpp_:80); a caller that
// wants that convention clamps its umu0 array itself.

// relative distance of an eigenvalue k^2 from the beam resonance 1/mu0^2 within which
// the layer kernels run jacobi_os_polish
constexpr double kResPolish = 3.0e-4;

// per-thread status bits (mirrors include/hdisort.h)
constexpr int kStBadInput = 0x01;
constexpr int kStEigen = 0x02;
constexpr int kStNonFinite = 0x04;
constexpr int kStResonance = 0x10;
constexpr int kStPivot = 0x20;

// Quadrature constants for NN = nstr/2 nodes (kept in __constant__ memory,
// see hd_kernels.hip; uniform across the wave -> scalar loads).
template <int NN>
struct Quad {
  double mu[NN];          // Gauss-Legendre nodes on (0,1)
  double w[NN];           // weights, sum = 1
  double sd[NN];          // sqrt(w/mu)
  double g[NN];           // sqrt(w*mu)  (flux-weighted basis scale)
  double rmu[NN];         // 1/mu
  double rg[NN];          // 1/g = sd/w   (note w/sd = g)
  double pt[2 * NN][NN];  // P_l(mu_i), l < nstr
};

// ----------------------------------------------------------------------------
// reciprocal / reciprocal square root: hardware estimate + 2 Newton steps
// (no IEEE division sequence; inputs are finite and nonzero where used)
// ----------------------------------------------------------------------------
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

__device__ __forceinline__ double rsq_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  double e = fma(-h * y, y, 0.5);
  y = fma(y, e, y);
  e = fma(-h * y, y, 0.5);
  return fma(y, e, y);
}

// one Newton step from the hardware estimate (measured on gfx950: |rel err| of
// v_rsq_f64 <= 2^-24.2, so one step leaves <= ~4e-15): used for the Jacobi
// rotation parameters, where c^2 + s^2 - 1 = O(1e-14) per rotation is far
// below what the fluxes can see (checked against the oracle in tests/)
__device__ __forceinline__ double rsq_nr1(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  const double e = fma(-0.5 * x * y, y, 0.5);
  return fma(y, e, y);
}

// symmetric access to the upper triangle (i, j compile-time after unrolling)
#define HD_SYM(a, i, j) a[((i) < (j) ? (i) : (j))][((i) < (j) ? (j) : (i))]

// ----------------------------------------------------------------------------
// Planck radiance integrated over [wlo, whi] cm^-1 -- the DISORT PLKAVG series
// (c_planck_func1): power series below v=1.5, exponential series truncated by
// the VCP table, iterated Simpson for narrow intervals.
// ----------------------------------------------------------------------------
__device__ __forceinline__ double plkf(double x) { return x * x * x / expm1(x); }

__device__ inline double plkavg(double wlo, double whi, double t) {
  if (!(t >= 0.0) || !(whi > wlo) || wlo < 0.0) return __builtin_nan("");
  if (t < 1.0e-4) return 0.0;
  const double sigdpi = 5.67032e-8 / kPi;
  const double conc = 15.0 / (kPi * kPi * kPi * kPi);
  const double c2 = 1.438786;
  const double v0 = c2 * wlo / t, v1 = c2 * whi / t;
  const double t4 = t * t * t * t;
  if (v0 > 2.220446049250313e-16 && v1 < 709.782712893384 && (whi - wlo) / whi < 1.0e-2) {
    const double hh = v1 - v0;
    const double val0 = plkf(v0) + plkf(v1);
    double oldval = 0.0, val = 0.0;
    for (int n = 1; n <= 10; ++n) {
      const double del = hh / (2 * n);
      val = val0;
      for (int k = 1; k <= 2 * n - 1; ++k) val += 2 * (1 + k % 2) * plkf(v0 + k * del);
      val = del / 3.0 * val;
      if (fabs((val - oldval) / val) <= 1.0e-6) break;
      oldval = val;
    }
    return sigdpi * t4 * conc * val;
  }
  double pv[2] = {0.0, 0.0}, dv[2] = {0.0, 0.0};
  int smallv = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const double vi = i == 0 ? v0 : v1;
    if (vi < 1.5) {
      smallv++;
      const double vsq = vi * vi;
      pv[i] = conc * vsq * vi *
              (1.0 / 3.0 +
               vi * (-1.0 / 8.0 +
                     vi * (1.0 / 60.0 +
                           vsq * (-1.0 / 5040.0 +
                                  vsq * (1.0 / 272160.0 +
                                         vsq * (-1.0 / 13305600.0 + vsq * (1.0 / 622702080.0)))))));
    } else {
      const int mmax = vi >= 10.25 ? 1 : vi >= 5.7 ? 2 : vi >= 3.9 ? 3 : vi >= 2.9 ? 4
                       : vi >= 2.3 ? 5 : vi >= 1.9 ? 6 : 7;
      const double ex = exp(-vi);
      double exm = 1.0, di = 0.0;
      for (int m = 1; m <= mmax; ++m) {
        const double mv = m * vi;
        exm *= ex;
        const double m2 = (double)m * m;
        di += exm * (6.0 + mv * (6.0 + mv * (3.0 + mv))) / (m2 * m2);
      }
      dv[i] = conc * di;
    }
  }
  double val;
  if (smallv == 2) val = pv[1] - pv[0];
  else if (smallv == 1) val = 1.0 - pv[0] - dv[1];
  else val = dv[0] - dv[1];
  return sigdpi * t4 * val;
}

// ----------------------------------------------------------------------------
// small dense kernels on register arrays
// ----------------------------------------------------------------------------

// In-place Cholesky: reads the SPD matrix from the upper triangle of a and
// writes the lower factor (diagonal included) into the lower triangle of the
// same array (the strict upper triangle keeps the input); rd = 1/diag(L).
// NN-loops of the per-lane matrix helpers: fully unrolled (matrices in
// registers) -- unless the including translation unit asks for rolled loops
// (hd_rad_wide.hip: the intensity path at nstr 18..32, matrices in private memory)
#ifndef HD_UNROLL_NN
#define HD_UNROLL_NN _Pragma("unroll")
#endif

template <int NN>
__device__ __forceinline__ bool chol_inplace(double (&a)[NN][NN], double (&rd)[NN]) {
  // the pivot test is folded into an integer at each step and pinned there: left
  // as a bool the compiler sinks every `s > 0` to the caller's status update and
  // keeps the NN pivots live across everything in between
  int ok = 1;
HD_UNROLL_NN
  for (int j = 0; j < NN; ++j) {
    double s = a[j][j];
HD_UNROLL_NN
    for (int k = 0; k < j; ++k) s = fma(-a[j][k], a[j][k], s);
    ok &= s > 0.0 ? 1 : 0;
    asm volatile("" : "+v"(ok));
    s = s > 1e-300 ? s : 1e-300;
    const double r = rsq_nr(s);
    a[j][j] = s * r;
    rd[j] = r;
HD_UNROLL_NN
    for (int i = j + 1; i < NN; ++i) {
      double t = a[j][i];
HD_UNROLL_NN
      for (int k = 0; k < j; ++k) t = fma(-a[i][k], a[j][k], t);
      a[i][j] = t * r;
    }
  }
  return ok != 0;
}

// x <- L^-1 x (forward substitution, L lower, rd = 1/diag(L))
template <int NN>
__device__ __forceinline__ void lower_solve(const double (&l)[NN][NN], const double (&rd)[NN],
                                            double (&x)[NN]) {
HD_UNROLL_NN
  for (int i = 0; i < NN; ++i) {
    double s = x[i];
HD_UNROLL_NN
    for (int k = 0; k < i; ++k) s = fma(-l[i][k], x[k], s);
    x[i] = s * rd[i];
  }
}

// x <- L^-T x (back substitution with the transpose of lower L)
template <int NN>
__device__ __forceinline__ void lower_t_solve(const double (&l)[NN][NN], const double (&rd)[NN],
                                              double (&x)[NN]) {
HD_UNROLL_NN
  for (int i = NN - 1; i >= 0; --i) {
    double s = x[i];
HD_UNROLL_NN
    for (int k = i + 1; k < NN; ++k) s = fma(-l[k][i], x[k], s);
    x[i] = s * rd[i];
  }
}

// (L L^T)^-1 from the Cholesky factor left in the lower triangle of a (rd =
// 1/diag(L)): K = L^-1 (lower, NN^3/6 fma), then inv = K^T K written into the
// upper triangle of a (diagonal included; L's diagonal is not needed again).
template <int NN>
__device__ __forceinline__ void spd_inverse_upper(double (&a)[NN][NN], const double (&rd)[NN]) {
  double k[NN][NN];  // lower
HD_UNROLL_NN
  for (int j = 0; j < NN; ++j) {
    k[j][j] = rd[j];
HD_UNROLL_NN
    for (int i = j + 1; i < NN; ++i) {
      double t = 0.0;
HD_UNROLL_NN
      for (int m = j; m < i; ++m) t = fma(a[i][m], k[m][j], t);
      k[i][j] = -t * rd[i];
    }
  }
HD_UNROLL_NN
  for (int i = 0; i < NN; ++i)
HD_UNROLL_NN
    for (int j = i; j < NN; ++j) {
      double t = 0.0;
HD_UNROLL_NN
      for (int m = j; m < NN; ++m) t = fma(k[m][i], k[m][j], t);
      a[i][j] = t;
    }
}

// ----------------------------------------------------------------------------
// Jacobi eigensolver, parallel (round-robin tournament) ordering: a sweep is
// P-1 rounds of P/2 disjoint rotations (P = NN rounded up to even).  The
// rotations of a round are independent, so their parameters (sqrt, rcp, rsq)
// and updates interleave -- ILP for one wave per SIMD.
// ----------------------------------------------------------------------------
__host__ __device__ constexpr int tour_a(int P, int r, int k) {
  return k == 0 ? P - 1 : (r + k) % (P - 1);
}
__host__ __device__ constexpr int tour_b(int P, int r, int k) {
  return k == 0 ? r : (r - k + (P - 1)) % (P - 1);
}

template <int NN>
__device__ __forceinline__ void jacobi_round(int r, double (&a)[NN][NN], double (&v)[NN][NN],
                                             bool on) {
  constexpr int P = NN + (NN & 1);
  constexpr int H = P / 2;
  double cc[H], ss[H], tt[H];
HD_UNROLL_NN
  for (int k = 0; k < H; ++k) {
    const int x = tour_a(P, r, k), y = tour_b(P, r, k);
    const int p = x < y ? x : y, q = x < y ? y : x;
    if (q >= NN) continue;
    // with w = sqrt(d^2 + 4 a^2), u = |d| + w, z = 1/sqrt(2 w u):
    //   c = u z,  s = sgn(d) 2 a z,  t = s/c = sgn(d) 2a/u = sgn(d) 4 a w z^2
    // (the standard t = sgn(theta)/(|theta| + sqrt(theta^2+1)), theta = d/2a)
    const double apq = a[p][q];
    const double d = a[q][q] - a[p][p];
    const double w2 = fma(d, d, 4.0 * apq * apq);
    const bool rot = on && w2 > 1.0e-280;
    const double w2s = rot ? w2 : 1.0;
    const double w = w2s * rsq_nr1(w2s);
    const double u = fabs(d) + w;
    const double z = rsq_nr1(2.0 * w * u);
    const double sg = d < 0.0 ? -2.0 : 2.0;
    cc[k] = rot ? u * z : 1.0;
    ss[k] = rot ? sg * apq * z : 0.0;
    tt[k] = rot ? sg * apq * (2.0 * w) * (z * z) : 0.0;
  }
HD_UNROLL_NN
  for (int k = 0; k < H; ++k) {
    const int x = tour_a(P, r, k), y = tour_b(P, r, k);
    const int p = x < y ? x : y, q = x < y ? y : x;
    if (q >= NN) continue;
    const double c = cc[k], s = ss[k], t = tt[k];
    const double apq = a[p][q];
    a[p][p] = fma(-t, apq, a[p][p]);
    a[q][q] = fma(t, apq, a[q][q]);
    a[p][q] = on ? 0.0 : apq;
HD_UNROLL_NN
    for (int i = 0; i < NN; ++i) {
      if (i == p || i == q) continue;
      const double aip = HD_SYM(a, i, p);
      const double aiq = HD_SYM(a, i, q);
      HD_SYM(a, i, p) = fma(c, aip, -s * aiq);
      HD_SYM(a, i, q) = fma(s, aip, c * aiq);
    }
HD_UNROLL_NN
    for (int i = 0; i < NN; ++i) {
      const double vip = v[i][p];
      const double viq = v[i][q];
      v[i][p] = fma(c, vip, -s * viq);
      v[i][q] = fma(s, vip, c * viq);
    }
  }
}

// a (upper triangle, symmetric) -> eigenvalues on the diagonal, eigenvectors
// in the columns of v.  A lane that has converged stops rotating (exact
// no-ops), so its result does not depend on which solves share its wave; the
// loop exits when every lane of the wave has converged or after max_sweeps.
template <int NN>
__device__ __forceinline__ void jacobi_eig(double (&a)[NN][NN], double (&v)[NN][NN],
                                           int max_sweeps) {
HD_UNROLL_NN
  for (int i = 0; i < NN; ++i)
HD_UNROLL_NN
    for (int j = 0; j < NN; ++j) v[i][j] = (i == j) ? 1.0 : 0.0;
  if constexpr (NN > 1) {
    constexpr int P = NN + (NN & 1);
    for (int sweep = 0; sweep < max_sweeps; ++sweep) {
      double off = 0.0, dia = 0.0;
HD_UNROLL_NN
      for (int i = 0; i < NN; ++i) {
        dia = fma(a[i][i], a[i][i], dia);
HD_UNROLL_NN
        for (int j = i + 1; j < NN; ++j) off = fma(a[i][j], a[i][j], off);
      }
      const bool done = !(off > 1.0e-30 * dia);  // off-diagonal <~ 1e-15 relative
      if (__all(done)) break;
HD_UNROLL_NN
      for (int r = 0; r < P - 1; ++r) jacobi_round<NN>(r, a, v, !done);
    }
  }
}

// ----------------------------------------------------------------------------
// One-sided (Hestenes) Jacobi on the columns of B, Sym = B^T B.  A rotation of
// the column pair (p, q) is exactly the two-sided rotation of B^T B for that
// pair, with a_pp = |b_p|^2 and a_qq = |b_q|^2 tracked (exact at every sweep
// start) and a_pq = b_p.b_q formed from the columns, so Sym is never formed and
// the rotations are not accumulated: with B = B0 V the eigenvectors are
// V = B0^-1 B afterwards (two triangular solves in the layer kernel), and
// k^2 = |b_j|^2.  Per rotation: 2 NN fma for the dot product, 4 NN ops for the
// columns -- against 2(NN-2) + 2 NN mul/fma pairs for the two-sided update of
// Sym and V.  Same tournament ordering and parameter formulas as jacobi_round.
// ----------------------------------------------------------------------------
// Column scales: b_j = sg_j x_j (x is what the registers hold), so the rotation
//   b_p' = c (b_p - t b_q),  b_q' = c (b_q + t b_p)
// becomes  x_p' = x_p - (t sg_q / sg_p) x_q,  x_q' = x_q + (t sg_p / sg_q) x_p,
// sg' = c sg: one FMA per element instead of a MUL and an FMA (rs = 1/sg is
// carried beside sg; 1/c = (1 + t^2) c).  The tracked norms |b_p|^2, |b_q|^2 move
// by -/+ t (b_p.b_q) -- the two-sided Jacobi diagonal update, exact at the exact
// angle and stationary in t there, so the FP32 angle's error only enters at second
// order; the norms are recomputed from the columns at every sweep start anyway.
template <int NN, bool F64 = false>
__device__ __forceinline__ void jacobi_os_round(int r, double (&b)[NN][NN], double (&nrm)[NN],
                                                double (&sg)[NN], double (&rs)[NN], bool on,
                                                double& off) {
  constexpr int P = NN + (NN & 1);
  constexpr int H = P / 2;
  double tt[H], cc[H], gg[H];
HD_UNROLL_NN
  for (int k = 0; k < H; ++k) {
    const int x = tour_a(P, r, k), y = tour_b(P, r, k);
    const int p = x < y ? x : y, q = x < y ? y : x;
    if (q >= NN) continue;
    double g0 = 0.0, g1 = 0.0;  // two chains
HD_UNROLL_NN
    for (int i = 0; i < NN; ++i) {
      if (i % 2 == 0) g0 = fma(b[i][p], b[i][q], g0);
      else g1 = fma(b[i][p], b[i][q], g1);
    }
    const double gam = (g0 + g1) * (sg[p] * sg[q]);
    const double app = nrm[p], aqq = nrm[q];
    const double g2 = gam * gam;
    off += g2;
    const bool rot = on && g2 > 1.0e-30 * (app * aqq);
    const double d = aqq - app;
    double t;
    if constexpr (HD_JACOBI_F32_ANGLE && !F64) {
      // The angle in FP32, t = tan(theta) = sgn(d) 2 g / (|d| + sqrt(d^2 + 4 g^2));
      // c = 1/sqrt(1 + t^2) in FP64, so the rotation is orthogonal to FP64 rounding
      // whatever t is: an angle good to ~1e-7 only leaves ~1e-7 of g behind, which
      // the next sweep removes (quadratic convergence until off ~ 1e-7 of the
      // diagonal; the stop rule sits at 1e-8)
      const float df = (float)d, g2f = 2.0f * (float)gam;
      const float wf = __builtin_amdgcn_sqrtf(__builtin_fmaf(g2f, g2f, df * df));
      const float tf = (df < 0.0f ? -g2f : g2f) * __builtin_amdgcn_rcpf(__builtin_fabsf(df) + wf);
      t = rot ? (double)tf : 0.0;
    } else {
      // w = sqrt(d^2 + 4 g^2): t = sgn(d) 2 g / (|d| + w)
      const double w2 = rot ? fma(d, d, 4.0 * g2) : 1.0;
      const double w = w2 * rsq_nr(w2);
      t = rot ? (d < 0.0 ? -2.0 : 2.0) * gam * rcp_nr(fabs(d) + w) : 0.0;
    }
    tt[k] = t;
    // exactly 1 for t = 0.  The column scales accumulate one factor c per rotation;
    // the polish sweep (jacobi_os_polish) takes c to the last bit
    cc[k] = F64 ? rsq_nr(fma(t, t, 1.0)) : rsq_nr1(fma(t, t, 1.0));
    gg[k] = gam;
  }
HD_UNROLL_NN
  for (int k = 0; k < H; ++k) {
    const int x = tour_a(P, r, k), y = tour_b(P, r, k);
    const int p = x < y ? x : y, q = x < y ? y : x;
    if (q >= NN) continue;
    const double t = tt[k], c = cc[k];
    const double al = -t * (sg[q] * rs[p]), be = t * (sg[p] * rs[q]);
HD_UNROLL_NN
    for (int i = 0; i < NN; ++i) {
      const double bp = b[i][p], bq = b[i][q];
      b[i][p] = fma(al, bq, bp);
      b[i][q] = fma(be, bp, bq);
    }
    const double rc = fma(t, t, 1.0) * c;  // 1/c
    sg[p] *= c;
    sg[q] *= c;
    rs[p] *= rc;
    rs[q] *= rc;
    nrm[p] = fma(-t, gg[k], nrm[p]);
    nrm[q] = fma(t, gg[k], nrm[q]);
  }
}

// Sweeps until the sweep in which the off-diagonal Frobenius norm of B^T B
// (accumulated from the pairs' b_p.b_q as they were rotated) stayed below
// 1e-8 of its diagonal: quadratic convergence leaves ~1e-16 after it (the
// criterion of jacobi_eig, measured one sweep earlier).  A converged lane stops
// rotating (exact no-ops: t = 0), so its result does not depend on which
// solves share its wave; the loop exits when every lane has converged.  The
// column scales are folded back into b at the end.  Returns false when this lane
// left at max_sweeps still rotating (not converged: the caller sets the EIGEN
// status bit).
template <int NN>
__device__ __forceinline__ bool jacobi_os(double (&b)[NN][NN], int max_sweeps) {
  bool on = false;
  if constexpr (NN > 1) {
    constexpr int P = NN + (NN & 1);
    on = true;
    double sg[NN], rs[NN];
HD_UNROLL_NN
    for (int j = 0; j < NN; ++j) sg[j] = rs[j] = 1.0;
    for (int sweep = 0; sweep < max_sweeps; ++sweep) {
      double nrm[NN], dia = 0.0, off = 0.0;
HD_UNROLL_NN
      for (int j = 0; j < NN; ++j) {
        double t = 0.0;
HD_UNROLL_NN
        for (int i = 0; i < NN; ++i) t = fma(b[i][j], b[i][j], t);
        nrm[j] = t * (sg[j] * sg[j]);
        dia = fma(nrm[j], nrm[j], dia);
      }
HD_UNROLL_NN
      for (int r = 0; r < P - 1; ++r) jacobi_os_round<NN>(r, b, nrm, sg, rs, on, off);
      on = on && off > 1.0e-16 * dia;
      if (__all(!on)) break;
    }
HD_UNROLL_NN
    for (int j = 0; j < NN; ++j)
HD_UNROLL_NN
      for (int i = 0; i < NN; ++i) b[i][j] *= sg[j];
  }
  return !on;
}

// One more sweep with the angles in FP64 for the lanes that ask (need): the FP32
// angles of jacobi_os leave up to ~1e-7 of each pair's coupling at its last sweep --
// for pairs of small columns of a graded B that is ~1e-13 of their eigenvectors,
// below anything the fluxes see, except where the beam's particular solution divides
// by 1/mu0^2 - k^2: within 3e-4 of that resonance the layer kernels polish
// (profiles/r06/resonance.txt: a C4 layer at 2.3e-6 of it gave 8.7e-7 in the fluxes
// without the polish, 3e-9 with FP64 angles).  No-op for the other lanes; the wave
// skips it when no lane needs it.
template <int NN>
__device__ __forceinline__ void jacobi_os_polish(double (&b)[NN][NN], bool need) {
  if constexpr (NN > 1) {
    if (!__any(need)) return;
    constexpr int P = NN + (NN & 1);
    double sg[NN], rs[NN], nrm[NN], off = 0.0;
HD_UNROLL_NN
    for (int j = 0; j < NN; ++j) {
      sg[j] = rs[j] = 1.0;
      double t = 0.0;
HD_UNROLL_NN
      for (int i = 0; i < NN; ++i) t = fma(b[i][j], b[i][j], t);
      nrm[j] = t;
    }
HD_UNROLL_NN
    for (int r = 0; r < P - 1; ++r) jacobi_os_round<NN, true>(r, b, nrm, sg, rs, need, off);
HD_UNROLL_NN
    for (int j = 0; j < NN; ++j)
HD_UNROLL_NN
      for (int i = 0; i < NN; ++i) b[i][j] *= sg[j];
  }
}

// true when some eigenvalue k^2 = |b_j|^2 of the rotated B lies within `tol` (relative)
// of the beam resonance k^2 = r2 = 1/mu0^2
template <int NN>
__device__ __forceinline__ bool near_resonance(const double (&b)[NN][NN], double r2, double tol) {
  bool near = false;
HD_UNROLL_NN
  for (int j = 0; j < NN; ++j) {
    double k2 = 0.0;
HD_UNROLL_NN
    for (int i = 0; i < NN; ++i) k2 = fma(b[i][j], b[i][j], k2);
    near = near || fabs(r2 - k2) < tol * r2;
  }
  return near;
}

}  // namespace hd
