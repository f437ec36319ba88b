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

namespace hd {

constexpr double kPi = 3.14159265358979323846;
// DISORT 2.0: ssalb == 1 is dithered to 1 - sqrt(10*DBL_EPSILON)
constexpr double kDither = 4.712160915387242e-08;

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
  double pt[2 * NN][NN];  // P_l(mu_i), l < nstr
};

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

// Cholesky of the SPD matrix in the upper triangle of a -> lower factor l.
// returns false on breakdown.
template <int NN>
__device__ __forceinline__ bool chol_lower(const double (&a)[NN][NN], double (&l)[NN][NN]) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < NN; ++j) {
    double s = HD_SYM(a, j, j);
#pragma unroll
    for (int k = 0; k < j; ++k) s -= l[j][k] * l[j][k];
    ok = ok && (s > 0.0);
    const double d = sqrt(s > 0.0 ? s : 1e-300);
    const double rd = 1.0 / d;
    l[j][j] = d;
#pragma unroll
    for (int i = j + 1; i < NN; ++i) {
      double t = HD_SYM(a, i, j);
#pragma unroll
      for (int k = 0; k < j; ++k) t -= l[i][k] * l[j][k];
      l[i][j] = t * rd;
    }
  }
  return ok;
}

// In-place Cholesky: reads the SPD matrix from the upper triangle of a and
// writes the lower factor (diagonal included) into the lower triangle of the
// same array (the strict upper triangle keeps the input).
template <int NN>
__device__ __forceinline__ bool chol_inplace(double (&a)[NN][NN]) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < NN; ++j) {
    double s = a[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= a[j][k] * a[j][k];
    ok = ok && (s > 0.0);
    const double d = sqrt(s > 0.0 ? s : 1e-300);
    const double rd = 1.0 / d;
    a[j][j] = d;
#pragma unroll
    for (int i = j + 1; i < NN; ++i) {
      double t = a[j][i];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= a[i][k] * a[j][k];
      a[i][j] = t * rd;
    }
  }
  return ok;
}

// x <- L^-1 x (forward substitution, L lower)
template <int NN>
__device__ __forceinline__ void lower_solve(const double (&l)[NN][NN], double (&x)[NN]) {
#pragma unroll
  for (int i = 0; i < NN; ++i) {
    double s = x[i];
#pragma unroll
    for (int k = 0; k < i; ++k) s -= l[i][k] * x[k];
    x[i] = s / l[i][i];
  }
}

// x <- L^-T x (back substitution with the transpose of lower L)
template <int NN>
__device__ __forceinline__ void lower_t_solve(const double (&l)[NN][NN], double (&x)[NN]) {
#pragma unroll
  for (int i = NN - 1; i >= 0; --i) {
    double s = x[i];
#pragma unroll
    for (int k = i + 1; k < NN; ++k) s -= l[k][i] * x[k];
    x[i] = s / l[i][i];
  }
}

// One Jacobi rotation on the symmetric matrix a (upper triangle) zeroing
// a[p][q]; accumulates the rotation into the columns of v.
template <int NN, int P, int Q>
__device__ __forceinline__ void jacobi_rot(double (&a)[NN][NN], double (&v)[NN][NN], bool on) {
  const double apq = a[P][Q];
  const double app = a[P][P];
  const double aqq = a[Q][Q];
  const double d = aqq - app;
  const double den = fabs(d) + sqrt(d * d + 4.0 * apq * apq);
  double t = (den > 0.0 && on) ? 2.0 * apq / den : 0.0;  // converged lanes: exact no-op
  t = d < 0.0 ? -t : t;
  const double c = 1.0 / sqrt(1.0 + t * t);
  const double s = t * c;
  a[P][P] = app - t * apq;
  a[Q][Q] = aqq + t * apq;
  a[P][Q] = on ? 0.0 : apq;
#pragma unroll
  for (int r = 0; r < NN; ++r) {
    if (r == P || r == Q) continue;
    const double arp = HD_SYM(a, r, P);
    const double arq = HD_SYM(a, r, Q);
    HD_SYM(a, r, P) = c * arp - s * arq;
    HD_SYM(a, r, Q) = s * arp + c * arq;
  }
#pragma unroll
  for (int k = 0; k < NN; ++k) {
    const double vkp = v[k][P];
    const double vkq = v[k][Q];
    v[k][P] = c * vkp - s * vkq;
    v[k][Q] = s * vkp + c * vkq;
  }
}

template <int NN, int P, int Q>
struct JacobiSweep {
  __device__ __forceinline__ static void run(double (&a)[NN][NN], double (&v)[NN][NN], bool on) {
    jacobi_rot<NN, P, Q>(a, v, on);
    if constexpr (Q + 1 < NN) {
      JacobiSweep<NN, P, Q + 1>::run(a, v, on);
    } else if constexpr (P + 2 < NN) {
      JacobiSweep<NN, P + 1, P + 2>::run(a, v, on);
    }
  }
};

// Cyclic Jacobi: a (upper triangle, symmetric) -> eigenvalues on the diagonal,
// eigenvectors in the columns of v.  Sweeps until every lane of the wave has
// converged (wave-uniform exit) or max_sweeps.
template <int NN>
__device__ __forceinline__ void jacobi_eig(double (&a)[NN][NN], double (&v)[NN][NN],
                                           int max_sweeps) {
#pragma unroll
  for (int i = 0; i < NN; ++i)
#pragma unroll
    for (int j = 0; j < NN; ++j) v[i][j] = (i == j) ? 1.0 : 0.0;
  if constexpr (NN > 1) {
    for (int sweep = 0; sweep < max_sweeps; ++sweep) {
      double off = 0.0, dia = 0.0;
#pragma unroll
      for (int i = 0; i < NN; ++i) {
        dia += a[i][i] * a[i][i];
#pragma unroll
        for (int j = i + 1; j < NN; ++j) off += a[i][j] * a[i][j];
      }
      // per-lane convergence: a converged lane stops rotating, so its result
      // does not depend on which other solves share the wave
      const bool done = !(off > 1.0e-34 * dia);
      if (__all(done)) break;
      JacobiSweep<NN, 0, 1>::run(a, v, !done);
    }
  }
}

}  // namespace hd
