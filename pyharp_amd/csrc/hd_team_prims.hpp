// hd_team_prims.hpp -- the 16-lane team primitives shared by the team kernels
// (hd_team.hip: VALU products; hd_team_mfma.hip: FP64 MFMA products).
//
// Team layout: a team is one DPP row (16 lanes of a wave64); lane i owns row i
// of every NN x NN matrix and element i of every vector (lanes i >= NN carry
// zeros).  Cross-lane traffic inside a team is DPP (row_newbcast:k hands lane
// k's value to the whole team; row_ror and the mirrors give the XOR
// permutations of the parallel Jacobi ordering and the team sums) and
// ds_swizzle.
#pragma once

#include <utility>

#include "hd_kernels.hpp"

namespace hd {

struct QuadTablesTeam {
  Quad<9> q9;
  Quad<10> q10;
  Quad<11> q11;
  Quad<12> q12;
  Quad<13> q13;
  Quad<14> q14;
  Quad<15> q15;
  Quad<16> q16;
};
// each translation unit keeps its own __constant__ copy (no relocatable device
// code) and passes it here
template <int NN>
__device__ __forceinline__ const Quad<NN>& tquad(const QuadTablesTeam& t) {
  if constexpr (NN == 9) return t.q9;
  else if constexpr (NN == 10) return t.q10;
  else if constexpr (NN == 11) return t.q11;
  else if constexpr (NN == 12) return t.q12;
  else if constexpr (NN == 13) return t.q13;
  else if constexpr (NN == 14) return t.q14;
  else if constexpr (NN == 15) return t.q15;
  else return t.q16;
}

// host: the team tables from the per-nn host quadrature (hd_team.hip)
void fill_quad_tables_team(const QuadHost* per_nn /* [kMaxNN], index nn-1 */, QuadTablesTeam& t);

// hd_team_mfma.hip: its copy of the team tables, and the MFMA layer kernel
hipError_t upload_quad_tables_team_mfma(const QuadTablesTeam& t);
hipError_t upload_warm_tables_team(const QuadHost* per_nn);  // team Jacobi warm start
hipError_t launch_team_layer_mfma(int nn, const LayerArgs& la, hipStream_t stream);
hipError_t launch_team_sweep_mfma(int nn, const SweepArgs& sa, hipStream_t stream);

namespace team {

constexpr int kTeam = 16;
constexpr int kTeamBlock = 256;
constexpr int kTeamsPerBlock = kTeamBlock / kTeam;

// ---- compile-time loops (DPP controls must be immediates) -------------------
template <int B, class F, int... Is>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, B + Is>{}), ...);
}
// f(k) for k = B .. E-1 (ascending)
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (E > B) sfor_impl<B>(f, std::make_integer_sequence<int, E - B>{});
}
template <int B, class F, int... Is>
__device__ __forceinline__ void sfor_rev_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, B - Is>{}), ...);
}
// f(k) for k = E-1 .. B (descending)
template <int B, int E, class F>
__device__ __forceinline__ void sfor_rev(F&& f) {
  if constexpr (E > B) sfor_rev_impl<E - 1>(f, std::make_integer_sequence<int, E - B>{});
}
#define HD_K(x) decltype(x)::value

// ---- DPP primitives ----------------------------------------------------------
__device__ __forceinline__ int tlane() { return (int)(threadIdx.x & (kTeam - 1)); }

template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
  return __builtin_amdgcn_update_dpp(0.0, x, CTRL, 0xF, 0xF, true);  // every source lane valid
}
// value held by team lane K (row_newbcast:K)
template <int K>
__device__ __forceinline__ double bc(double x) {
  return dpp<0x150 + K>(x);
}
constexpr int quad_xor(int m) {
  return (0 ^ m) | ((1 ^ m) << 2) | ((2 ^ m) << 4) | ((3 ^ m) << 6);
}
// value held by team lane (i ^ M): XOR masks compose, so M = hi ^ lo is built
// from row_half_mirror (^7), row_ror:8 (^8), row_mirror (^15) and a quad_perm
template <int M>
__device__ __forceinline__ double xperm(double x) {
  static_assert(M > 0 && M < 16, "team XOR mask");
  constexpr int hi = M & 12;
  constexpr int lo = (hi == 4 || hi == 12) ? ((M & 3) ^ 3) : (M & 3);
  if constexpr (hi == 4) x = dpp<0x141>(x);
  else if constexpr (hi == 8) x = dpp<0x128>(x);
  else if constexpr (hi == 12) x = dpp<0x140>(x);
  if constexpr (lo != 0) x = dpp<quad_xor(lo)>(x);
  return x;
}
// value held by team lane (i ^ M) through the LDS crossbar (ds_swizzle, bit
// mode: and 0x1f, xor M inside each 32-lane half): no LDS storage, and the
// exchange issues on the LDS pipe instead of the VALU the Jacobi rounds saturate
template <int M>
__device__ __forceinline__ double xswz(double x) {
  static_assert(M > 0 && M < 16, "team XOR mask");
  constexpr int pat = 0x1F | (M << 10);
  const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(x), pat);
  const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(x), pat);
  return __hiloint2double(hi, lo);
}
// sum over the 16 lanes of the team (every lane receives a sum; the
// association differs per lane, so take bc<0>() where a uniform value matters)
__device__ __forceinline__ double team_sum(double x) {
  x += dpp<0x128>(x);
  x += dpp<0x124>(x);
  x += dpp<0x122>(x);
  x += dpp<0x121>(x);
  return x;
}

// ---- team linear algebra (lane i = row i) ------------------------------------

// Cholesky of the SPD matrix whose row i lane i holds in a.  Out: a = row i of
// L (zeros above the diagonal); lt = row i of L^T (column i of L) if WANT_LT;
// rd = 1/L_ii.  Returns false on a non-positive pivot (uniform over the team).
template <int NN, bool WANT_LT>
__device__ __forceinline__ bool team_chol(double (&a)[NN], double (&lt)[NN], double& rd) {
  const int i = tlane();
  // the pivot test is folded into an integer at each step and pinned there: left
  // as a bool the compiler sinks every `d > 0` to the caller's status update and
  // keeps all NN pivots live until then (spilled to scratch in the team kernels)
  int ok = 1;
  rd = 0.0;
  if constexpr (WANT_LT) sfor<0, NN>([&](auto J) { lt[HD_K(J)] = 0.0; });
  sfor<0, NN>([&](auto K) {
    constexpr int k = HD_K(K);
    double d = bc<k>(a[k]);
    ok &= d > 0.0 ? 1 : 0;
    asm volatile("" : "+v"(ok));
    d = d > 1.0e-300 ? d : 1.0e-300;
    const double r = rsq_nr(d);
    const double lkk = d * r;
    const double aik = a[k] * r;  // on lane k: d r = lkk (d is lane k's a[k])
    a[k] = i >= k ? aik : 0.0;
    if (i == k) rd = r;
    if constexpr (WANT_LT) {
      if (i == k) lt[k] = lkk;
    }
    sfor<k + 1, NN>([&](auto J) {
      constexpr int j = HD_K(J);
      const double ljk = bc<j>(a[k]);
      a[j] = fma(-a[k], ljk, a[j]);  // above the diagonal: zeroed at step j
      if constexpr (WANT_LT) {
        if (i == k) lt[j] = ljk;
      }
    });
  });
  return ok != 0;
}

// x <- L^-1 x  (x distributed: lane i holds x_i)
template <int NN>
__device__ __forceinline__ void team_lsolve(const double (&l)[NN], double rd, double& x) {
  const int i = tlane();
  sfor<0, NN>([&](auto K) {
    constexpr int k = HD_K(K);
    if (i == k) x *= rd;
    const double xk = bc<k>(x);
    if (i > k) x = fma(-l[k], xk, x);
  });
}

// x <- L^-T x  (lt = rows of L^T)
template <int NN>
__device__ __forceinline__ void team_usolve(const double (&lt)[NN], double rd, double& x) {
  const int i = tlane();
  sfor_rev<0, NN>([&](auto K) {
    constexpr int k = HD_K(K);
    if (i == k) x *= rd;
    const double xk = bc<k>(x);
    if (i < k) x = fma(-lt[k], xk, x);
  });
}

// X <- L^-T X  (X rows distributed)
template <int NN>
__device__ __forceinline__ void team_umsolve(const double (&lt)[NN], double rd, double (&x)[NN]) {
  const int i = tlane();
  sfor_rev<0, NN>([&](auto K) {
    constexpr int k = HD_K(K);
    const double sc = i == k ? rd : 1.0;
    sfor<0, NN>([&](auto J) { x[HD_K(J)] *= sc; });
    const double m = i < k ? lt[k] : 0.0;
    sfor<0, NN>([&](auto J) {
      constexpr int j = HD_K(J);
      x[j] = fma(-m, bc<k>(x[j]), x[j]);
    });
  });
}

// ---- Jacobi eigensolver, XOR parallel ordering --------------------------------
// Round M pairs lane i with lane i^M; rounds 1..15 cover every pair once.
template <int NN>
__host__ __device__ constexpr bool round_has_pair(int m) {
  for (int p = 0; p < NN; ++p)
    if ((p ^ m) > p && (p ^ m) < NN) return true;
  return false;
}

// One-sided (Hestenes) Jacobi on the columns of B: lane j holds column j of B.
// Round M rotates the column pair (j, j^M) to make the two orthogonal --
// exactly the two-sided Jacobi rotation of B^T B for that pair, built from
// column dot products -- so B^T B is never formed and no diagonal has to be
// fished out of a lane-indexed register.  Both lanes of a pair form their
// operands in the same order (products commute exactly), so the two rotations
// agree bitwise.  The rotations are not accumulated: with B = B0 V the
// eigenvectors come out afterwards as V = B0^-1 B (two triangular solves, see
// the layer kernel), which removes half of the cross-lane traffic per round.
constexpr double kJacobiTol2 = 1.0e-30;  // rotate while (b_p.b_q)^2 > tol |b_p|^2 |b_q|^2
// the last sweep needed: the one whose off-diagonal Frobenius norm of B^T B
// (accumulated from the pairs' b_p.b_q as they were rotated) stayed below 1e-8
// of its diagonal -- quadratic convergence leaves ~1e-16 after it (the register
// path's jacobi_os rule; at nstr = 32 one sweep fewer than a per-pair 1e-9 cosine
// bound for the same residual, ~4e-15)
constexpr double kJacobiLastFrob2 = 1.0e-16;

// Column scales (HD_JACOBI_SCALED): lane j holds b_j = sig_j x_j, so a rotation
//   b_p' = c b_p - s b_q  becomes  x_p' = x_p - (s sig_q / (c sig_p)) x_q,  sig_p' = c sig_p
// -- one FMA per element instead of a MUL and an FMA (c >= 1/sqrt(2), so the
// scales shrink by at most 2^-1/2 per rotation; they are folded back into x at
// every sweep start).  The rotation angle, the tracked norms and the stop rule
// are those of the unscaled form.
#ifndef HD_JACOBI_SCALED
#define HD_JACOBI_SCALED 1
#endif

template <int NN, int M>
__device__ __forceinline__ void team_jacobi_round(double (&b)[NN], double& own, double& sig,
                                                  bool on, double& off) {
  const int i = tlane();
  const int pi = i ^ M;
  double bq[NN];
  sfor<0, NN>([&](auto K) { bq[HD_K(K)] = xswz<M>(b[HD_K(K)]); });
  const double oth = xswz<M>(own);  // |b_partner|^2, tracked by the partner
  double g0 = 0.0, g1 = 0.0;  // two chains: the partner columns arrive in order
  sfor<0, NN>([&](auto K) {
    constexpr int k = HD_K(K);
    if constexpr (k % 2 == 0) g0 = fma(b[k], bq[k], g0);
    else g1 = fma(b[k], bq[k], g1);
  });
#if HD_JACOBI_SCALED
  const double sq = xswz<M>(sig);
  const double gam = (g0 + g1) * (sig * sq);
#else
  const double gam = g0 + g1;
#endif
  // the lane with the lower index (bit hb of i clear) holds column p, its partner q;
  // the q side's sign flips are XORs of the sign bit (no 64-bit selects):
  // d = a_qq - a_pp, se = -s on the p side, the norm update's cross term
  constexpr int hb = M >= 8 ? 3 : M >= 4 ? 2 : M >= 2 ? 1 : 0;
  const int qside = (i >> hb) & 1;
  const int qmask = (int)((unsigned)qside << 31);  // sign flip on the q side
  const int pmask = (int)((unsigned)qmask ^ 0x80000000u);  // sign flip on the p side
  auto flip = [](double x, int m) {
    return __hiloint2double(__double2hiint(x) ^ m, __double2loint(x));
  };
  const bool pair = i < NN && pi < NN;
  const double g2 = gam * gam, pq = own * oth;
  const bool r = on && pair && g2 > kJacobiTol2 * pq;
  off += pair ? g2 : 0.0;  // each pair counted by both of its lanes
  const double d = flip(oth - own, qmask);  // a_qq - a_pp on both sides (bitwise equal)
#if HD_JACOBI_F32_ANGLE
  // the angle in FP32, c and s normalised in FP64 (see jacobi_os_round)
  const float df = (float)d, g2f = 2.0f * (float)gam;
  const float wf = __builtin_amdgcn_sqrtf(__builtin_fmaf(g2f, g2f, df * df));
  const float tf = (df < 0.0f ? -g2f : g2f) * __builtin_amdgcn_rcpf(__builtin_fabsf(df) + wf);
  const double t = r ? (double)tf : 0.0;
  // c to the last bit: with HD_JACOBI_SCALED the column scale accumulates c
  // (jacobi_os_round)
  const double c = rsq_nr(fma(t, t, 1.0));  // exactly 1 for t = 0
  const double s = t * c;
#else
  // w = sqrt(d^2 + 4 g^2), u = |d| + w, z = 1/sqrt(2 w u): c = u z, s = sgn(d) 2 g z
  const double w2 = r ? fma(d, d, 4.0 * g2) : 1.0;
  const double w = w2 * rsq_nr1(w2);
  const double u = fabs(d) + w;
  const double z = rsq_nr1(2.0 * w * u);
  const double sg = d < 0.0 ? -2.0 : 2.0;
  const double c = r ? u * z : 1.0;
  const double s = r ? sg * gam * z : 0.0;
#endif
  const double se = flip(s, pmask);  // p side: c b_p - s b_q ; q side: s b_p + c b_q
#if HD_JACOBI_SCALED
  const double tq = se * sq * rcp_nr(c * sig);
  sfor<0, NN>([&](auto K) { b[HD_K(K)] = fma(tq, bq[HD_K(K)], b[HD_K(K)]); });
  sig *= c;
#else
  (void)sig;
  sfor<0, NN>([&](auto K) { b[HD_K(K)] = fma(se, bq[HD_K(K)], c * b[HD_K(K)]); });
#endif
  // rotated norms: |c b_p - s b_q|^2 and |s b_p + c b_q|^2 (own: this lane's column)
  const double cc = c * c, ss2 = s * s, cs2 = 2.0 * c * s * gam;
  own = fma(cc, own, fma(ss2, oth, flip(cs2, pmask)));
}

// Sweeps of rounds 1..15 until the sweep that was the last one needed
// (kJacobiLastFrob2), or max_sweeps.  A converged team issues no-op rotations
// (c = 1, s = 0) while its wave-mates finish.  Returns false when the team left
// at max_sweeps with pairs still rotating (the caller sets the EIGEN status bit).
template <int NN>
__device__ __forceinline__ bool team_jacobi(double (&b)[NN], int max_sweeps) {
  bool on = true;
  double sig = 1.0;  // b = sig x (HD_JACOBI_SCALED)
  for (int sweep = 0; sweep < max_sweeps; ++sweep) {
    double off = 0.0;  // this lane's sum of (b_p.b_q)^2 over its pairs in this sweep
    double own = 0.0;  // |b_j|^2, exact at the start of every sweep, then tracked
    sfor<0, NN>([&](auto K) {
      b[HD_K(K)] *= sig;
      own = fma(b[HD_K(K)], b[HD_K(K)], own);
    });
    sig = 1.0;
    const double dia = bc<0>(team_sum(own * own));  // sum_j |b_j|^4 (team-uniform)
    sfor<1, kTeam>([&](auto Mc) {
      constexpr int m = HD_K(Mc);
      if constexpr (round_has_pair<NN>(m)) team_jacobi_round<NN, m>(b, own, sig, on, off);
    });
    // every pair was counted twice (once per lane): compare 2x the bound
    on = on && bc<0>(team_sum(off)) > 2.0 * kJacobiLastFrob2 * dia;
    if (__all(!on)) break;
  }
  sfor<0, NN>([&](auto K) { b[HD_K(K)] *= sig; });
  return !on;
}

}  // namespace team

template <int NN>
constexpr int ne1t() {
  return 2 * NN * NN + 2 * NN + 2;
}
template <int NN>
constexpr int ne2t() {
  return (NN * NN + 2 * NN + 2) & ~1;
}

}  // namespace hd
