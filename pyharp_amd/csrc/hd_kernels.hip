// hd_kernels.hip -- gfx950 kernels of the flux-only discrete-ordinate solve.
//
//   hd_planck_kernel     one lane per (solve, level): Planck radiance of every
//                        level + surface + top emission   [cdisort c_planck_func1]
//   hd_layer_kernel<NN>  one lane per (solve, layer): delta-M, phase-matrix
//                        assembly, symmetric eigenproblem (Cholesky + Jacobi),
//                        beam/thermal particular solutions, and the layer's
//                        reflection/transmission operators + sources in the
//                        flux-weighted basis.   [c_setdis, c_soleig, c_upbeam,
//                        c_upisot]
//   hd_sweep_kernel<NN>  one lane per solve: adding sweep top->bottom,
//                        Lambertian surface, back-substitution bottom->top,
//                        level fluxes in harp layout.  [c_setmtx, c_solve0,
//                        c_fluxes; pydisort gather + level reversal]
//
// Scratch layout per chunk (solve-interleaved: lane = solve, so every global
// access of a wave is 64 consecutive doubles):
//   planck      [L+3][nsc]       B(level 0..L, harp order), B(btemp), temis*B(ttemp)
//   layer ops   [lc][pair][nsc] double2: RecL (R~ upper, T~ upper, S~+, S~-,
//                                tau'; 45 pairs at NN = 8)
//   back-sub    [lc][pair][nsc] double2: RecB (ZT column-major, t, rc, cs; 41
//                                pairs at NN = 8)
//   (16 bytes per lane and record access: half the memory instructions, so half
//   the vmcnt-ordered round trips of the one-wave-per-SIMD sweep)
#include <cmath>
#include <cstring>
#include <utility>
#include <vector>

#include "hd_kernels.hpp"

namespace hd {

// quadrature tables for every NN, in the constant address space
struct QuadTables {
  Quad<1> q1;
  Quad<2> q2;
  Quad<3> q3;
  Quad<4> q4;
  Quad<5> q5;
  Quad<6> q6;
  Quad<7> q7;
  Quad<8> q8;
};
__constant__ QuadTables c_quad;
// 1/n for the beam's Legendre recursion (uniform index: scalar loads)
__constant__ double c_inv_int[2 * kMaxRegNN + 2] = {
    0.0,        1.0,        1.0 / 2,  1.0 / 3,  1.0 / 4,  1.0 / 5,  1.0 / 6,
    1.0 / 7,    1.0 / 8,    1.0 / 9,  1.0 / 10, 1.0 / 11, 1.0 / 12, 1.0 / 13,
    1.0 / 14,   1.0 / 15,   1.0 / 16, 1.0 / 17};

template <int NN>
__device__ __forceinline__ const Quad<NN>& quad() {
  if constexpr (NN == 1) return c_quad.q1;
  else if constexpr (NN == 2) return c_quad.q2;
  else if constexpr (NN == 3) return c_quad.q3;
  else if constexpr (NN == 4) return c_quad.q4;
  else if constexpr (NN == 5) return c_quad.q5;
  else if constexpr (NN == 6) return c_quad.q6;
  else if constexpr (NN == 7) return c_quad.q7;
  else return c_quad.q8;
}
// the same table through a pointer the compiler cannot see through: inside a
// loop, products of table entries are then formed where used instead of being
// hoisted out of the loop and held (the column kernel's layer loop spilled 60 of
// them), and the entries come back by scalar loads
template <int NN>
__device__ __forceinline__ const Quad<NN>& quad_opaque() {
  const Quad<NN>* p = &quad<NN>();
  asm volatile("" : "+s"(p));
  return *p;
}

// one wave per block: a layer-kernel wave can take any SIMD the previous chunk's
// sweep leaves free (hd_solve runs the two on separate streams)
constexpr int kLayerBlock = 64;
// The layer kernel warms L2 with the prop record of the block dispatched this many blocks
// later (same XCD; 0: off).  Swept on the GPU, profiles/r06/layer_prefetch_ab.txt: layer
// kernel alone 1.70 -> 1.60-1.65 ms; C4 +0.7 %, the 8-GPU rank shape +4 % at 384.
#ifndef HD_LAYER_PREFETCH
#define HD_LAYER_PREFETCH 384
#endif
constexpr int kLayersPerBlock = kLayerBlock / 64;

// phase boundary: keeps the scheduler from hoisting the next phase's loads
// (and their registers) above the current phase
#define HD_PHASE() __builtin_amdgcn_sched_barrier(0)

// ============================================================================
// K0: Planck radiance per (solve, level)
// ============================================================================
__global__ __launch_bounds__(256) void hd_planck_kernel(PlanckArgs A) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int nl = A.nlyr + 3;
  if (tid >= (long)A.nsc * nl) return;
  const int lev = (int)(tid / A.nsc);
  const int sl = (int)(tid - (long)lev * A.nsc);
  const long s = solve_of(A.s0 + sl, A.cmaj, A.nwave, A.ncol);
  const int w = (int)(s / A.ncol);
  const int c = (int)(s - (long)w * A.ncol);
  double b;
  if (lev <= A.nlyr) {
    b = plkavg(A.wlo[w], A.whi[w], A.temf[(size_t)c * (A.nlyr + 1) + lev]);
  } else if (lev == A.nlyr + 1) {
    b = plkavg(A.wlo[w], A.whi[w], A.btemp ? A.btemp[s] : 0.0);
  } else {
    const double te = A.temis ? A.temis[s] : 0.0;
    b = te != 0.0 ? te * plkavg(A.wlo[w], A.whi[w], A.ttemp ? A.ttemp[s] : 0.0) : 0.0;
  }
  A.out[(size_t)lev * A.nsc + sl] = b;
}

// ============================================================================
// K0b: cumulative delta-M-scaled optical depth above every layer (beam only)
// ============================================================================
__global__ __launch_bounds__(256) void hd_tauc_kernel(TaucArgs A) {
  const long sl = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (sl >= A.nsc) return;
  const long s = solve_of(A.s0 + sl, A.cmaj, A.nwave, A.ncol);
  const int L = A.nlyr, np = A.nprop;
  const double* p = A.prop + (size_t)s * L * np;
  double tauc = 0.0;
  for (int lc = 0; lc < L; ++lc) {  // solver order: top (harp layer L-1) first
    const double* q = p + (size_t)(L - 1 - lc) * np;
    double a = np > 1 ? q[1] : 0.0;
    if (a == 1.0) a = 1.0 - kDither;
    const double f = A.use_f ? q[A.f_slot] : 0.0;
    A.out[(size_t)lc * A.nsc + sl] = tauc;
    tauc += (1.0 - a * f) * q[0];
  }
}

// ============================================================================
// K1: per-(solve, layer) setup
// ============================================================================
// Psi^T staging per lane; also holds L while the Jacobi runs (NN = 2: 5 > 4 doubles)
template <int NN>
__host__ __device__ constexpr int psi_doubles() {
  return NN > 1 ? (NN == 2 ? 5 : NN * NN) : 1;
}

// On-chip layer record of the column kernel: its layer setup writes the RecL
// elements here and its adding sweep reads them back -- no record in HBM.  R~ and
// S~+ (used first) stay in registers (compile-time indices after unrolling); T~,
// S~- and tau' (used after the sweep's LU) go to this lane's Psi^T staging area
// of LDS, free between the layer setup's last Psi^T read and the next layer's
// Jacobi, so that they are not live in registers across the LU.
template <int NN>
struct ColRec {
  using RL = RecL<NN>;
  static constexpr int kSm = even_up(RL::nsym);  // LDS slot of S~-[0]
  static_assert(kSm + (RL::Tau + 1 - RL::Sm) <= psi_doubles<NN>() || NN == 1,
                "T~, S~-, tau' do not fit the Psi^T staging area");
  double v[RL::T + even_up(NN)];  // R~ | S~+ (at RL::T ..)
  double* lds;                   // psi_lds + lane
  __device__ __forceinline__ int slot(int e) const { return e < RL::Sp ? e - RL::T : kSm + (e - RL::Sm); }
  __device__ __forceinline__ void put(int e, double x) {
    if (e < RL::T) v[e] = x;
    else if (e >= RL::Sp && e < RL::Sm) v[RL::T + (e - RL::Sp)] = x;
    else if (e <= RL::Tau) lds[slot(e) * kLayerBlock] = x;
  }
  __device__ __forceinline__ double get(int e) const {
    if (e < RL::T) return v[e];
    if (e >= RL::Sp && e < RL::Sm) return v[RL::T + (e - RL::Sp)];
    return lds[slot(e) * kLayerBlock];
  }
  __device__ __forceinline__ void close(int) {}
};

// The layer setup of (solve s, solver layer lc) into the record sink `out`
// (PairOut: RecL in HBM; ColRec: on chip).  psi_lds: this wave's Psi^T
// staging, element e of lane lt at e * kLayerBlock + lt.  Returns the status bits.
// OPQ: the quadrature table through quad_opaque (the column kernel's layer loop)
template <int NN, bool OPQ, class Out>
__device__ __forceinline__ int layer_body(const LayerArgs& A, long s, int sl, int lc,
                                          double* psi_lds, int lt, Out& out,
                                          const double* pf = nullptr, float* pf_sink = nullptr) {
  constexpr int N = 2 * NN;
  constexpr int kPsi = psi_doubles<NN>();
  const Quad<NN>& Qc = OPQ ? quad_opaque<NN>() : quad<NN>();
  const int L = A.nlyr;
  const int nm = A.nmom;
  const int np = A.nprop;
  int st = 0;

  // ---- inputs of this layer (harp layer L-1-lc) + delta-M (c_setdis) ----
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

  // ---- phase matrix even/odd parts (-A+ in ap, -A- in lch, upper) and the
  //      beam source vectors; one even/odd Legendre pair per iteration so the
  //      constant tables stream through a few scalar registers ----
  double lch[NN][NN], ap[NN][NN], xs[NN], xd[NN];
#pragma unroll
  for (int i = 0; i < NN; ++i) {
    xs[i] = xd[i] = 0.0;
#pragma unroll
    for (int j = i; j < NN; ++j) lch[i][j] = ap[i][j] = 0.0;
  }
  {
    double pprev = 0.0, pcur = 1.0;  // P_{l-1}(mu0), P_l(mu0) for the beam
#pragma nounroll
    for (int l2 = 0; l2 < NN; ++l2) {
      const int le = 2 * l2, lo = le + 1;
      const double che = le == 0 ? 1.0 : (le <= nm ? q[1 + le] : 0.0);
      const double cho = lo <= nm ? q[1 + lo] : 0.0;
      const double ge = (2 * le + 1) * (che - f) * rf;
      const double go = (2 * lo + 1) * (cho - f) * rf;
      const double pe0 = pcur;  // P_le(mu0)
      const double po0 = ((2 * lo - 1) * mub * pcur - (lo - 1) * pprev) * c_inv_int[lo];
      pprev = po0;
      pcur = ((2 * lo + 1) * mub * po0 - lo * pe0) * c_inv_int[lo + 1];
      double ue[NN], uo[NN];
#pragma unroll
      for (int i = 0; i < NN; ++i) {
        ue[i] = ge * Qc.pt[le][i];
        uo[i] = go * Qc.pt[lo][i];
        xs[i] = fma(ue[i], pe0, xs[i]);
        xd[i] = fma(uo[i], po0, xd[i]);
      }
#pragma unroll
      for (int i = 0; i < NN; ++i)
#pragma unroll
        for (int j = i; j < NN; ++j) {
          ap[i][j] = fma(ue[i], Qc.pt[le][j], ap[i][j]);
          lch[i][j] = fma(uo[i], Qc.pt[lo][j], lch[i][j]);
        }
    }
  }
#pragma unroll
  for (int i = 0; i < NN; ++i)
#pragma unroll
    for (int j = i; j < NN; ++j) {
      const double diag = (i == j) ? Qc.rmu[i] : 0.0;
      const double sij = Qc.sd[i] * Qc.sd[j];
      lch[i][j] = fma(-sij, lch[i][j], diag);
      ap[i][j] = fma(-sij, ap[i][j], diag);
    }
  // L L^T = -A-  (lower triangle of lch)
  double rdl[NN];
  if (!chol_inplace<NN>(lch, rdl)) st |= kStEigen;

  // ---- pre-Jacobi vectors (depend on L only) ----
  // beam: y2 = L^-1 W D^-1/2 rv, rv = -(M D^1/2)^-1 L L^T D^1/2 xs + M^-1 xd/mu0,
  //       lxd = L^-T L^-1 D^1/2 xd  (linv(xd) = (sd/w) lxd)
  double y2[NN], lxd[NN];
  const double fb2 = fb * (0.5 / kPi);
  if (beam) {
    double y[NN], z[NN];
#pragma unroll
    for (int i = 0; i < NN; ++i) y[i] = Qc.sd[i] * (fb2 * xs[i]);
#pragma unroll
    for (int i = 0; i < NN; ++i) {  // z = L^T y
      double t = 0.0;
#pragma unroll
      for (int k = i; k < NN; ++k) t = fma(lch[k][i], y[k], t);
      z[i] = t;
    }
#pragma unroll
    for (int i = 0; i < NN; ++i) {  // y = L z
      double t = 0.0;
#pragma unroll
      for (int k = 0; k <= i; ++k) t = fma(lch[i][k], z[k], t);
      y[i] = t;
    }
#pragma unroll
    for (int i = 0; i < NN; ++i) {
      // rv = (-y/sd + xd/mu0)/mu, with 1/(sd mu) = 1/g; W D^-1/2 = diag(w/sd) = diag(g)
      const double xdi = -fb2 * xd[i];
      const double rv = fma(-y[i], Qc.rg[i], xdi * rmu0 * Qc.rmu[i]);
      y2[i] = Qc.g[i] * rv;
      lxd[i] = Qc.sd[i] * xdi;
    }
    lower_solve<NN>(lch, rdl, y2);    // V^T y2 below (V = B K^-1 after the Jacobi)
    lower_solve<NN>(lch, rdl, lxd);   // lxd = L^-T L^-1 D^1/2 xd
    lower_t_solve<NN>(lch, rdl, lxd);
  } else {
#pragma unroll
    for (int i = 0; i < NN; ++i) y2[i] = lxd[i] = 0.0;
  }
  // thermal: cvec = dB + 2 (dB/tau') h,  h = W^-1 D^1/2 L^-T L^-1 D^1/2 mu
  double cvec[NN];
  double db = 0.0, bsum = 0.0;
  if (A.planck) {
    const double bt = A.planckv[(size_t)(L - lc) * A.nsc + sl];
    // a transparent layer carries its top level's Planck value through
    // (c_disort's xr1 = 0 when dtaucpr = 0: B(tau) = xr0 = B_top)
    const double bb = taup > 0.0 ? A.planckv[(size_t)(L - lc - 1) * A.nsc + sl] : bt;
    db = bb - bt;
    bsum = bt + bb;
    const double b1 = taup > 0.0 ? 2.0 * db / taup : 0.0;
#pragma unroll
    for (int i = 0; i < NN; ++i) cvec[i] = Qc.sd[i] * Qc.mu[i];
    lower_solve<NN>(lch, rdl, cvec);
    lower_t_solve<NN>(lch, rdl, cvec);
#pragma unroll
    for (int i = 0; i < NN; ++i) cvec[i] = fma(b1 * Qc.rg[i], cvec[i], db);
  } else {
#pragma unroll
    for (int i = 0; i < NN; ++i) cvec[i] = 0.0;
  }

  // ---- eigenpairs (c_soleig): Sym = L^T (-A+) L = V diag(k^2) V^T ----
  // With C C^T = -A+ (SPD exactly when Sym is), X = L^T C has X X^T = Sym: the
  // one-sided Jacobi on X's columns gives B = X W with orthogonal columns, and
  // Sym B = X (X^T X) W = B diag(k^2), so k_j = |b_j| and V = B K^-1 directly --
  // no triangular solve for the eigenvectors, and C is dead before the Jacobi.
  // X^T X = C^T (-A-) C is closer to diagonal than B0^T B0 for B0 = X^T (the
  // round-1..5 form): 4.0 instead of 4.8 sweeps per 64-lane wave at C4
  // (per lane 3.76 vs 3.86; numpy model of this loop).
  double rdc[NN];
  if (!chol_inplace<NN>(ap, rdc)) st |= kStEigen;  // lower ap <- C
  double v[NN][NN];  // X, then B = X W, then Omega = L B K^-1 Delta^1/2
#pragma unroll
  for (int i = 0; i < NN; ++i)
#pragma unroll
    for (int j = 0; j < NN; ++j) {  // X_ij = sum_{k >= max(i,j)} L_ki C_kj
      double t = 0.0;
#pragma unroll
      for (int k = (i > j ? i : j); k < NN; ++k) t = fma(lch[k][i], ap[k][j], t);
      v[i][j] = t;
    }
  // L is not needed again until the beam solution: park it in this lane's (not
  // yet used) Psi staging area of LDS while B and the rotation temporaries hold
  // the registers.
  constexpr int kPark = NN * (NN + 1) / 2 + NN;
  static_assert(kPark <= kPsi || NN == 1, "L does not fit the Psi staging area");
  if constexpr (NN > 1) {
    int e = 0;
#pragma unroll
    for (int i = 0; i < NN; ++i) {
#pragma unroll
      for (int k = 0; k <= i; ++k) psi_lds[(e++) * kLayerBlock + lt] = lch[i][k];
      psi_lds[(e++) * kLayerBlock + lt] = rdl[i];
    }
  }
  asm volatile("" ::: "memory");
#if HD_LAYER_PREFETCH
  // warm L2 with the record of the block dispatched HD_LAYER_PREFETCH blocks later (same
  // XCD): three LDS-DMA dword loads touch the lines of its (2 + nmom)-double record (144
  // bytes at C4; longer records are touched at their first 144 bytes); the data lands in
  // a sink nobody reads.  Issued here, after this layer's own loads are consumed
  // and L is parked, so the Jacobi's ~36 k cycles of pure VALU cover the round trip.
  if (pf) {
    using gp = const __attribute__((address_space(1))) void*;
    using lp = __attribute__((address_space(3))) void*;
    const int o1 = np > 16 ? 16 : np - 1, o2 = np > 17 ? 17 : np - 1;  // inside the record
    __builtin_amdgcn_global_load_lds((gp)(pf), (lp)(pf_sink), 4, 0, 0);
    __builtin_amdgcn_global_load_lds((gp)(pf + o1), (lp)(pf_sink), 4, 0, 0);
    __builtin_amdgcn_global_load_lds((gp)(pf + o2), (lp)(pf_sink), 4, 0, 0);
  }
#endif
  HD_PHASE();
  if (!jacobi_os<NN>(v, A.max_sweeps)) st |= kStEigen;
  jacobi_os_polish<NN>(v, beam && near_resonance<NN>(v, rmu0 * rmu0, kResPolish));
  HD_PHASE();
  double kk[NN], rk[NN];  // k_j = |b_j|, 1/k_j
#pragma unroll
  for (int j = 0; j < NN; ++j) {
    double k2 = 0.0;
#pragma unroll
    for (int i = 0; i < NN; ++i) k2 = fma(v[i][j], v[i][j], k2);
    if (!(k2 > 0.0)) st |= kStEigen;
    const double r = k2 > 0.0 ? rsq_nr(k2) : 0.0;
    kk[j] = k2 * r;
    rk[j] = r;
  }
  // beam, the part that needs only B and k (before L is back: y2 dies first)
  double ybt[NN];  // B K^-1 tt, tt = V^T y2 / (1/mu0^2 - k^2), V = B K^-1
  if (beam) {
    double tt[NN];
    const double r2 = rmu0 * rmu0;
#pragma unroll
    for (int j = 0; j < NN; ++j) {
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < NN; ++i) t = fma(v[i][j], y2[i], t);
      double den = fma(-kk[j], kk[j], r2);
      if (fabs(den) < 1.0e-9 * r2) {
        st |= kStResonance;
        den = den < 0.0 ? -1.0e-9 * r2 : 1.0e-9 * r2;
      }
      tt[j] = t * (rk[j] * rk[j]) * rcp_nr(den);  // K^-1 (V^T y2 / den)
    }
#pragma unroll
    for (int i = 0; i < NN; ++i) {
      double t = 0.0;
#pragma unroll
      for (int j = 0; j < NN; ++j) t = fma(v[i][j], tt[j], t);
      ybt[i] = t;
    }
  }
  HD_PHASE();
  if constexpr (NN > 1) {  // L back from LDS
    // the empty asm with a memory clobber makes this a real reload (not the
    // parked registers kept live across the Jacobi) and keeps it in place
    asm volatile("" ::: "memory");
    int e = 0;
#pragma unroll
    for (int i = 0; i < NN; ++i) {
#pragma unroll
      for (int k = 0; k <= i; ++k) lch[i][k] = psi_lds[(e++) * kLayerBlock + lt];
      rdl[i] = psi_lds[(e++) * kLayerBlock + lt];
    }
  }
  HD_PHASE();

  // ---- beam particular solution Z+/- (c_upbeam), unit attenuation above ----
  double zp[NN], zm[NN];
  double e0 = 0.0;
  if (beam) {
    double sv[NN], y[NN];
#pragma unroll
    for (int i = NN - 1; i >= 0; --i) {  // s = W^-1 D^1/2 L V tt = W^-1 D^1/2 L (B K^-1 tt)
      double t = 0.0;
#pragma unroll
      for (int k = 0; k <= i; ++k) t = fma(lch[i][k], ybt[k], t);
      sv[i] = Qc.rg[i] * t;
    }
    // dd = (lxd - D^1/2 L^-T L^-1 D^1/2 (mu s) / mu0) / w
#pragma unroll
    for (int i = 0; i < NN; ++i) y[i] = Qc.sd[i] * Qc.mu[i] * sv[i];
    lower_solve<NN>(lch, rdl, y);
    lower_t_solve<NN>(lch, rdl, y);
    // scaled depth of the layer top; without the prologue's depths the beam is
    // taken as unit at the top and the sweep applies exp(-tau_c/mu0)
    const double tauc = A.tauc ? A.tauc[(size_t)lc * A.nsc + sl] : 0.0;
    const double att = 0.5 * exp(-tauc * rmu0);
#pragma unroll
    for (int i = 0; i < NN; ++i) {
      const double dd = Qc.rg[i] * fma(-y[i], rmu0, lxd[i]);  // (sd/w)(lxd - y/mu0)
      zp[i] = (sv[i] + dd) * att;
      zm[i] = (sv[i] - dd) * att;
    }
    e0 = exp(-taup * rmu0);
  } else {
#pragma unroll
    for (int i = 0; i < NN; ++i) zp[i] = zm[i] = 0.0;
  }

  HD_PHASE();
  // ---- layer operators in the flux-weighted basis ----
  // Delta = tanh(k tau'/2)/k, Gamma = k tanh(k tau'/2): Gamma^1/2 K^-1 = Delta^1/2
  double dsq[NN];
#pragma unroll
  for (int j = 0; j < NN; ++j) {
    const double x = kk[j] * taup;
    const double m = -expm1(-x);           // 1 - exp(-k tau')
    const double th = m * rcp_nr(2.0 - m);  // tanh(k tau'/2)
    const double delta = x > 1.0e-8 ? th * rcp_nr(kk[j] > 0.0 ? kk[j] : 1.0) : 0.5 * taup;
    dsq[j] = delta > 0.0 ? delta * rsq_nr1(delta) : 0.0;
  }
  // Psi^T = L^-T V Gamma^1/2 = L^-T B Delta^1/2 -> LDS (one column per step)
#pragma unroll
  for (int j = 0; j < NN; ++j) {
    double x[NN];
#pragma unroll
    for (int i = 0; i < NN; ++i) x[i] = v[i][j] * dsq[j];
    lower_t_solve<NN>(lch, rdl, x);
#pragma unroll
    for (int i = 0; i < NN; ++i) psi_lds[(i * NN + j) * kLayerBlock + lt] = x[i];
  }
  HD_PHASE();
  // Omega = U Delta^1/2 = L B K^-1 Delta^1/2, in place over v (rows bottom-up)
#pragma unroll
  for (int j = 0; j < NN; ++j) {
    const double sc = rk[j] * dsq[j];
#pragma unroll
    for (int i = 0; i < NN; ++i) v[i][j] *= sc;
  }
#pragma unroll
  for (int i = NN - 1; i >= 0; --i)
#pragma unroll
    for (int j = 0; j < NN; ++j) {
      double t = 0.0;
#pragma unroll
      for (int k = 0; k <= i; ++k) t = fma(lch[i][k], v[k][j], t);
      v[i][j] = t;
    }
  HD_PHASE();

  using RL = RecL<NN>;
  constexpr int nsym = NN * (NN + 1) / 2;
  double ga[NN], gb[NN];
#pragma unroll
  for (int i = 0; i < NN; ++i) {
    ga[i] = Qc.g[i] * (cvec[i] - fma(-zp[i], e0, zm[i]));
    gb[i] = Qc.g[i] * (fma(zp[i], e0, zm[i]) + bsum);
  }
  // By Woodbury, Q~- = Omega (I + Omega^T Omega)^-1 Omega^T = I - A-  and
  // Q~+ = -Psi^T (I + Psi Psi^T)^-1 Psi = A+ - I  with the SPD inverses
  // A- = (I + Omega Omega^T)^-1, A+ = (I + Psi^T Psi)^-1 (eigenvalues in (0, 1]),
  // so R~ = A+ - A-, T~ = A- + A+ - I and the sources need A-/A+ times a vector.
  double pvec[NN], am_[NN][NN];
  {
#pragma unroll
    for (int i = 0; i < NN; ++i)
#pragma unroll
      for (int j = i; j < NN; ++j) {
        double t = (i == j) ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < NN; ++k) t = fma(v[i][k], v[j][k], t);
        am_[i][j] = t;
      }
    double rdh[NN];
    if (!chol_inplace<NN>(am_, rdh)) st |= kStEigen;
    spd_inverse_upper<NN>(am_, rdh);
#pragma unroll
    for (int i = 0; i < NN; ++i) {  // p = Q~- ga = ga - A- ga
      double t = ga[i];
#pragma unroll
      for (int j = 0; j < NN; ++j) t = fma(-HD_SYM(am_, i, j), ga[j], t);
      pvec[i] = t;
    }
  }
  double ap_[NN][NN], qvec[NN];
  {
    double pt_[NN][NN];  // pt_[i][j] = Psi^T[i][j]
#pragma unroll
    for (int i = 0; i < NN; ++i)
#pragma unroll
      for (int j = 0; j < NN; ++j) pt_[i][j] = psi_lds[(i * NN + j) * kLayerBlock + lt];
#pragma unroll
    for (int i = 0; i < NN; ++i)
#pragma unroll
      for (int j = i; j < NN; ++j) {
        double t = (i == j) ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < NN; ++k) t = fma(pt_[i][k], pt_[j][k], t);
        ap_[i][j] = t;
      }
    double rdh[NN];
    if (!chol_inplace<NN>(ap_, rdh)) st |= kStEigen;
    spd_inverse_upper<NN>(ap_, rdh);
#pragma unroll
    for (int i = 0; i < NN; ++i) {  // q = Q~+ gb = A+ gb - gb
      double t = -gb[i];
#pragma unroll
      for (int j = 0; j < NN; ++j) t = fma(HD_SYM(ap_, i, j), gb[j], t);
      qvec[i] = t;
    }
  }

  // ---- store: R~ = A+ - A-, T~ = A- + A+ - I (upper), S~+, S~-, tau' ----
  double chk = 0.0;
  {
    int e = 0;
#pragma unroll
    for (int i = 0; i < NN; ++i)
#pragma unroll
      for (int j = i; j < NN; ++j, ++e) {
        const double r = ap_[i][j] - am_[i][j];
        out.put(RL::R + e, r);
        chk += r;
      }
    out.close(RL::R + nsym - 1);
    e = 0;
#pragma unroll
    for (int i = 0; i < NN; ++i)
#pragma unroll
      for (int j = i; j < NN; ++j, ++e) {
        const double t = (am_[i][j] + ap_[i][j]) - ((i == j) ? 1.0 : 0.0);
        out.put(RL::T + e, t);
        chk += t;
      }
    out.close(RL::T + nsym - 1);
  }
  double smv[NN];
#pragma unroll
  for (int i = 0; i < NN; ++i) {
    const double sp = Qc.g[i] * (zp[i] * (1.0 - e0) - db) + pvec[i] - qvec[i];
    smv[i] = Qc.g[i] * (-zm[i] * (1.0 - e0) + db) - pvec[i] - qvec[i];
    out.put(RL::Sp + i, sp);
    chk += sp + smv[i];
  }
  out.close(RL::Sp + NN - 1);
#pragma unroll
  for (int i = 0; i < NN; ++i) out.put(RL::Sm + i, smv[i]);
  out.close(RL::Sm + NN - 1);
  out.put(RL::Tau, taup);
  // the pad after tau': the layer's direct-beam transmission e^(-tau'/mu0) (1
  // without a beam), from which hd_sweep_lean_kernel carries the beam down as a
  // running product instead of an exp of the running depth
  out.put(RL::Tau + 1, beam ? e0 : 1.0);
  if (!isfinite(chk + taup)) st |= kStNonFinite;
  return st;
}

template <int NN, bool NT>
__global__ __launch_bounds__(kLayerBlock) void hd_layer_kernel(LayerArgs A) {
  __shared__ double psi_lds[psi_doubles<NN>() * kLayerBlock];  // Psi^T staged per lane
  // block = 64 consecutive solves (one wave each) x kLayersPerBlock consecutive
  // layers: a wave's stores are coalesced (same layer, consecutive solves).
  // Neighbouring layers of a solve share 128-B lines of prop (18 doubles per
  // record), so the blocks of one solve tile are numbered layer-fastest and
  // dealt to the same XCD (blocks b and b + 8 share an XCD's L2): the second
  // reader of a line finds it in L2 instead of HBM
  const int lt = threadIdx.x;
  const int ntl = (A.nlyr + kLayersPerBlock - 1) / kLayersPerBlock;
  const int nb = (int)gridDim.x;
  auto tile_of = [&](int b, int& ts, int& tl) {
    const int x = b & 7, base = nb >> 3, extra = nb & 7;
    const int logical = x * base + (x < extra ? x : extra) + (b >> 3);
    ts = logical / ntl;
    tl = logical - ts * ntl;
  };
  int ts, tl;
  tile_of((int)blockIdx.x, ts, tl);
  const int sl = ts * 64 + (lt & 63);
  const int lc = tl * kLayersPerBlock + (lt >> 6);  // solver layer, 0 = top
  if (sl >= A.nsc || lc >= A.nlyr) return;
  const long s = solve_of(A.s0 + sl, A.cmaj, A.nwave, A.ncol);
  PairOutT<NT> out{reinterpret_cast<double2*>(A.scr) + (size_t)lc * RecL<NN>::pairs * A.nsc + sl,
                   (size_t)A.nsc, 0.0};
#if HD_LAYER_PREFETCH
  __shared__ float pf_sink[kLayerBlock];
  const double* pf = nullptr;
  if ((int)blockIdx.x + HD_LAYER_PREFETCH < nb) {
    int ts2, tl2;
    tile_of((int)blockIdx.x + HD_LAYER_PREFETCH, ts2, tl2);
    int sl2 = ts2 * 64 + (lt & 63);
    const int lc2 = tl2 * kLayersPerBlock + (lt >> 6);
    if (sl2 >= A.nsc) sl2 = A.nsc - 1;
    if (lc2 < A.nlyr) {
      const long s2 = solve_of(A.s0 + sl2, A.cmaj, A.nwave, A.ncol);
      pf = A.prop + ((size_t)s2 * A.nlyr + (A.nlyr - 1 - lc2)) * A.nprop;
    }
  }
  const int st = layer_body<NN, false>(A, s, sl, lc, psi_lds, lt, out, pf, pf_sink);
#else
  const int st = layer_body<NN, false>(A, s, sl, lc, psi_lds, lt, out);
#endif
  if (st) {
    atomicOr(&A.status[s], st);
    if (st & 0x0F) atomicOr(A.anyerr, 1);
  }
}

// ============================================================================
// K2: per-solve adding sweep + back-substitution
// ============================================================================
// The adding sweep of solve s (chunk lane sl): layer lc's record through
// rec_at(lc), a callable returning a getter e -> RecL element e (hd_sweep_kernel:
// loads from the HBM record; hd_column_kernel: the layer setup run right there
// into registers).  Stores the back-substitution records, the surface level and
// x; returns the status bits.
template <int NN, bool NT, class RecAt>
__device__ __forceinline__ int sweep_body(const SweepArgs& A, long sl, long s, RecAt&& rec_at) {
  const Quad<NN>& Qc = quad<NN>();
  const int L = A.nlyr;
  const size_t nsc = A.nsc;
  constexpr int nsym = NN * (NN + 1) / 2;
  int st = 0;

  const double mu0 = A.umu0 ? A.umu0[s] : 1.0;
  const double fb = A.fbeam ? A.fbeam[s] : 0.0;
  const bool beam = fb > 0.0 && mu0 > 0.0;
  const double alb = A.albedo ? A.albedo[s] : 0.0;
  if (!(alb >= 0.0) || !(alb <= 1.0)) st |= kStBadInput;
  double top = A.fisot ? A.fisot[s] : 0.0;
  double bsurf = 0.0;
  if (A.planck) {
    bsurf = A.planckv[(size_t)(L + 1) * nsc + sl];
    top += A.planckv[(size_t)(L + 2) * nsc + sl];
  }
  const double twopi = 2.0 * kPi;
  const double rmu0 = beam ? 1.0 / mu0 : 0.0;
  const double f0mu0 = beam ? fb * mu0 : 0.0;

  double ra[NN][NN];  // reflection of the stack above (upper triangle)
  double sd[NN];      // diffuse downward source at the current interface
#pragma unroll
  for (int i = 0; i < NN; ++i) {
    sd[i] = Qc.g[i] * top;
#pragma unroll
    for (int j = i; j < NN; ++j) ra[i][j] = 0.0;
  }
  double tauc = 0.0;

  for (int lc = 0; lc < L; ++lc) {
    using RL = RecL<NN>;
    using RB = RecB<NN>;
    auto rec = rec_at(lc);
    PairOutT<NT> bp{reinterpret_cast<double2*>(A.bsub) + (size_t)lc * RB::pairs * nsc + sl, nsc, 0.0};
    // this layer's R~ (upper) and S~+ ; each record element is read once
    double rl[NN][NN], spl[NN];
    {
      int e = 0;
#pragma unroll
      for (int i = 0; i < NN; ++i)
#pragma unroll
        for (int j = i; j < NN; ++j) rl[i][j] = rec(RL::R + (e++));
#pragma unroll
      for (int i = 0; i < NN; ++i) spl[i] = rec(RL::Sp + i);
    }
    // direct beam at the layer top; the sources of a unit-beam record scale with it
    const double eb = exp(-tauc * rmu0);
    const double sscale = A.beam_scale ? eb : 1.0;
#pragma unroll
    for (int i = 0; i < NN; ++i) spl[i] *= sscale;

    // level lc (top of layer lc): F_dn = rc . I+ + cs
    {
      double cs = 0.0;
#pragma unroll
      for (int i = 0; i < NN; ++i) {
        double t = 0.0;
#pragma unroll
        for (int j = 0; j < NN; ++j) t = fma(HD_SYM(ra, j, i), Qc.g[j], t);
        bp.put(RB::Rc + i, twopi * t);
        cs = fma(Qc.g[i], sd[i], cs);
      }
      bp.close(RB::Rc + NN - 1);
      bp.put(RB::Cs, fma(twopi, cs, f0mu0 * eb));
      bp.close(RB::Cs);
    }
    HD_PHASE();
    // A = Ra (full); W1 = I - R_l A ; v1 = R_l Sd + S+
    double am[NN][NN], w1[NN][NN], t1[NN];
#pragma unroll
    for (int i = 0; i < NN; ++i)
#pragma unroll
      for (int j = 0; j < NN; ++j) am[i][j] = HD_SYM(ra, i, j);
#pragma unroll
    for (int i = 0; i < NN; ++i) {
#pragma unroll
      for (int j = 0; j < NN; ++j) {
        double t = (i == j) ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < NN; ++k) t = fma(-HD_SYM(rl, i, k), am[k][j], t);
        w1[i][j] = t;
      }
      double t = spl[i];
#pragma unroll
      for (int k = 0; k < NN; ++k) t = fma(HD_SYM(rl, i, k), sd[k], t);
      t1[i] = t;
    }
    HD_PHASE();
    // LU without pivoting (W1 = I - product of reflections; pivot watch);
    // reciprocal pivots kept on the diagonal
#pragma unroll
    for (int k = 0; k < NN; ++k) {
      const double piv = w1[k][k];
      if (!(fabs(piv) > 1.0e-12)) st |= kStPivot;
      const double rp = rcp_nr(piv);
      w1[k][k] = rp;
#pragma unroll
      for (int i = k + 1; i < NN; ++i) {
        const double l = w1[i][k] * rp;
        w1[i][k] = l;
#pragma unroll
        for (int j = k + 1; j < NN; ++j) w1[i][j] = fma(-l, w1[k][j], w1[i][j]);
      }
    }
    // t = W1^-1 v1
#pragma unroll
    for (int i = 0; i < NN; ++i)
#pragma unroll
      for (int k = 0; k < i; ++k) t1[i] = fma(-w1[i][k], t1[k], t1[i]);
#pragma unroll
    for (int i = NN - 1; i >= 0; --i) {
#pragma unroll
      for (int k = i + 1; k < NN; ++k) t1[i] = fma(-w1[i][k], t1[k], t1[i]);
      t1[i] *= w1[i][i];
    }
    // u = A t + Sd
    double u[NN];
#pragma unroll
    for (int i = 0; i < NN; ++i) {
      double t = sd[i];
#pragma unroll
      for (int k = 0; k < NN; ++k) t = fma(am[i][k], t1[k], t);
      u[i] = t;
      bp.put(RB::Tv + i, t1[i]);
    }
    bp.close(RB::Tv + NN - 1);
    HD_PHASE();
    // M1 = A W1^-1, row-wise in place:  x W1 = a  ->  (x L) U = a
#pragma unroll
    for (int r = 0; r < NN; ++r) {
#pragma unroll
      for (int j = 0; j < NN; ++j) {  // z U = a  (forward over columns)
        double t = am[r][j];
#pragma unroll
        for (int k = 0; k < j; ++k) t = fma(-am[r][k], w1[k][j], t);
        am[r][j] = t * w1[j][j];
      }
#pragma unroll
      for (int j = NN - 1; j >= 0; --j) {  // x L = z  (backward, unit L)
        double t = am[r][j];
#pragma unroll
        for (int k = j + 1; k < NN; ++k) t = fma(-am[r][k], w1[k][j], t);
        am[r][j] = t;
      }
    }
    HD_PHASE();
    // T~ (upper), read once, with S~- and tau': the loads are issued before this
    // layer's ZT stores and Sd <- T_l u + S- is formed right away.  Loaded after the
    // stores (where Sd is first needed), each S~- element's s_waitcnt also waited for
    // all 32 ZT stores to retire -- four round trips per layer
    double tl[NN][NN];
    {
      int e = 0;
#pragma unroll
      for (int i = 0; i < NN; ++i)
#pragma unroll
        for (int j = i; j < NN; ++j) tl[i][j] = rec(RL::T + (e++));
    }
    {
      double sm_[NN];
#pragma unroll
      for (int i = 0; i < NN; ++i) sm_[i] = rec(RL::Sm + i);
      const double taul = rec(RL::Tau);
#pragma unroll
      for (int i = 0; i < NN; ++i) {
        double t = sm_[i] * sscale;
#pragma unroll
        for (int k = 0; k < NN; ++k) t = fma(HD_SYM(tl, i, k), u[k], t);
        sd[i] = t;
      }
      tauc += taul;
    }
#pragma unroll
    for (int j = 0; j < NN; ++j) {
      double x[NN];
#pragma unroll
      for (int i = 0; i < NN; ++i) x[i] = HD_SYM(tl, i, j);
#pragma unroll
      for (int i = 0; i < NN; ++i)
#pragma unroll
        for (int k = 0; k < i; ++k) x[i] = fma(-w1[i][k], x[k], x[i]);
#pragma unroll
      for (int i = NN - 1; i >= 0; --i) {
#pragma unroll
        for (int k = i + 1; k < NN; ++k) x[i] = fma(-w1[i][k], x[k], x[i]);
        x[i] *= w1[i][i];
      }
      // ZT column-major: column j is elements j NN .. j NN + NN-1
#pragma unroll
      for (int i = 0; i < NN; ++i) bp.put(RB::Z + j * NN + i, x[i]);
    }
    bp.close(RB::Z + NN * NN - 1);
    HD_PHASE();
    // P = M1 T_l (row-wise in place)
#pragma unroll
    for (int r = 0; r < NN; ++r) {
      double row[NN];
#pragma unroll
      for (int j = 0; j < NN; ++j) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < NN; ++k) t = fma(am[r][k], HD_SYM(tl, k, j), t);
        row[j] = t;
      }
#pragma unroll
      for (int j = 0; j < NN; ++j) am[r][j] = row[j];
    }
    HD_PHASE();
    // Ra <- R_l + T_l P (upper)
#pragma unroll
    for (int i = 0; i < NN; ++i) {
#pragma unroll
      for (int j = i; j < NN; ++j) {
        double t = rl[i][j];
#pragma unroll
        for (int k = 0; k < NN; ++k) t = fma(HD_SYM(tl, i, k), am[k][j], t);
        ra[i][j] = t;
      }
    }
  }

  // ---- Lambertian surface: I+ = g x ----
  double gsd = 0.0, grg = 0.0;
#pragma unroll
  for (int i = 0; i < NN; ++i) {
    gsd += Qc.g[i] * sd[i];
#pragma unroll
    for (int j = 0; j < NN; ++j) grg += Qc.g[i] * HD_SYM(ra, i, j) * Qc.g[j];
  }
  double esurf = (1.0 - alb) * bsurf;
  const double dirsurf = f0mu0 * exp(-tauc * rmu0);
  if (beam) esurf += alb * dirsurf / kPi;
  const double x = (2.0 * alb * gsd + esurf) / (1.0 - 2.0 * alb * grg);
  double ip[NN];
#pragma unroll
  for (int i = 0; i < NN; ++i) ip[i] = Qc.g[i] * x;
  double chk = 0.0;
  {
    double up = 0.0, dn = 0.0;
#pragma unroll
    for (int i = 0; i < NN; ++i) {
      up += Qc.g[i] * ip[i];
      double t = sd[i];
#pragma unroll
      for (int j = 0; j < NN; ++j) t += HD_SYM(ra, i, j) * ip[j];
      dn += Qc.g[i] * t;
    }
    const double f0 = twopi * up, f1 = twopi * dn + dirsurf;
    if (A.flux) {
      double* fo = A.flux + (size_t)s * (L + 1) * 2;
      fo[0] = f0;
      fo[1] = f1;
    }
    if (A.fsurf) {  // band epilogue: the back-substitution sums the surface level too
      A.fsurf[sl] = f0;
      A.fsurf[nsc + sl] = f1;
    }
    chk += f0 + f1;
  }
  A.xsurf[sl] = x;
  if (!isfinite(chk)) st |= kStNonFinite;
  return st;
}

template <int NN, bool NT>
__global__ __launch_bounds__(64) void hd_sweep_kernel(SweepArgs A) {
  const long sl = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (sl >= A.nsc) return;
  const long s = solve_of(A.s0 + sl, A.cmaj, A.nwave, A.ncol);
  const size_t nsc = A.nsc;
  auto rec_at = [&](int lc) {
    const double2* lp =
        reinterpret_cast<const double2*>(A.scr) + (size_t)lc * RecL<NN>::pairs * nsc + sl;
    return [lp, nsc](int e) { return pair_get<NT>(lp, nsc, e); };
  };
  const int st = sweep_body<NN, NT>(A, sl, s, rec_at);
  if (st) {
    atomicOr(&A.status[s], st);
    if (st & 0x0F) atomicOr(A.anyerr, 1);
  }
}

template <int NN, bool PRE, bool NT>
__device__ __forceinline__ void backsub_body(const SweepArgs& A);

#if HD_AB_VARIANTS
// ============================================================================
// K1+K2+K3 in one pass per solve (the column kernel): one lane walks its solve's
// layers top -> bottom, runs each layer's setup (layer_body) into registers and
// feeds it straight to the adding sweep (sweep_body), then walks back up through
// the back-substitution records it wrote (backsub_body).  The same source
// arithmetic as hd_layer_kernel + hd_sweep_kernel + the back-substitution (to
// rounding: the compiler may contract differently in the fused body), but the
// layer records (RecL: 90 doubles per (solve, layer), written once and read once)
// never reach HBM, and the three kernels' time-sharing of the SIMDs -- neither
// the layer kernel nor the sweep leaves room on a SIMD for the other -- becomes
// one instruction stream per wave.  Measured slower at one wave per SIMD (A/B
// only, HD_COLUMN; profiles/r05/column_ab.txt).
// ============================================================================
template <int NN>
__global__ __launch_bounds__(64) void hd_column_kernel(LayerArgs LA, SweepArgs A) {
  __shared__ double psi_lds[psi_doubles<NN>() * kLayerBlock];
  static_assert(kLayerBlock == 64, "column kernel: one wave per block");
  const int lt = threadIdx.x;
  const long sl = (long)blockIdx.x * 64 + lt;
  if (sl < A.nsc) {
    const long s = solve_of(A.s0 + sl, A.cmaj, A.nwave, A.ncol);
    ColRec<NN> r;
    r.lds = psi_lds + lt;
    int lst = 0;
    auto rec_at = [&](int lc) {
      lst |= layer_body<NN, true>(LA, s, (int)sl, lc, psi_lds, lt, r);
      return [&r](int e) { return r.get(e); };
    };
    const int st = sweep_body<NN, false>(A, sl, s, rec_at) | lst;
    if (st) {
      atomicOr(&A.status[s], st);
      if (st & 0x0F) atomicOr(A.anyerr, 1);
    }
  }
  // the back-substitution reads what this wave wrote (with the band epilogue, lanes
  // past the chunk read the last solve's records)
  __syncthreads();
  backsub_body<NN, true, false>(A);
}

// ============================================================================
// K2 for nstr 16 (NN = 8) at two waves per SIMD: the adding sweep of
// hd_sweep_kernel with the stack state (Ra packed upper, Sd) parked in LDS
// between its uses instead of in registers, and the layer's R~ / T~ read from
// the record where they are used.  hd_sweep_kernel holds Ra, R~, T~, W1 and
// M1/P together (492 VGPRs: one wave per SIMD, VALU busy half the time on its
// dependency chains); here at most W1 and one symmetric 8 x 8 matrix are live
// (<= 256 VGPRs), so two sweep waves share a SIMD and fill each other's stalls.
//   W1 = I - R~ Ra          Ra streamed from LDS, packed pair by pair
//   t1 = W1^-1 (R~ Sd + S+) pivot-free LU (hd_sweep_kernel's)
//   u  = Ra t1 + Sd         -> LDS (over Sd)
//   ZT = W1^-1 T~           column by column, stored
//   M1 = Ra W1^-1           row by row, upper triangle kept (M1 is symmetric)
//   Ra <- R~ + T~ (M1 T~)   column by column -> LDS; Sd <- T~ u + S-
// The level fluxes' row vector rc = 2 pi Ra g of the next level is formed while
// Ra is written and stored into that level's record.  Records as hd_sweep_kernel
// (RecL in, RecB out): the back-substitution kernels are shared.
// ============================================================================
template <int NN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
void hd_sweep_lean_kernel(SweepArgs A) {
  static_assert(NN % 2 == 0, "even NN: Sd fills whole pairs");
  constexpr int nsym = NN * (NN + 1) / 2;
  constexpr int kRaP = (nsym + 1) / 2;  // LDS pairs of packed Ra
  constexpr int kSdP = NN / 2;          // then Sd (or u)
  __shared__ double2 stk[kRaP + kSdP][64];
  const Quad<NN>& Qc = quad<NN>();
  const int lt = (int)threadIdx.x;
  const long sl = (long)blockIdx.x * blockDim.x + lt;
  if (sl >= A.nsc) return;  // one wave per block: no barrier below
  const long s = solve_of(A.s0 + sl, A.cmaj, A.nwave, A.ncol);
  const int L = A.nlyr;
  const size_t nsc = A.nsc;
  using RL = RecL<NN>;
  using RB = RecB<NN>;
  int st = 0;

  const double twopi = 2.0 * kPi;
  double f0mu0;
  {
    const double mu0 = A.umu0 ? A.umu0[s] : 1.0;
    const double fb = A.fbeam ? A.fbeam[s] : 0.0;
    f0mu0 = fb > 0.0 && mu0 > 0.0 ? fb * mu0 : 0.0;
  }

  // packed element e of Ra / element i of Sd in this lane's LDS slots
  auto ra_at = [&](int e) {
    const double2 q = stk[e >> 1][lt];
    return (e & 1) ? q.y : q.x;
  };
  auto sd_load = [&](double (&v)[NN]) {
#pragma unroll
    for (int p = 0; p < kSdP; ++p) {
      const double2 q = stk[kRaP + p][lt];
      v[2 * p] = q.x;
      v[2 * p + 1] = q.y;
    }
  };
  auto sd_store = [&](const double (&v)[NN]) {
#pragma unroll
    for (int p = 0; p < kSdP; ++p) stk[kRaP + p][lt] = make_double2(v[2 * p], v[2 * p + 1]);
  };
  {
    double top = A.fisot ? A.fisot[s] : 0.0;
    if (A.planck) top += A.planckv[(size_t)(L + 2) * nsc + sl];
    double sd0[NN];
#pragma unroll
    for (int i = 0; i < NN; ++i) sd0[i] = Qc.g[i] * top;
#pragma unroll
    for (int p = 0; p < kRaP; ++p) stk[p][lt] = make_double2(0.0, 0.0);
    sd_store(sd0);
    // level 0 (top): Ra = 0, so rc = 0 and cs = g . Sd
    PairOut bp{reinterpret_cast<double2*>(A.bsub) + sl, nsc, 0.0};
    double cs = 0.0;
#pragma unroll
    for (int i = 0; i < NN; ++i) {
      bp.put(RB::Rc + i, 0.0);
      cs = fma(Qc.g[i], sd0[i], cs);
    }
    bp.close(RB::Rc + NN - 1);
    bp.put(RB::Cs, fma(twopi, cs, f0mu0));
    bp.close(RB::Cs);
  }
  double eb = 1.0;  // direct beam at the layer top: running product of transmissions

  for (int lc = 0; lc < L; ++lc) {
    const double2* lp = reinterpret_cast<const double2*>(A.scr) + (size_t)lc * RL::pairs * nsc + sl;
    auto rec = [&](int e) { return pair_get(lp, nsc, e); };
    PairOut bp{reinterpret_cast<double2*>(A.bsub) + (size_t)lc * RB::pairs * nsc + sl, nsc, 0.0};
    const double sscale = A.beam_scale ? eb : 1.0;

    // ---- W1 = I - R Ra ; v1 = R Sd + S+  (each packed element of Ra once, in
    //      increasing k for every W1[i][j]: hd_sweep_kernel's fma order) ----
    double w1[NN][NN], t1[NN];
    {
      double rl[NN][NN];  // R~ upper
      {
        int e = 0;
#pragma unroll
        for (int i = 0; i < NN; ++i)
#pragma unroll
          for (int j = i; j < NN; ++j) rl[i][j] = rec(RL::R + (e++));
      }
#pragma unroll
      for (int i = 0; i < NN; ++i)
#pragma unroll
        for (int j = 0; j < NN; ++j) w1[i][j] = (i == j) ? 1.0 : 0.0;
      int e = 0;
#pragma unroll
      for (int a = 0; a < NN; ++a)
#pragma unroll
        for (int b = a; b < NN; ++b, ++e) {
          const double x = ra_at(e);  // Ra[a][b] = Ra[b][a]
#pragma unroll
          for (int i = 0; i < NN; ++i) {
            w1[i][b] = fma(-HD_SYM(rl, i, a), x, w1[i][b]);
            if (a != b) w1[i][a] = fma(-HD_SYM(rl, i, b), x, w1[i][a]);
          }
        }
      double sd[NN];
      sd_load(sd);
#pragma unroll
      for (int i = 0; i < NN; ++i) {
        double t = rec(RL::Sp + i) * sscale;
#pragma unroll
        for (int k = 0; k < NN; ++k) t = fma(HD_SYM(rl, i, k), sd[k], t);
        t1[i] = t;
      }
    }
    HD_PHASE();
    // LU without pivoting, reciprocal pivots on the diagonal (hd_sweep_kernel's)
#pragma unroll
    for (int k = 0; k < NN; ++k) {
      const double piv = w1[k][k];
      if (!(fabs(piv) > 1.0e-12)) st |= kStPivot;
      const double rp = rcp_nr(piv);
      w1[k][k] = rp;
#pragma unroll
      for (int i = k + 1; i < NN; ++i) {
        const double l = w1[i][k] * rp;
        w1[i][k] = l;
#pragma unroll
        for (int j = k + 1; j < NN; ++j) w1[i][j] = fma(-l, w1[k][j], w1[i][j]);
      }
    }
#pragma unroll
    for (int i = 0; i < NN; ++i)
#pragma unroll
      for (int k = 0; k < i; ++k) t1[i] = fma(-w1[i][k], t1[k], t1[i]);
#pragma unroll
    for (int i = NN - 1; i >= 0; --i) {
#pragma unroll
      for (int k = i + 1; k < NN; ++k) t1[i] = fma(-w1[i][k], t1[k], t1[i]);
      t1[i] *= w1[i][i];
    }
#pragma unroll
    for (int i = 0; i < NN; ++i) bp.put(RB::Tv + i, t1[i]);
    bp.close(RB::Tv + NN - 1);
    // u = Ra t1 + Sd -> LDS (Sd is not needed again)
    {
      double u[NN];
      sd_load(u);
      int e = 0;
#pragma unroll
      for (int a = 0; a < NN; ++a)
#pragma unroll
        for (int b = a; b < NN; ++b, ++e) {
          const double x = ra_at(e);
          u[a] = fma(x, t1[b], u[a]);
          if (a != b) u[b] = fma(x, t1[a], u[b]);
        }
      sd_store(u);
    }
    HD_PHASE();
    // ---- ZT = W1^-1 T~ column by column (stored) ----
    {
      double tl[NN][NN];
      {
        int e = 0;
#pragma unroll
        for (int i = 0; i < NN; ++i)
#pragma unroll
          for (int j = i; j < NN; ++j) tl[i][j] = rec(RL::T + (e++));
      }
#pragma unroll
      for (int j = 0; j < NN; ++j) {
        double x[NN];
#pragma unroll
        for (int i = 0; i < NN; ++i) x[i] = HD_SYM(tl, i, j);
#pragma unroll
        for (int i = 0; i < NN; ++i)
#pragma unroll
          for (int k = 0; k < i; ++k) x[i] = fma(-w1[i][k], x[k], x[i]);
#pragma unroll
        for (int i = NN - 1; i >= 0; --i) {
#pragma unroll
          for (int k = i + 1; k < NN; ++k) x[i] = fma(-w1[i][k], x[k], x[i]);
          x[i] *= w1[i][i];
        }
#pragma unroll
        for (int i = 0; i < NN; ++i) bp.put(RB::Z + j * NN + i, x[i]);
      }
      bp.close(RB::Z + NN * NN - 1);
    }
    HD_PHASE();
    // ---- M1 = Ra W1^-1 (upper): row r solves x W1 = Ra[r,:] -> (x L) U = a ----
    double m1[NN][NN];
    {
#pragma unroll
      for (int r = 0; r < NN; ++r) {
        double x[NN];
#pragma unroll
        for (int j = 0; j < NN; ++j) {  // z U = a (forward over columns)
          double t = ra_at(sym_index<NN>(r, j));
#pragma unroll
          for (int k = 0; k < j; ++k) t = fma(-x[k], w1[k][j], t);
          x[j] = t * w1[j][j];
        }
#pragma unroll
        for (int j = NN - 1; j >= r; --j) {  // x L = z (backward, unit L): j >= r only
          double t = x[j];
#pragma unroll
          for (int k = j + 1; k < NN; ++k) t = fma(-x[k], w1[k][j], t);
          x[j] = t;
        }
#pragma unroll
        for (int j = r; j < NN; ++j) m1[r][j] = x[j];
      }
    }
    HD_PHASE();
    // ---- Ra <- R~ + T~ P, P = M1 T~ (column by column) ; Sd <- T~ u + S- ----
    {
      double tl[NN][NN];
      {
        int e = 0;
#pragma unroll
        for (int i = 0; i < NN; ++i)
#pragma unroll
          for (int j = i; j < NN; ++j) tl[i][j] = rec(RL::T + (e++));
      }
      double rcn[NN];
#pragma unroll
      for (int i = 0; i < NN; ++i) rcn[i] = 0.0;
      double* ldsd = reinterpret_cast<double*>(&stk[0][0]);
#pragma unroll
      for (int j = 0; j < NN; ++j) {
        double pc[NN];
#pragma unroll
        for (int k = 0; k < NN; ++k) {
          double t = 0.0;
#pragma unroll
          for (int m = 0; m < NN; ++m) t = fma(HD_SYM(m1, k, m), HD_SYM(tl, m, j), t);
          pc[k] = t;
        }
#pragma unroll
        for (int i = 0; i <= j; ++i) {
          const int e = sym_index<NN>(i, j);
          double t = rec(RL::R + e);
#pragma unroll
          for (int k = 0; k < NN; ++k) t = fma(HD_SYM(tl, i, k), pc[k], t);
          ldsd[((e >> 1) * 64 + lt) * 2 + (e & 1)] = t;
          rcn[i] = fma(t, Qc.g[j], rcn[i]);
          if (i != j) rcn[j] = fma(t, Qc.g[i], rcn[j]);
        }
      }
      double u[NN], sdn[NN];
      sd_load(u);
      double cs = 0.0;
#pragma unroll
      for (int i = 0; i < NN; ++i) {
        double t = rec(RL::Sm + i) * sscale;
#pragma unroll
        for (int k = 0; k < NN; ++k) t = fma(HD_SYM(tl, i, k), u[k], t);
        sdn[i] = t;
        cs = fma(Qc.g[i], t, cs);
      }
      sd_store(sdn);
      eb *= rec(RL::Tau + 1);
      if (lc + 1 < L) {  // level lc+1 (top of layer lc+1): F_dn = rc . I+ + cs
        PairOut bn{reinterpret_cast<double2*>(A.bsub) + (size_t)(lc + 1) * RB::pairs * nsc + sl,
                   nsc, 0.0};
#pragma unroll
        for (int i = 0; i < NN; ++i) bn.put(RB::Rc + i, twopi * rcn[i]);
        bn.close(RB::Rc + NN - 1);
        bn.put(RB::Cs, fma(twopi, cs, f0mu0 * eb));
        bn.close(RB::Cs);
      }
    }
    HD_PHASE();
  }

  // ---- Lambertian surface: I+ = g x (hd_sweep_kernel's arithmetic) ----
  double ra[NN][NN], sd[NN];
  {
    int e = 0;
#pragma unroll
    for (int i = 0; i < NN; ++i)
#pragma unroll
      for (int j = i; j < NN; ++j) ra[i][j] = ra_at(e++);
    sd_load(sd);
  }
  // (surface inputs read here: nothing of them is live across the layer loop)
  const double alb = A.albedo ? A.albedo[s] : 0.0;
  if (!(alb >= 0.0) || !(alb <= 1.0)) st |= kStBadInput;
  const double bsurf = A.planck ? A.planckv[(size_t)(L + 1) * nsc + sl] : 0.0;
  const bool beam = f0mu0 > 0.0;
  double gsd = 0.0, grg = 0.0;
#pragma unroll
  for (int i = 0; i < NN; ++i) {
    gsd += Qc.g[i] * sd[i];
#pragma unroll
    for (int j = 0; j < NN; ++j) grg += Qc.g[i] * HD_SYM(ra, i, j) * Qc.g[j];
  }
  double esurf = (1.0 - alb) * bsurf;
  const double dirsurf = f0mu0 * eb;
  if (beam) esurf += alb * dirsurf / kPi;
  const double x = (2.0 * alb * gsd + esurf) / (1.0 - 2.0 * alb * grg);
  double chk = 0.0;
  {
    double up = 0.0, dn = 0.0;
#pragma unroll
    for (int i = 0; i < NN; ++i) {
      const double ipi = Qc.g[i] * x;
      up += Qc.g[i] * ipi;
      double t = sd[i];
#pragma unroll
      for (int j = 0; j < NN; ++j) t += HD_SYM(ra, i, j) * (Qc.g[j] * x);
      dn += Qc.g[i] * t;
    }
    const double f0 = twopi * up, f1 = twopi * dn + dirsurf;
    if (A.flux) {
      double* fo = A.flux + (size_t)s * (L + 1) * 2;
      fo[0] = f0;
      fo[1] = f1;
    }
    if (A.fsurf) {
      A.fsurf[sl] = f0;
      A.fsurf[nsc + sl] = f1;
    }
    chk += f0 + f1;
  }
  A.xsurf[sl] = x;
  if (!isfinite(chk)) st |= kStNonFinite;
  if (st) {
    atomicOr(&A.status[s], st);
    if (st & 0x0F) atomicOr(A.anyerr, 1);
  }
}

#endif  // HD_AB_VARIANTS

// ============================================================================
// K2 for nstr 4 and 8 (NN = 2, 4) in NN-lane teams: the adding sweep of
// hd_sweep_kernel with one solve per team, lane i holding row i of every NN x NN
// matrix (A = Ra, R~, T~, W1, ZT, P) and element i of every vector; rows reach
// the team's other lanes by DPP quad permutations (one v_mov_b64_dpp per element,
// no LDS).  At these sizes the one-lane sweep is latency-bound -- a call of a few
// hundred or thousand solves runs one or two waves per SIMD, each walking its
// layers through dependent chains (C1 amars_lw: 16 solves, ~70 us of a ~120 us
// step) -- and NN lanes per solve cut each lane's chain by ~NN and give the SIMDs
// NN times the waves.  The pivot-free LU becomes a Gauss-Jordan elimination of
// [W1 | T~ | v1] with the same pivots (lane i ends with row i of ZT = W1^-1 T~
// and t1_i); records as the one-lane sweep (RecL in, RecB out), so the
// back-substitution kernels are shared.
// ============================================================================
namespace {
// lane k of this lane's NN-lane team (NN = 2: pairs, 4: quads) via quad_perm
template <int NN, int K>
__device__ __forceinline__ double qbc(double x) {
  constexpr int ctrl = NN == 4 ? (K | (K << 2) | (K << 4) | (K << 6))
                               : (K | (K << 2) | ((2 + K) << 4) | ((2 + K) << 6));
  return __builtin_amdgcn_update_dpp(0.0, x, ctrl, 0xF, 0xF, true);
}
// sum over the team (a butterfly: every lane holds the same bits)
template <int NN>
__device__ __forceinline__ double qsum(double x) {
  x += __builtin_amdgcn_update_dpp(0.0, x, 1 | (0 << 2) | (3 << 4) | (2 << 6), 0xF, 0xF, true);
  if constexpr (NN == 4)
    x += __builtin_amdgcn_update_dpp(0.0, x, 2 | (3 << 2) | (0 << 4) | (1 << 6), 0xF, 0xF, true);
  return x;
}
template <int B, int E, class F, int... Is>
__device__ __forceinline__ void qfor_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, B + Is>{}), ...);
}
template <int B, int E, class F>
__device__ __forceinline__ void qfor(F&& f) {  // f(k), k = B .. E-1 (compile-time)
  if constexpr (E > B) qfor_impl<B, E>(f, std::make_integer_sequence<int, E - B>{});
}
#define HD_Q(x) decltype(x)::value
}  // namespace

template <int NN>
__global__ __launch_bounds__(64) void hd_sweep_quad_kernel(SweepArgs A) {
  static_assert(NN == 2 || NN == 4, "pair / quad teams");
  const Quad<NN>& Qc = quad<NN>();
  const int lane = (int)threadIdx.x;
  const int i = lane & (NN - 1);
  const long slq = ((long)blockIdx.x * 64 + lane) / NN;
  // a team past the chunk repeats the chunk's last solve and stores nothing: every
  // lane of a quad takes part in its DPP exchanges
  const bool valid = slq < A.nsc;
  const long sl = valid ? slq : A.nsc - 1;
  const long s = solve_of(A.s0 + sl, A.cmaj, A.nwave, A.ncol);
  const int L = A.nlyr;
  const size_t nsc = A.nsc;
  using RL = RecL<NN>;
  using RB = RecB<NN>;
  int st = 0;

  const double mu0 = A.umu0 ? A.umu0[s] : 1.0;
  const double fb = A.fbeam ? A.fbeam[s] : 0.0;
  const bool beam = fb > 0.0 && mu0 > 0.0;
  const double alb = A.albedo ? A.albedo[s] : 0.0;
  if (!(alb >= 0.0) || !(alb <= 1.0)) st |= kStBadInput;
  double top = A.fisot ? A.fisot[s] : 0.0;
  double bsurf = 0.0;
  if (A.planck) {
    bsurf = A.planckv[(size_t)(L + 1) * nsc + sl];
    top += A.planckv[(size_t)(L + 2) * nsc + sl];
  }
  const double twopi = 2.0 * kPi;
  const double rmu0 = beam ? 1.0 / mu0 : 0.0;
  const double f0mu0 = beam ? fb * mu0 : 0.0;
  const double g_i = Qc.g[i];
  // record element e of this solve in a layer's record ([pair][nsc] of double2)
  auto eoff = [&](int e) { return ((size_t)(e >> 1) * nsc + sl) * 2 + (e & 1); };

  double ra[NN];  // row i of the reflection of the stack above
#pragma unroll
  for (int j = 0; j < NN; ++j) ra[j] = 0.0;
  double sd = g_i * top;
  double tauc = 0.0;

  // layer records one layer ahead: a wave walks its layers one after another, and
  // at 16 or 20 000 solves nothing else hides a record load's latency (C1 is one wave)
  double rn[NN], tn[NN], spn, smn, tpn;
  auto fetch = [&](int lc) {
    const double* lb = A.scr + (size_t)lc * RL::pairs * nsc * 2;
#pragma unroll
    for (int j = 0; j < NN; ++j) {
      rn[j] = lb[eoff(RL::R + sym_index<NN>(i, j))];
      tn[j] = lb[eoff(RL::T + sym_index<NN>(i, j))];
    }
    spn = lb[eoff(RL::Sp + i)];
    smn = lb[eoff(RL::Sm + i)];
    tpn = lb[eoff(RL::Tau)];
  };
  fetch(0);
  for (int lc = 0; lc < L; ++lc) {
    double* bb = A.bsub + (size_t)lc * RB::pairs * nsc * 2;
    double r[NN], tr[NN];
#pragma unroll
    for (int j = 0; j < NN; ++j) {
      r[j] = rn[j];
      tr[j] = tn[j];
    }
    const double eb = exp(-tauc * rmu0);
    const double sscale = A.beam_scale ? eb : 1.0;
    const double spl = spn * sscale;
    const double sml = smn * sscale;
    const double taup = tpn;
    fetch(lc + 1 < L ? lc + 1 : lc);

    // level lc (top of layer lc): F_dn = rc . I+ + cs  (A symmetric: column i = row i)
    {
      double rc = 0.0;
#pragma unroll
      for (int j = 0; j < NN; ++j) rc = fma(ra[j], Qc.g[j], rc);
      const double cs = qsum<NN>(g_i * sd);
      if (valid) {
        bb[eoff(RB::Rc + i)] = twopi * rc;
        if (i == 0) bb[eoff(RB::Cs)] = fma(twopi, cs, f0mu0 * eb);
      }
    }
    // W1 = I - R A ; v1 = R Sd + S+
    double w[NN];
#pragma unroll
    for (int j = 0; j < NN; ++j) w[j] = i == j ? 1.0 : 0.0;
    double v = spl;
    qfor<0, NN>([&](auto K) {
      constexpr int k = HD_Q(K);
#pragma unroll
      for (int j = 0; j < NN; ++j) w[j] = fma(-r[k], qbc<NN, k>(ra[j]), w[j]);
      v = fma(r[k], qbc<NN, k>(sd), v);
    });
    // Gauss-Jordan on [W1 | T~ | v1] (the one-lane sweep's LU pivots), rows
    // normalised at the end: lane i ends with d_i [e_i | ZT_i | t1_i]
    double z[NN], d = 1.0;
#pragma unroll
    for (int j = 0; j < NN; ++j) z[j] = tr[j];
    qfor<0, NN>([&](auto K) {
      constexpr int k = HD_Q(K);
      const double pk = qbc<NN, k>(w[k]);
      st |= fabs(pk) > 1.0e-12 ? 0 : kStPivot;
      d = i == k ? pk : d;
      const double f = i == k ? 0.0 : w[k] * rcp_nr(pk);
      qfor<k + 1, NN>([&](auto J) { w[HD_Q(J)] = fma(-f, qbc<NN, k>(w[HD_Q(J)]), w[HD_Q(J)]); });
#pragma unroll
      for (int j = 0; j < NN; ++j) z[j] = fma(-f, qbc<NN, k>(z[j]), z[j]);
      v = fma(-f, qbc<NN, k>(v), v);
    });
    {
      const double rd = rcp_nr(d);
#pragma unroll
      for (int j = 0; j < NN; ++j) z[j] *= rd;  // row i of ZT
      v *= rd;                                  // t1_i
    }
    if (valid) {
#pragma unroll
      for (int j = 0; j < NN; ++j) bb[eoff(RB::Z + j * NN + i)] = z[j];
      bb[eoff(RB::Tv + i)] = v;
    }
    // u = A t1 + Sd ; P = A ZT ; Ra <- R + T P ; Sd <- T u + S-
    double u = sd, p_[NN];
#pragma unroll
    for (int j = 0; j < NN; ++j) p_[j] = 0.0;
    qfor<0, NN>([&](auto K) {
      constexpr int k = HD_Q(K);
      u = fma(ra[k], qbc<NN, k>(v), u);
#pragma unroll
      for (int j = 0; j < NN; ++j) p_[j] = fma(ra[k], qbc<NN, k>(z[j]), p_[j]);
    });
    double sdn = sml;
#pragma unroll
    for (int j = 0; j < NN; ++j) ra[j] = r[j];
    qfor<0, NN>([&](auto K) {
      constexpr int k = HD_Q(K);
#pragma unroll
      for (int j = 0; j < NN; ++j) ra[j] = fma(tr[k], qbc<NN, k>(p_[j]), ra[j]);
      sdn = fma(tr[k], qbc<NN, k>(u), sdn);
    });
    sd = sdn;
    tauc += taup;
  }

  // ---- Lambertian surface: I+ = g x ----
  double rgi = 0.0;
#pragma unroll
  for (int j = 0; j < NN; ++j) rgi = fma(ra[j], Qc.g[j], rgi);
  const double gsd = qsum<NN>(g_i * sd);
  const double grg = qsum<NN>(g_i * rgi);
  double esurf = (1.0 - alb) * bsurf;
  const double dirsurf = f0mu0 * exp(-tauc * rmu0);
  if (beam) esurf += alb * dirsurf / kPi;
  const double x = (2.0 * alb * gsd + esurf) / (1.0 - 2.0 * alb * grg);
  const double up = qsum<NN>(g_i * (g_i * x));
  const double dn = qsum<NN>(g_i * fma(rgi, x, sd));
  const double f0 = twopi * up, f1 = twopi * dn + dirsurf;
  if (valid && i == 0) {
    if (A.flux) {
      double* fo = A.flux + (size_t)s * (L + 1) * 2;
      fo[0] = f0;
      fo[1] = f1;
    }
    if (A.fsurf) {
      A.fsurf[sl] = f0;
      A.fsurf[nsc + sl] = f1;
    }
    A.xsurf[sl] = x;
  }
  if (!isfinite(f0 + f1)) st |= kStNonFinite;
  if (valid && st && i == 0) {
    atomicOr(&A.status[s], st);
    if (st & 0x0F) atomicOr(A.anyerr, 1);
  }
}

// ============================================================================
// K3: per-solve back-substitution bottom -> top.  Split from the adding sweep
// so that it runs at the occupancy of its own small register footprint (the
// sweep's register file allows one wave per SIMD): a pure stream over the
// back-substitution records, I+_top = t + ZT I+_bottom, fluxes per level.
// ============================================================================
// The arithmetic of both back-substitution kernels (identical expression order,
// so a solve's fluxes do not depend on which kernel ran its chunk).  PRE: the
// next layer's record is loaded into registers before this layer is computed.
template <int NN, bool PRE, bool NT>
__device__ __forceinline__ void backsub_body(const SweepArgs& A) {
  const Quad<NN>& Qc = quad<NN>();
  const long lane_sl = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = lane_sl < A.nsc;
  const bool band = A.part != nullptr;
  // with the band epilogue every lane of a wave takes part in the cross-lane
  // sums: lanes past the chunk run on the last solve's records with weight 0
  if (!live && !band) return;
  const long sl = live ? lane_sl : A.nsc - 1;
  const long s = solve_of(A.s0 + sl, A.cmaj, A.nwave, A.ncol);
  const int L = A.nlyr;
  const size_t nsc = A.nsc;
  const double twopi = 2.0 * kPi;
  const double x = A.xsurf[sl];
  double ip[NN];
#pragma unroll
  for (int i = 0; i < NN; ++i) ip[i] = Qc.g[i] * x;
  double* fo = A.flux ? A.flux + (size_t)s * (L + 1) * 2 : nullptr;
  double chk = 0.0;
  // band epilogue (cmaj order, q = col*nwave + w): lanes of one column form a
  // run; Hillis-Steele suffix sums inside the run leave the run's total (fixed
  // association order) in its first lane, which stores the wave's partial
  double wgt = 0.0;
  unsigned same = 0;  // bit k: lane + 2^k is in this lane's run
  bool head = false;
  double* pp = nullptr;
  if (band) {
    const long q = A.s0 + lane_sl;
    const long col = q / A.nwave;
    const int lane = (int)(lane_sl & 63);
    wgt = live ? A.wts[q - col * A.nwave] : 0.0;
    for (int k = 0; k < A.rsteps; ++k) {
      const int d = 1 << k;
      const long oc = __shfl_down(col, d);
      if (lane + d < 64 && oc == col) same |= 1u << k;
    }
    head = live && (lane == 0 || q % A.nwave == 0);
    const long wv = lane_sl >> 6;
    const long cfirst = (A.s0 + (wv << 6)) / A.nwave;
    pp = A.part + ((size_t)wv * A.nslot + (size_t)(col - cfirst)) * (L + 1) * 2;
  }
  auto emit = [&](int lev, double up, double dn, bool write_flux) {
    if (write_flux && fo && live) {
      fo[2 * lev] = up;
      fo[2 * lev + 1] = dn;
    }
    if (band) {
      double a = wgt * up, b = wgt * dn;
      for (int k = 0; k < A.rsteps; ++k) {
        const double a2 = __shfl_down(a, 1 << k);
        const double b2 = __shfl_down(b, 1 << k);
        if (same & (1u << k)) {
          a += a2;
          b += b2;
        }
      }
      if (head) {
        pp[2 * lev] = a;
        pp[2 * lev + 1] = b;
      }
    }
  };
  if (band) {  // surface level, from the sweep
    const double f0 = A.fsurf[sl], f1 = A.fsurf[nsc + sl];
    emit(0, f0, f1, false);
  }
  // this layer's record through `get` (RecB element indices: ZT column-major, t,
  // rc, cs)
  using RB = RecB<NN>;
  auto layer = [&](int lc, auto&& get) {
    double nip[NN];
#pragma unroll
    for (int i = 0; i < NN; ++i) {
      double t = get(RB::Tv + i);
#pragma unroll
      for (int j = 0; j < NN; ++j) t += get(RB::Z + j * NN + i) * ip[j];
      nip[i] = t;
    }
    double up = 0.0, dn = get(RB::Cs);
#pragma unroll
    for (int i = 0; i < NN; ++i) {
      ip[i] = nip[i];
      up += Qc.g[i] * nip[i];
      dn += get(RB::Rc + i) * nip[i];
    }
    const int lev = L - lc;
    emit(lev, twopi * up, dn, true);
    chk += twopi * up + dn;
  };
  auto rec_ptr = [&](int lc) {
    return reinterpret_cast<const double2*>(A.bsub) + (size_t)lc * RB::pairs * nsc + sl;
  };
  if constexpr (PRE) {
    constexpr int NP = RB::pairs;
    double2 cur[NP], nxt[NP];
    {
      const double2* bp = rec_ptr(L - 1);
#pragma unroll
      for (int e = 0; e < NP; ++e) cur[e] = rec_load<NT>(bp + e * nsc);
    }
    for (int lc = L - 1; lc >= 0; --lc) {
      if (lc > 0) {
        const double2* bp = rec_ptr(lc - 1);
#pragma unroll
        for (int e = 0; e < NP; ++e) nxt[e] = rec_load<NT>(bp + e * nsc);
      }
      layer(lc, [&](int e) { return (e & 1) ? cur[e >> 1].y : cur[e >> 1].x; });
#pragma unroll
      for (int e = 0; e < NP; ++e) cur[e] = nxt[e];
    }
  } else {
    for (int lc = L - 1; lc >= 0; --lc) {
      const double2* bp = rec_ptr(lc);
      layer(lc, [&](int e) { return pair_get<NT>(bp, nsc, e); });
    }
  }
  if (live && !isfinite(chk)) {
    atomicOr(&A.status[s], kStNonFinite);
    atomicOr(A.anyerr, 1);
  }
}

// K3: per-solve back-substitution bottom -> top.  Split from the adding sweep
// so that it runs at the occupancy of its own small register footprint (the
// sweep's register file allows one wave per SIMD): a pure stream over the
// back-substitution records, I+_top = t + ZT I+_bottom, fluxes per level.
// This one runs on the side stream beside the next chunk's layer kernel, so it
// must stay small: at most 96 VGPRs (five waves per SIMD), which fit next to a
// layer-kernel wave as long as that one stays at <= 416 (410 now).  The 16-byte
// record loads want the registers of a whole pair set in flight (8 waves per SIMD,
// 64 VGPRs, spilled).
template <int NN, bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5)))
void hd_backsub_kernel(SweepArgs A) {
  backsub_body<NN, false, NT>(A);
}

// K3 for the last chunk of a call, which nothing overlaps: no occupancy cap,
// a whole layer record in flight at once and the next one loaded while this
// one is computed (the capped kernel issues the 81 loads of a layer in small
// register-limited batches, each waiting out a memory latency).
template <int NN, bool NT>
__global__ __launch_bounds__(64) void hd_backsub_tail_kernel(SweepArgs A) {
  backsub_body<NN, true, NT>(A);
}

// ============================================================================
// K4: fused band epilogue of one chunk (hd_solve_band), per (column, level,
// direction): bflux[c] = (first chunk of c ? 0 : bflux[c]) + the chunk's part,
// summed in wave-point order -- deterministic, no atomics
// ============================================================================
__global__ __launch_bounds__(64) void hd_band_reduce_kernel(BandArgs B) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int per = 2 * B.nlev;
  const long W = B.nwave;
  const long q0 = B.s0, q1 = B.s0 + B.nsc;
  if (B.part) {  // register path, column-major chunk: the waves' run partials
    const long c = q0 / W + tid / per;
    if (c > (q1 - 1) / W) return;
    const int e = (int)(tid % per);
    const long qa = c * W > q0 ? c * W : q0;
    const long qb = ((c + 1) * W < q1 ? (c + 1) * W : q1) - 1;
    double sum = 0.0;
    for (long wv = (qa - q0) >> 6; wv <= (qb - q0) >> 6; ++wv) {
      const long cf = (q0 + (wv << 6)) / W;
      sum += B.part[((size_t)wv * B.nslot + (size_t)(c - cf)) * per + e];
    }
    double* o = B.bflux + (size_t)c * per + e;
    *o = c * W >= q0 ? sum : *o + sum;
  } else {  // team path: the chunk's fluxes, solves s = w*ncol + c in [s0, s1)
    const long c = tid / per;
    if (c >= B.ncol) return;
    const int e = (int)(tid % per);
    const long wa = q0 <= c ? 0 : (q0 - c + B.ncol - 1) / B.ncol;
    if (q1 - 1 < c) return;
    long wb = (q1 - 1 - c) / B.ncol;
    if (wb > W - 1) wb = W - 1;
    if (wa > wb) return;
    double sum = 0.0;
    for (long w = wa; w <= wb; ++w)
      sum += B.wts[w] * B.fchunk[(size_t)(w * B.ncol + c - q0) * per + e];
    double* o = B.bflux + (size_t)c * per + e;
    *o = wa == 0 ? sum : *o + sum;
  }
}

hipError_t launch_band_reduce(const BandArgs& ba, hipStream_t stream) {
  long n;
  if (ba.part) {
    n = ((ba.s0 + ba.nsc - 1) / ba.nwave - ba.s0 / ba.nwave + 1) * 2L * ba.nlev;
  } else {
    n = (long)ba.ncol * 2 * ba.nlev;
  }
  // one-wave blocks: on the side stream beside a team layer kernel (two 239-VGPR waves
  // per SIMD) a 4-wave block waited up to 9 ms for a CU with four free wave slots
  hipLaunchKernelGGL(hd_band_reduce_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0,
                     stream, ba);
  return hipGetLastError();
}

// ============================================================================
// host side: constant tables + launchers
// ============================================================================
template <int NN>
static void fill_quad(Quad<NN>& q, const QuadHost& h) {
  for (int i = 0; i < NN; ++i) {
    q.mu[i] = h.mu[i];
    q.w[i] = h.w[i];
    q.sd[i] = h.sd[i];
    q.g[i] = h.g[i];
    q.rmu[i] = 1.0 / h.mu[i];
    q.rg[i] = 1.0 / h.g[i];
    for (int l = 0; l < 2 * NN; ++l) q.pt[l][i] = h.pt[l][i];
  }
}

// ---- warm-start eigenvectors of the team Jacobi (hd_kernels.hpp) ----
namespace {
typedef long double ld_t;
// cyclic two-sided Jacobi of the symmetric n x n a; v <- its eigenvectors (columns)
void host_sym_eig(int n, ld_t (*a)[kMaxNN], ld_t (*v)[kMaxNN]) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) v[i][j] = i == j ? 1.0L : 0.0L;
  for (int sweep = 0; sweep < 64; ++sweep) {
    ld_t off = 0.0L, dia = 0.0L;
    for (int i = 0; i < n; ++i) {
      dia += a[i][i] * a[i][i];
      for (int j = i + 1; j < n; ++j) off += a[i][j] * a[i][j];
    }
    if (!(off > 1.0e-40L * dia)) break;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) {
        const ld_t apq = a[p][q];
        if (apq == 0.0L) continue;
        const ld_t th = (a[q][q] - a[p][p]) / (2.0L * apq);
        const ld_t t = (th >= 0.0L ? 1.0L : -1.0L) / (fabsl(th) + sqrtl(th * th + 1.0L));
        const ld_t c = 1.0L / sqrtl(t * t + 1.0L), s = t * c;
        for (int k = 0; k < n; ++k) {  // columns p, q of a and v
          const ld_t kp = a[k][p], kq = a[k][q];
          a[k][p] = c * kp - s * kq;
          a[k][q] = s * kp + c * kq;
          const ld_t vp = v[k][p], vq = v[k][q];
          v[k][p] = c * vp - s * vq;
          v[k][q] = s * vp + c * vq;
        }
        for (int k = 0; k < n; ++k) {  // rows p, q of a
          const ld_t pk = a[p][k], qk = a[q][k];
          a[p][k] = c * pk - s * qk;
          a[q][k] = s * pk + c * qk;
        }
      }
  }
}
// lower Cholesky factor in place (the upper triangle is zeroed)
void host_chol(int n, ld_t (*a)[kMaxNN]) {
  for (int j = 0; j < n; ++j) {
    ld_t d = a[j][j];
    for (int k = 0; k < j; ++k) d -= a[j][k] * a[j][k];
    const ld_t r = sqrtl(d > 0.0L ? d : 1.0e-300L);
    a[j][j] = r;
    for (int i = j + 1; i < n; ++i) {
      ld_t x = a[i][j];
      for (int k = 0; k < j; ++k) x -= a[i][k] * a[j][k];
      a[i][j] = x / r;
      a[j][i] = 0.0L;
    }
  }
}
}  // namespace

void warm_eigvecs(int nn, const QuadHost& q, int ia, int ib, double* vout) {
  // the layer kernel's S+ = -A+ and S- = -A- for an HG layer at the bin centre
  const int N = 2 * nn;
  const ld_t ssa = (ia + 0.5L) / kWarmG, g = (ib + 0.5L) / kWarmG;
  const ld_t f = powl(g, (ld_t)N);
  const ld_t om = ssa * (1.0L - f) / (1.0L - ssa * f), rf = om / (1.0L - f);
  ld_t sp[kMaxNN][kMaxNN] = {}, sm[kMaxNN][kMaxNN] = {};
  for (int l = 0; l < N; ++l) {
    const ld_t gl = (2 * l + 1) * ((l == 0 ? 1.0L : powl(g, (ld_t)l)) - f) * rf;
    for (int i = 0; i < nn; ++i)
      for (int k = 0; k < nn; ++k) {
        const ld_t x = gl * (ld_t)q.pt[l][i] * (ld_t)q.pt[l][k];
        if (l % 2 == 0) sp[i][k] += x;
        else sm[i][k] += x;
      }
  }
  for (int i = 0; i < nn; ++i)
    for (int k = 0; k < nn; ++k) {
      const ld_t sij = (ld_t)q.sd[i] * (ld_t)q.sd[k];
      const ld_t dg = i == k ? 1.0L / (ld_t)q.mu[i] : 0.0L;
      sp[i][k] = dg - sij * sp[i][k];
      sm[i][k] = dg - sij * sm[i][k];
    }
  host_chol(nn, sm);  // L
  host_chol(nn, sp);  // C
  ld_t b0[kMaxNN][kMaxNN], sym[kMaxNN][kMaxNN], v[kMaxNN][kMaxNN];
  for (int i = 0; i < nn; ++i)
    for (int k = 0; k < nn; ++k) {
      ld_t t = 0.0L;
      for (int m = 0; m < nn; ++m) t += sp[m][i] * sm[m][k];  // (C^T L)_ik
      b0[i][k] = t;
    }
  for (int i = 0; i < nn; ++i)
    for (int k = 0; k < nn; ++k) {
      ld_t t = 0.0L;
      for (int m = 0; m < nn; ++m) t += b0[m][i] * b0[m][k];
      sym[i][k] = t;
    }
  host_sym_eig(nn, sym, v);
  for (int i = 0; i < nn; ++i)
    for (int j = 0; j < nn; ++j) vout[i * nn + j] = (double)v[i][j];
}

hipError_t upload_quad_tables(const QuadHost* per_nn /* [kMaxNN], index nn-1 */) {
  QuadTables t;
  fill_quad<1>(t.q1, per_nn[0]);
  fill_quad<2>(t.q2, per_nn[1]);
  fill_quad<3>(t.q3, per_nn[2]);
  fill_quad<4>(t.q4, per_nn[3]);
  fill_quad<5>(t.q5, per_nn[4]);
  fill_quad<6>(t.q6, per_nn[5]);
  fill_quad<7>(t.q7, per_nn[6]);
  fill_quad<8>(t.q8, per_nn[7]);
  return hipMemcpyToSymbol(HIP_SYMBOL(c_quad), &t, sizeof(t), 0, hipMemcpyHostToDevice);
}

void launch_prologue(const PlanckArgs* pa, const TaucArgs* ta, hipStream_t stream) {
  if (ta) {
    hipLaunchKernelGGL(hd_tauc_kernel, dim3((unsigned)((ta->nsc + 255) / 256)), dim3(256), 0,
                       stream, *ta);
  }
  if (pa) {
    const long n0 = (long)pa->nsc * (pa->nlyr + 3);
    hipLaunchKernelGGL(hd_planck_kernel, dim3((unsigned)((n0 + 255) / 256)), dim3(256), 0,
                       stream, *pa);
  }
}

template <int NN>
static void launch_sweep(const SweepArgs& sa, hipStream_t stream) {
  if constexpr (NN == 2 || NN == 4) {
    if (sa.quad > 0 || (sa.quad < 0 && sa.nsc <= kQuadMaxSolves)) {  // NN-lane teams
      hipLaunchKernelGGL(hd_sweep_quad_kernel<NN>, dim3((unsigned)((sa.nsc * NN + 63) / 64)),
                         dim3(64), 0, stream, sa);
      return;
    }
  }
#if HD_AB_VARIANTS
  if constexpr (NN == 8) {
    if (sa.lean8) {
      hipLaunchKernelGGL(hd_sweep_lean_kernel<NN>, dim3((unsigned)((sa.nsc + 63) / 64)), dim3(64),
                         0, stream, sa);
      return;
    }
  }
#endif
  if (sa.nsc >= kNtMinSolves)
    hipLaunchKernelGGL((hd_sweep_kernel<NN, true>), dim3((unsigned)((sa.nsc + 63) / 64)), dim3(64),
                       0, stream, sa);
  else
    hipLaunchKernelGGL((hd_sweep_kernel<NN, false>), dim3((unsigned)((sa.nsc + 63) / 64)), dim3(64),
                       0, stream, sa);
}

template <int NN>
static hipError_t launch_chunk(const PlanckArgs* pa, const TaucArgs* ta, const LayerArgs& la,
                               const SweepArgs& sa, hipStream_t stream, hipEvent_t* ev) {
  launch_prologue(pa, ta, stream);
  const unsigned nb1 = (unsigned)(((la.nsc + 63) / 64) *
                                  ((la.nlyr + kLayersPerBlock - 1) / kLayersPerBlock));
  if (ev) (void)hipEventRecord(ev[0], stream);
  if (la.nsc >= kNtMinSolves)
    hipLaunchKernelGGL((hd_layer_kernel<NN, true>), dim3(nb1), dim3(kLayerBlock), 0, stream, la);
  else
    hipLaunchKernelGGL((hd_layer_kernel<NN, false>), dim3(nb1), dim3(kLayerBlock), 0, stream, la);
  if (ev) (void)hipEventRecord(ev[1], stream);
  launch_sweep<NN>(sa, stream);
  if (ev) (void)hipEventRecord(ev[2], stream);
  return hipGetLastError();
}

template <int NN>
static void launch_backsub(const SweepArgs& sa, hipStream_t stream, bool tail) {
  const dim3 gt((unsigned)((sa.nsc + 63) / 64)), gc((unsigned)((sa.nsc + 255) / 256));
  const bool nt = sa.nsc >= kNtMinSolves;
  if (tail && nt) hipLaunchKernelGGL((hd_backsub_tail_kernel<NN, true>), gt, dim3(64), 0, stream, sa);
  else if (tail) hipLaunchKernelGGL((hd_backsub_tail_kernel<NN, false>), gt, dim3(64), 0, stream, sa);
  else if (nt) hipLaunchKernelGGL((hd_backsub_kernel<NN, true>), gc, dim3(256), 0, stream, sa);
  else hipLaunchKernelGGL((hd_backsub_kernel<NN, false>), gc, dim3(256), 0, stream, sa);
}

hipError_t launch_backsub_nn(int nn, const SweepArgs& sa, hipStream_t stream, bool tail) {
  switch (nn) {
    case 1: launch_backsub<1>(sa, stream, tail); break;
    case 2: launch_backsub<2>(sa, stream, tail); break;
    case 3: launch_backsub<3>(sa, stream, tail); break;
    case 4: launch_backsub<4>(sa, stream, tail); break;
    case 5: launch_backsub<5>(sa, stream, tail); break;
    case 6: launch_backsub<6>(sa, stream, tail); break;
    case 7: launch_backsub<7>(sa, stream, tail); break;
    case 8: launch_backsub<8>(sa, stream, tail); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_solve_chunk_nn(int nn, const PlanckArgs* pa, const TaucArgs* ta,
                                 const LayerArgs& la, const SweepArgs& sa, hipStream_t stream,
                                 hipEvent_t* ev) {
  switch (nn) {
    case 1: return launch_chunk<1>(pa, ta, la, sa, stream, ev);
    case 2: return launch_chunk<2>(pa, ta, la, sa, stream, ev);
    case 3: return launch_chunk<3>(pa, ta, la, sa, stream, ev);
    case 4: return launch_chunk<4>(pa, ta, la, sa, stream, ev);
    case 5: return launch_chunk<5>(pa, ta, la, sa, stream, ev);
    case 6: return launch_chunk<6>(pa, ta, la, sa, stream, ev);
    case 7: return launch_chunk<7>(pa, ta, la, sa, stream, ev);
    case 8: return launch_chunk<8>(pa, ta, la, sa, stream, ev);
    default: return hipErrorInvalidValue;
  }
}

template <int NN>
static void launch_layer(const LayerArgs& la, hipStream_t stream) {
  const unsigned nb1 = (unsigned)(((la.nsc + 63) / 64) *
                                  ((la.nlyr + kLayersPerBlock - 1) / kLayersPerBlock));
  if (la.nsc >= kNtMinSolves)
    hipLaunchKernelGGL((hd_layer_kernel<NN, true>), dim3(nb1), dim3(kLayerBlock), 0, stream, la);
  else
    hipLaunchKernelGGL((hd_layer_kernel<NN, false>), dim3(nb1), dim3(kLayerBlock), 0, stream, la);
}

hipError_t launch_layer_nn(int nn, const LayerArgs& la, hipStream_t stream) {
  switch (nn) {
    case 1: launch_layer<1>(la, stream); break;
    case 2: launch_layer<2>(la, stream); break;
    case 3: launch_layer<3>(la, stream); break;
    case 4: launch_layer<4>(la, stream); break;
    case 5: launch_layer<5>(la, stream); break;
    case 6: launch_layer<6>(la, stream); break;
    case 7: launch_layer<7>(la, stream); break;
    case 8: launch_layer<8>(la, stream); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
hipError_t launch_column_nn(int nn, const LayerArgs& la, const SweepArgs& sa, hipStream_t stream) {
#if HD_AB_VARIANTS
  const dim3 grid((unsigned)((sa.nsc + 63) / 64)), block(64);
  switch (nn) {
    case 8: hipLaunchKernelGGL(hd_column_kernel<8>, grid, block, 0, stream, la, sa); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
#else
  (void)nn, (void)la, (void)sa, (void)stream;
  return hipErrorInvalidValue;  // A/B build only
#endif
}

hipError_t launch_sweep_nn(int nn, const SweepArgs& sa, hipStream_t stream) {
  switch (nn) {
    case 1: launch_sweep<1>(sa, stream); break;
    case 2: launch_sweep<2>(sa, stream); break;
    case 3: launch_sweep<3>(sa, stream); break;
    case 4: launch_sweep<4>(sa, stream); break;
    case 5: launch_sweep<5>(sa, stream); break;
    case 6: launch_sweep<6>(sa, stream); break;
    case 7: launch_sweep<7>(sa, stream); break;
    case 8: launch_sweep<8>(sa, stream); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// register path: records in 16-byte pairs (RecL / RecB), groups padded to even
static size_t reg_pairs_l(int nn) {
  const int nsym = nn * (nn + 1) / 2;
  return (size_t)(2 * even_up(nsym) + 2 * even_up(nn) + 2) / 2;
}
static size_t reg_pairs_b(int nn) {
  return (size_t)(even_up(nn * nn) + 2 * even_up(nn) + 2) / 2;
}

size_t layer_record_doubles(int nn) {
  if (nn <= kMaxRegNN) return 2 * reg_pairs_l(nn);
  return (size_t)(2 * nn * nn + 2 * nn + 2);  // team layout: full R, T rows (+ pad to even)
}

size_t bsub_record_doubles(int nn) {
  if (nn <= kMaxRegNN) return 2 * reg_pairs_b(nn);
  return (size_t)((nn * nn + 2 * nn + 2) & ~1);
}

static_assert(RecL<8>::pairs == 45 && RecB<8>::pairs == 41, "C4 record pairs");

size_t scratch_doubles_per_solve(int nn, int nlyr, bool planck) {
  // every per-chunk region is double-buffered: chunk k+1's layer kernel (and its
  // tauc/planck prologue) runs beside chunk k's sweep on another stream, and on
  // the register path chunk k's back-substitution beside chunk k+1's layer
  // kernel on a third (see hd_solve)
  const size_t nb = 2;
  return nb * (layer_record_doubles(nn) * nlyr + bsub_record_doubles(nn) * nlyr + 1 +
               (planck ? (size_t)nlyr + 3 : 0) + (size_t)nlyr);
}

}  // namespace hd
