// hd_team_mfma.hip -- per-(solve, layer) setup for nstr 18..32 with the dense
// 16 x 16 products on FP64 MFMA (v_mfma_f64_16x16x4_f64).
//
//   hd_team_mfma_layer_kernel<NN>  one wave = four (solve, layer) problems, the
//                                  same per-layer setup as hd_team_layer_kernel
//                                  (delta-M, phase matrix, Cholesky + one-sided
//                                  Jacobi eigenproblem, beam/thermal particular
//                                  solutions, R~/T~/S~ in the flux-weighted
//                                  basis)  [c_setdis,
//                                  c_soleig, c_upbeam, c_upisot]
//
// The work splits by shape:
//   * sequential, one-problem-per-team algebra stays on the VALU in the team
//     layout (T: team t = lanes 16t..16t+15, lane i holds row i): phase-matrix
//     rows, the four Cholesky factorisations (S-, S+, I + Omega Omega^T,
//     I + Psi^T Psi), their triangular inverses, the Jacobi sweeps and the
//     vector recurrences of the particular solutions;
//   * every dense 16 x 16 product runs on the matrix core in the MFMA layout
//     (M: for problem t, lane 16h + c holds X_t[h + 4m][c] in register m), four
//     k-steps per product and problem:
//        B0^T = L^T C            (Jacobi input)
//        U    = C^-T B,  U^T = B^T C^-1
//        W    = L^-T L^-1        (= (-A-)^-1)
//        Psi  = Gamma^1/2 U^T W,  Omega^T = Delta^1/2 U^T
//        I + Omega Omega^T,  I + Psi^T Psi
//        A-   = K-^T K-,  A+ = K+^T K+   (K = J^-1, J J^T = I + ...)
//     MFMA needs no cross-lane broadcasts: the operand of k-step s of A.B is
//     register s of A^T and of B in the M layout, and the product comes out in
//     the M layout, so chains of products need no data movement.  T <-> M goes
//     through two LDS tile-sets per wave (row stride 17 doubles).
//
// Replaces the DPP-broadcast products of hd_team_layer_kernel, whose row
// broadcasts, 64-bit selects and register spills were 39% of its VALU
// instructions at one wave per SIMD (profiles/r02_c5_team_counters_v1.json).
#include <cmath>
#include <mutex>
#include <vector>

#include "hd_rad.hpp"
#include "hd_team_prims.hpp"

namespace hd {

namespace {

__constant__ QuadTablesTeam c_qt;

using namespace team;

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kS = 17;           // tile row stride (doubles): conflict-free row and column reads
constexpr int kTile = 16 * kS;   // one problem's 16 x 16 tile
constexpr int kSet = 4 * kTile;  // a wave's four problems

// ---- T <-> LDS <-> M ----------------------------------------------------------
// T row i of team t -> tile_t[i][0..NN)
template <int NN>
__device__ __forceinline__ void put_rows(double* ts, int t, int i, const double (&x)[NN]) {
  double* r = ts + t * kTile + i * kS;
  sfor<0, NN>([&](auto J) { r[HD_K(J)] = x[HD_K(J)]; });
}
template <int NN>
__device__ __forceinline__ void get_rows(const double* ts, int t, int i, double (&x)[NN]) {
  const double* r = ts + t * kTile + i * kS;
  sfor<0, NN>([&](auto J) { x[HD_K(J)] = r[HD_K(J)]; });
}
// column i of tile_t -> x (the row of the transposed matrix)
template <int NN>
__device__ __forceinline__ void get_cols(const double* ts, int t, int i, double (&x)[NN]) {
  const double* r = ts + t * kTile + i;
  sfor<0, NN>([&](auto J) { x[HD_K(J)] = r[HD_K(J) * kS]; });
}
// M layout of every problem: X[t][m] = tile_t[h + 4m][c]
__device__ __forceinline__ void put_m(double* ts, int h, int c, const double (&x)[4][4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int m = 0; m < 4; ++m) ts[t * kTile + (h + 4 * m) * kS + c] = x[t][m];
}
__device__ __forceinline__ void get_m(const double* ts, int h, int c, double (&x)[4][4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int m = 0; m < 4; ++m) x[t][m] = ts[t * kTile + (h + 4 * m) * kS + c];
}
// M layout of the transposed tiles: X[t][m] = tile_t[c][h + 4m]
__device__ __forceinline__ void get_mt(const double* ts, int h, int c, double (&x)[4][4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int m = 0; m < 4; ++m) x[t][m] = ts[t * kTile + c * kS + h + 4 * m];
}
// LDS reads of one wave complete in order after its writes; this keeps the
// compiler from moving LDS accesses -- or anything else: the scheduler would
// hoist the next phase's loads and their registers -- across phase boundaries
__device__ __forceinline__ void lds_fence() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// D_t = A_t B_t (+ I) for the wave's four problems; at = A^T and b = B in M
template <bool ADD_I>
__device__ __forceinline__ void mprod(const double (&at)[4][4], const double (&b)[4][4],
                                      double (&d)[4][4], int h, int c) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    d4 acc;
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[m] = (ADD_I && h + 4 * m == c) ? 1.0 : 0.0;
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(at[t][s], b[t][s], acc, 0, 0, 0);
#pragma unroll
    for (int m = 0; m < 4; ++m) d[t][m] = acc[m];
  }
}

// Redefines x for the compiler (no instruction): broadcasts of x issued after a
// pin cannot be hoisted above it.  Without the pins the scheduler computes every
// row broadcast of a triangular loop up front -- NN(NN-1)/2 live doubles -- and
// the kernel spills.
template <int NN>
__device__ __forceinline__ void pin(double (&x)[NN]) {
#pragma unroll
  for (int k = 0; k < NN; ++k) asm volatile("" : "+v"(x[k]));
}
__device__ __forceinline__ void pin(double& x) { asm volatile("" : "+v"(x)); }

// XCD-aware block numbering (hardware deals blocks round-robin over the 8 XCDs):
// the blocks of one XCD take consecutive logical ids, ordered layer-fastest
__device__ __forceinline__ int block_logical() {
  const int nb = (int)gridDim.x, b = (int)blockIdx.x;
  const int x = b & 7, base = nb >> 3, extra = nb & 7;
  return x * base + (x < extra ? x : extra) + (b >> 3);
}
__device__ __forceinline__ int block_group(int L) { return block_logical() / L; }
__device__ __forceinline__ int block_layer(int L) { return block_logical() % L; }


// Y_l^m(mu_i) tables of nstr 18..32 for the intensity path's team kernels (mode
// m, degree l < nstr, node i) and the Y_l^m recurrence coefficients; filled
// from the same host recurrence as hd_rad.hip's tables (upload_rad_tables_team)
template <int NN>
struct RadTabTeam {
  double lam[2 * NN][2 * NN][NN];
};
struct RadTabsTeam {
  RadTabTeam<9> t9;
  RadTabTeam<10> t10;
  RadTabTeam<11> t11;
  RadTabTeam<12> t12;
  RadTabTeam<13> t13;
  RadTabTeam<14> t14;
  RadTabTeam<15> t15;
  RadTabTeam<16> t16;
  double seed[2 * kMaxNN];               // prod_{a<=m} sqrt((2a-1)/(2a))
  double ra[2 * kMaxNN][2 * kMaxNN];     // (2l-1)/sqrt(l^2-m^2), l > m
  double rb[2 * kMaxNN][2 * kMaxNN];     // sqrt((l-1)^2-m^2)/sqrt(l^2-m^2), l > m
};
__constant__ RadTabsTeam c_rtt;

template <int NN>
__device__ __forceinline__ const double* rad_lam(int m) {
  if constexpr (NN == 9) return &c_rtt.t9.lam[m][0][0];
  else if constexpr (NN == 10) return &c_rtt.t10.lam[m][0][0];
  else if constexpr (NN == 11) return &c_rtt.t11.lam[m][0][0];
  else if constexpr (NN == 12) return &c_rtt.t12.lam[m][0][0];
  else if constexpr (NN == 13) return &c_rtt.t13.lam[m][0][0];
  else if constexpr (NN == 14) return &c_rtt.t14.lam[m][0][0];
  else if constexpr (NN == 15) return &c_rtt.t15.lam[m][0][0];
  else return &c_rtt.t16.lam[m][0][0];
}

// warm-start tables of the team Jacobi (hd_kernels.hpp), every nn 9..16: entry e
// of nn holds V0 in the M layout, lane (h, c)'s four values V0[h + 4m][c] at
// (4c + h) * 4 + m (zero beyond nn)
constexpr int kWarmTeam = 256;
__device__ double d_warm_team[kMaxNN - kMaxRegNN][kWarmEntries * kWarmTeam];
template <int NN>
__device__ __forceinline__ const double* warm_tab_team() {
  return d_warm_team[NN - kMaxRegNN - 1];
}

// lane i of each team: column i of the inverse of the lower-triangular J whose
// rows the team holds (forward substitution J z = e_i), i.e. row i of J^-T
template <int NN>
__device__ __forceinline__ void team_tri_inverse_col(double (&jr)[NN], double& jrd,
                                                     double (&z)[NN]) {
  const int i = tlane();
  sfor<0, NN>([&](auto R) {
    constexpr int r = HD_K(R);
    double t = (double)(i == r);  // one conversion instead of two 32-bit selects
    sfor<0, r>([&](auto K) { t = fma(-bc<r>(jr[HD_K(K)]), z[HD_K(K)], t); });
    z[r] = t * bc<r>(jrd);
    pin<NN>(jr);
    pin(jrd);
  });
}

// lane i of each team: (X x)_i for X's row i (xr) and x distributed over the team
template <int NN>
__device__ __forceinline__ double team_matvec(const double (&xr)[NN], double x) {
  // x's broadcasts stay here: hoisted to where x is computed they outlive the
  // phases in between, and the compiler spills all NN of them to scratch
  pin(x);
  double y = 0.0;
  sfor<0, NN>([&](auto K) { y = fma(xr[HD_K(K)], bc<HD_K(K)>(x), y); });
  return y;
}

}  // namespace

// ============================================================================
// K1 (team, MFMA): per-(solve, layer) setup, four problems per wave
// ============================================================================
template <int NN, bool NT>
__global__ __launch_bounds__(64, 2) void hd_team_mfma_layer_kernel(LayerArgs A) {
  __shared__ double lds[2 * kSet + 4 * 2 * 16];
  double* S0 = lds;
  double* S1 = lds + kSet;
  double* G = lds + 2 * kSet;  // [t][dsq | gsq][16]
  constexpr int N = 2 * NN;
  const Quad<NN>& Qc = tquad<NN>(c_qt);
  const int lane = (int)threadIdx.x;
  const int h = lane >> 4, c = lane & 15;  // M layout
  const int t = h, i = c;                  // T layout: team t, row i
  const bool act = i < NN;
  const int ii = act ? i : 0;
  const int L = A.nlyr;
  // block = 4 consecutive solves (one per team) of one layer: their records are
  // contiguous.  Blocks are numbered layer-fastest within a group of solves and
  // dealt to one XCD (blocks b and b + 8 share an L2), so the neighbouring
  // layers of a solve -- which share prop's cache lines -- are read close together
  const int grp = block_group(L);  // first solve of this block / 4
  const int lc = block_layer(L);
  // every lane takes part in the MFMA and LDS exchanges: a team past the end
  // recomputes the block's first solve and stores nothing
  const bool valid = grp * 4 + t < A.nsc;
  const int sl = valid ? grp * 4 + t : grp * 4;
  const long s = A.s0 + sl;
  const int nm = A.nmom;
  const int np = A.nprop;
  int st = 0;

  // padding columns (>= NN) of both tile-sets are zero for the whole kernel
  // except where a product's identity padding lands (block diagonal: harmless)
  for (int k = lane; k < 2 * kSet; k += 64) lds[k] = 0.0;
  lds_fence();

  const double msk = act ? 1.0 : 0.0;
  const double mu_i = fma(msk, Qc.mu[ii] - 1.0, 1.0);
  const double sd_i = Qc.sd[ii] * msk;
  const double g_i = Qc.g[ii] * msk;
  const double rmu_i = Qc.rmu[ii] * msk;
  const double rg_i = Qc.rg[ii] * msk;

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

  // ---- phase-matrix rows: S+ = -A+ (ap), S- = -A- (lch); beam source sums ----
  // chi_1 .. chi_{N-1} of the team's record staged in LDS (the G area, free until the
  // eigenvalues): lane i of team t loads chi_{i+1} and chi_{i+17}, one round trip for the
  // whole record instead of one per iteration of the loop below
  {
    double* gm = G + t * 32;
    const int l1 = i + 1, l2 = i + 1 + 16;
    gm[i] = (l1 < N && l1 <= nm) ? q[1 + l1] : 0.0;
    gm[16 + i] = (l2 < N && l2 <= nm) ? q[1 + l2] : 0.0;
    lds_fence();
  }
  double ap[NN], lch[NN];
  double xs = 0.0, xd = 0.0;
  sfor<0, NN>([&](auto J) { ap[HD_K(J)] = lch[HD_K(J)] = 0.0; });
  {
    double pprev = 0.0, pcur = 1.0;
    const double* gm = G + t * 32 - 1;  // gm[l] = chi_l
#pragma nounroll
    for (int l2 = 0; l2 < NN; ++l2) {
      const int le = 2 * l2, lo = le + 1;
      const double che = le == 0 ? 1.0 : gm[le];
      const double cho = gm[lo];
      const double ge = (2 * le + 1) * (che - f) * rf;
      const double go = (2 * lo + 1) * (cho - f) * rf;
      const double pe0 = pcur;
      const double po0 = ((2 * lo - 1) * mub * pcur - (lo - 1) * pprev) / lo;
      pprev = po0;
      pcur = ((2 * lo + 1) * mub * po0 - lo * pe0) / (lo + 1);
      const double ue = ge * Qc.pt[le][ii] * msk;
      const double uo = go * Qc.pt[lo][ii] * msk;
      xs = fma(ue, pe0, xs);
      xd = fma(uo, po0, xd);
      sfor<0, NN>([&](auto J) {
        constexpr int j = HD_K(J);
        ap[j] = fma(ue, Qc.pt[le][j], ap[j]);
        lch[j] = fma(uo, Qc.pt[lo][j], lch[j]);
      });
    }
  }
  sfor<0, NN>([&](auto J) {
    constexpr int j = HD_K(J);
    const double diag = i == j ? rmu_i : 0.0;
    const double sij = sd_i * Qc.sd[j];
    lch[j] = fma(-sij, lch[j], diag);
    ap[j] = fma(-sij, ap[j], diag);
  });
  // L L^T = S-
  double lt[NN], rdl;
  if (!team_chol<NN, true>(lch, lt, rdl)) st |= kStEigen;

  // ---- pre-Jacobi vectors (depend on L only) ----
  double w2 = 0.0, lxd = 0.0;  // w2 = L^-T L^-1 g rv: V^T (L^-1 g rv) = U^T w2 later
  const double fb2 = fb * (0.5 / kPi);
  if (beam) {
    const double y = sd_i * (fb2 * xs);
    double z = 0.0;  // z = L^T y
    sfor<0, NN>([&](auto K) { z = fma(lt[HD_K(K)], bc<HD_K(K)>(y), z); });
    const double yl = team_matvec<NN>(lch, z);  // L z
    const double xdi = -fb2 * xd;
    const double rv = fma(-yl, rg_i, xdi * rmu0 * rmu_i);
    w2 = g_i * rv;
    lxd = sd_i * xdi;
    team_lsolve<NN>(lch, rdl, w2);
    team_usolve<NN>(lt, rdl, w2);
    team_lsolve<NN>(lch, rdl, lxd);
    team_usolve<NN>(lt, rdl, lxd);
  }
  double cvec = 0.0, db = 0.0, bsum = 0.0;
  if (A.planck) {
    const double bt = A.planckv[(size_t)(L - lc) * A.nsc + sl];
    // a transparent layer carries its top level's Planck value through
    // (c_disort's xr1 = 0 when dtaucpr = 0: B(tau) = xr0 = B_top)
    const double bb = taup > 0.0 ? A.planckv[(size_t)(L - lc - 1) * A.nsc + sl] : bt;
    db = bb - bt;
    bsum = bt + bb;
    const double b1 = taup > 0.0 ? 2.0 * db / taup : 0.0;
    cvec = sd_i * mu_i;
    team_lsolve<NN>(lch, rdl, cvec);
    team_usolve<NN>(lt, rdl, cvec);
    cvec = fma(b1 * rg_i, cvec, db) * msk;
  }
  {
    double z[NN];
    team_tri_inverse_col<NN>(lch, rdl, z);  // row i of L^-T -> S0 (lch dies here)
    put_rows<NN>(S0, t, i, z);
  }

  // ---- C C^T = S+ ; B0 = C^T L (lane j: column j) ; C^-1 to LDS ----
  double bcol[NN];
  {
    double unused[NN], rdc;
    if (!team_chol<NN, false>(ap, unused, rdc)) st |= kStEigen;  // ap <- rows of C
    sfor<0, NN>([&](auto I) {
      constexpr int r = HD_K(I);
      double u = 0.0;
      sfor<r, NN>([&](auto K) { u = fma(bc<HD_K(K)>(ap[r]), lt[HD_K(K)], u); });
      bcol[r] = u;
      pin<NN>(ap);
    });
    // Warm start (hd_kernels.hpp): B0 <- B0 V0 on the matrix core, V0 the
    // tabulated eigenvectors of each team's (ssa, chi_1) bin (identity for a
    // non-scattering layer), read straight into the M layout; S1 is free until
    // C^-T is written to it below
    if (A.warm) {
      const double g1 = nm >= 1 ? q[2] : 0.0;
      const int e = ssa > 0.0 ? warm_bin(ssa) * kWarmG + warm_bin(g1) : kWarmG * kWarmG;
      int es[4];
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) es[tt] = __builtin_amdgcn_readlane(e, 16 * tt);
      if (es[0] != kWarmG * kWarmG || es[1] != kWarmG * kWarmG || es[2] != kWarmG * kWarmG ||
          es[3] != kWarmG * kWarmG) {
        double X[4][4], V[4][4];
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          const double2* p = reinterpret_cast<const double2*>(warm_tab_team<NN>() +
                                                              (size_t)es[tt] * kWarmTeam) +
                             (c * 4 + h) * 2;
          const double2 a = p[0], b = p[1];
          V[tt][0] = a.x;
          V[tt][1] = a.y;
          V[tt][2] = b.x;
          V[tt][3] = b.y;
        }
        lds_fence();
        put_rows<NN>(S1, t, i, bcol);  // tile = B0^T
        lds_fence();
        get_m(S1, h, c, X);           // B0^T (M): the A^T operand of B0 V0
        mprod<false>(X, V, X, h, c);  // B0 V0 (M)
        lds_fence();
        put_m(S1, h, c, X);
        lds_fence();
        get_cols<NN>(S1, t, i, bcol);  // lane j: column j of B0 V0
        lds_fence();
      }
    }
    double z[NN];
    team_tri_inverse_col<NN>(ap, rdc, z);  // row i of C^-T -> S1
    put_rows<NN>(S1, t, i, z);
  }

  // ---- eigenpairs (c_soleig): Sym = L^T S+ L = B0^T B0 = V diag(k^2) V^T ----
  lds_fence();
  if (!team_jacobi<NN>(bcol, A.max_sweeps)) st |= kStEigen;  // B = B0 V, lane j: column j
  lds_fence();
  double kk;
  {
    double k2 = 0.0;
    sfor<0, NN>([&](auto K) { k2 = fma(bcol[HD_K(K)], bcol[HD_K(K)], k2); });
    if (act && !(k2 > 0.0)) st |= kStEigen;
    kk = sqrt(k2 > 0.0 ? k2 : 0.0) * msk;
    // Delta = tanh(k tau'/2)/k, Gamma = k tanh(k tau'/2) (lane j)
    const double x = kk * taup;
    const double m = -expm1(-x);
    const double th = m * rcp_nr(2.0 - m);
    const double delta = x > 1.0e-8 ? th * rcp_nr(kk > 0.0 ? kk : 1.0) : 0.5 * taup;
    G[t * 32 + i] = sqrt(delta) * msk;
    G[t * 32 + 16 + i] = sqrt(kk * th) * msk;
  }

  // ---- the dense products on the matrix core; vectors of the beam solution ----
  // LDS holds what the next phase reads: S0 = L^-T rows, then W; S1 = C^-T rows,
  // then B^T rows, then U^T (whose rows and columns feed the two beam matvecs)
  double zp = 0.0, zm = 0.0, e0 = 0.0;
  {
    double X[4][4], Y[4][4], U[4][4], UT[4][4];
    get_mt(S0, h, c, X);          // L^-1 (M)
    mprod<false>(X, X, Y, h, c);  // W = L^-T L^-1
    get_mt(S1, h, c, X);          // C^-1 (M)
    lds_fence();
    put_m(S0, h, c, Y);            // W, row-major
    put_rows<NN>(S1, t, i, bcol);  // rows of B^T
    lds_fence();
    get_mt(S1, h, c, Y);           // B (M)
    mprod<false>(X, Y, U, h, c);   // U = C^-T B
    mprod<false>(Y, X, UT, h, c);  // U^T = B^T C^-1
    lds_fence();
    put_m(S1, h, c, UT);
    lds_fence();
    // beam (c_upbeam): tt = U^T w2 / (1/mu0^2 - k^2), sv = W^-1 D^1/2 U tt, then
    // yy = W (sd mu sv) -- rows of U^T, columns of U^T, rows of W from LDS
    if (beam) {
      double r_[NN];
      get_rows<NN>(S1, t, i, r_);
      const double r2 = rmu0 * rmu0;
      const double tv = team_matvec<NN>(r_, w2);
      double den = fma(-kk, kk, r2);
      if (act && fabs(den) < 1.0e-9 * r2) {
        st |= kStResonance;
        den = den < 0.0 ? -1.0e-9 * r2 : 1.0e-9 * r2;
      }
      const double ttv = tv / den * msk;
      get_cols<NN>(S1, t, i, r_);
      const double sv = team_matvec<NN>(r_, ttv) * rg_i;
      get_rows<NN>(S0, t, i, r_);
      const double yy = team_matvec<NN>(r_, sd_i * mu_i * sv);
      // tauc null: sources for a unit beam at the layer top (the sweep scales them)
      const double tauc = A.tauc ? A.tauc[(size_t)lc * A.nsc + sl] : 0.0;
      const double att = 0.5 * exp(-tauc * rmu0);
      const double dd = rg_i * fma(-yy, rmu0, lxd);
      zp = (sv + dd) * att;
      zm = (sv - dd) * att;
      e0 = exp(-taup * rmu0);
    }
    get_m(S0, h, c, Y);            // W (M)
    mprod<false>(U, Y, X, h, c);   // U^T W
    // row scalings: Psi = Gamma^1/2 U^T W, Omega^T = Delta^1/2 U^T
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        X[tt][m] *= G[tt * 32 + 16 + h + 4 * m];
        UT[tt][m] *= G[tt * 32 + h + 4 * m];
      }
    mprod<true>(UT, UT, U, h, c);  // I + Omega Omega^T
    mprod<true>(X, X, Y, h, c);    // I + Psi^T Psi
    lds_fence();
    put_m(S0, h, c, U);
    put_m(S1, h, c, Y);
    lds_fence();
  }
  const double ga = g_i * (cvec - fma(-zp, e0, zm));
  const double gb = g_i * (fma(zp, e0, zm) + bsum);

  // ---- A- = (I + Omega Omega^T)^-1, A+ = (I + Psi^T Psi)^-1 ----
  // J J^T = H (team Cholesky), K = J^-1 (team columns), A = K^T K (MFMA);
  // Q~- ga = ga - A- ga, Q~+ gb = A+ gb - gb from the rows of A-, A+
  double Am[4][4], Ap[4][4];
  double pv, qv;
  {
    double hr[NN], unused[NN], z[NN], jrd, X[4][4];
    get_rows<NN>(S0, t, i, hr);
    if (!team_chol<NN, false>(hr, unused, jrd)) st |= kStEigen;
    team_tri_inverse_col<NN>(hr, jrd, z);  // row i of K-^T
    lds_fence();
    put_rows<NN>(S0, t, i, z);
    lds_fence();
    get_mt(S0, h, c, X);
    mprod<false>(X, X, Am, h, c);
    lds_fence();
    put_m(S0, h, c, Am);
    lds_fence();
    get_rows<NN>(S0, t, i, hr);
    pv = ga - team_matvec<NN>(hr, ga);
    get_rows<NN>(S1, t, i, hr);
    if (!team_chol<NN, false>(hr, unused, jrd)) st |= kStEigen;
    team_tri_inverse_col<NN>(hr, jrd, z);  // row i of K+^T
    lds_fence();
    put_rows<NN>(S1, t, i, z);
    lds_fence();
    get_mt(S1, h, c, X);
    mprod<false>(X, X, Ap, h, c);
    lds_fence();
    put_m(S1, h, c, Ap);
    lds_fence();
    get_rows<NN>(S1, t, i, hr);
    qv = team_matvec<NN>(hr, gb) - gb;
  }

  // ---- store: R~ = A+ - A-, T~ = A- + A+ - I (M layout), S~+, S~-, tau' (T) ----
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) {
    double chk = 0.0;
    const bool ok = grp * 4 + tt < A.nsc;
    const int slt = ok ? grp * 4 + tt : grp * 4, lct = lc;
    double* rec = A.scr + ((size_t)lct * A.nsc + slt) * ne1t<NN>();
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int r = h + 4 * m;
      const double rr = Ap[tt][m] - Am[tt][m];
      const double tr = (Am[tt][m] + Ap[tt][m]) - (r == c ? 1.0 : 0.0);
      // whole 128-B rows per problem: nontemporal for a large chunk (hd_kernels.hpp);
      // the team reads stay plain (8-byte pieces: with nt C5 ran 20 % slower)
      if (ok && r < NN && c < NN) {
        rec_st<NT>(&rec[r * NN + c], rr);
        rec_st<NT>(&rec[NN * NN + r * NN + c], tr);
      }
      chk += rr + tr;
    }
    // this lane's share of problem tt's R~/T~: a non-finite entry flags problem tt
    if (ok && !isfinite(chk)) {
      atomicOr(&A.status[A.s0 + slt], kStNonFinite);
      atomicOr(A.anyerr, 1);
    }
  }
  double chk = 0.0;
  const double sp = g_i * (zp * (1.0 - e0) - db) + pv - qv;
  const double sm = g_i * (-zm * (1.0 - e0) + db) - pv - qv;
  double* rec = A.scr + ((size_t)lc * A.nsc + sl) * ne1t<NN>();
  if (valid && act) {
    rec[2 * NN * NN + ii] = sp;
    rec[2 * NN * NN + NN + ii] = sm;
  }
  chk += sp + sm;
  if (valid && i == 0) rec[2 * NN * NN + 2 * NN] = taup;
  if (act && !isfinite(chk + taup)) st |= kStNonFinite;
  if (valid && st) {
    atomicOr(&A.status[s], st);
    if (st & 0x0F) atomicOr(A.anyerr, 1);
  }
}

#if HD_AB_VARIANTS  // the one-wave team sweep: A/B build only (the product runs the lean one)
// ============================================================================
// K2 (team, MFMA): adding sweep + back-substitution, four solves per wave.
// The register/team sweep's update per layer
//   W1 = I - R A,  ZT = W1^-1 T,  A <- R + T A ZT,  Sd <- T (A t1 + Sd) + S-
// (A = reflection of the stack above, t1 = W1^-1 (R Sd + S+)) with the three
// dense 16 x 16 products (R A, A ZT, T (A ZT)) on the matrix core in the M
// layout -- R~, T~ and A are symmetric, so each is its own transpose operand --
// and the pivot-free LU of W1, the ZT solves and the vectors on the VALU in the
// team layout (lane i = row i), as hd_team_sweep_kernel; W1 goes M -> T and ZT
// T -> M through LDS, A is kept in both layouts.  Identical record formats, so
// the back-substitution pass is hd_team_sweep_kernel's.  One wave per SIMD: at
// two (256 registers) it spills 144 VGPRs and ran C5 at 0.81M solves/s against
// 1.02M here and 0.97M for the VALU sweep (scripts/ab/sw_ab.sh).
// ============================================================================
template <int NN>
__global__ __launch_bounds__(64, 1) void hd_team_mfma_sweep_kernel(SweepArgs A) {
  __shared__ double lds[2 * kSet];
  double* S0 = lds;
  double* S1 = lds + kSet;
  const Quad<NN>& Qc = tquad<NN>(c_qt);
  const int lane = (int)threadIdx.x;
  const int h = lane >> 4, c = lane & 15;  // M layout
  const int t = h, i = c;                  // T layout: team t, row i
  const bool act = i < NN;
  const int ii = act ? i : 0;
  const int grp = (int)blockIdx.x;
  // every lane takes part in the MFMA / LDS / DPP exchanges: a team past the end
  // repeats the block's first solve and stores nothing
  const bool valid = grp * 4 + t < A.nsc;
  const int sl = valid ? grp * 4 + t : grp * 4;
  const long s = solve_of(A.s0 + sl, A.cmaj, A.nwave, A.ncol);
  const int L = A.nlyr;
  const size_t nsc = A.nsc;
  int st = 0;
  const double msk = act ? 1.0 : 0.0;
  const double g_i = Qc.g[ii] * msk;

  for (int k = lane; k < 2 * kSet; k += 64) lds[k] = 0.0;
  lds_fence();

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

  // the wave's four solves in M layout: problem tt's records
  int slm[4];
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) slm[tt] = grp * 4 + tt < A.nsc ? grp * 4 + tt : grp * 4;

  double ram[4][4];  // A (M layout)
  double ra[NN];     // A row i (T layout)
  double sd = g_i * top;
#pragma unroll
  for (int tt = 0; tt < 4; ++tt)
#pragma unroll
    for (int m = 0; m < 4; ++m) ram[tt][m] = 0.0;
  sfor<0, NN>([&](auto J) { ra[HD_K(J)] = 0.0; });
  double tauc = 0.0;

  for (int lc = 0; lc < L; ++lc) {
    const double* rec = A.scr + ((size_t)lc * nsc + sl) * ne1t<NN>();
    double* bp = A.bsub + ((size_t)lc * nsc + sl) * ne2t<NN>();
    double* bw = (act && valid) ? bp : A.sink;
    // R~, T~ of the four problems in M layout (zero padding beyond NN)
    double rm[4][4], tm[4][4];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const double* rt = A.scr + ((size_t)lc * nsc + slm[tt]) * ne1t<NN>();
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int r = h + 4 * m;
        const bool in = r < NN && c < NN;
        const int e = in ? r * NN + c : 0;
        rm[tt][m] = in ? rt[e] : 0.0;
        tm[tt][m] = in ? rt[NN * NN + e] : 0.0;
      }
    }
    // this problem's rows in T layout
    double rl[NN], tr[NN];
    sfor<0, NN>([&](auto J) {
      rl[HD_K(J)] = rec[ii * NN + HD_K(J)] * msk;
      tr[HD_K(J)] = rec[NN * NN + ii * NN + HD_K(J)] * msk;
    });
    // direct beam at the layer top; a unit-beam record's sources scale with it
    const double eb = exp(-tauc * rmu0);
    const double sscale = A.beam_scale ? eb : 1.0;
    const double spl = rec[2 * NN * NN + ii] * msk * sscale;
    const double sml = rec[2 * NN * NN + NN + ii] * msk * sscale;

    // level lc (top of layer lc): F_dn = rc . I+ + cs
    {
      double tq = 0.0;
      sfor<0, NN>([&](auto J) { tq = fma(ra[HD_K(J)], Qc.g[HD_K(J)], tq); });
      bw[NN * NN + NN + ii] = twopi * tq;
      const double cs = team_sum(g_i * sd);
      if (i == 0 && valid) bp[NN * NN + 2 * NN] = fma(twopi, cs, f0mu0 * eb);
    }
    // W1 = I - R A on the matrix core, to team rows through LDS
    {
      double pw[4][4];
      mprod<false>(rm, ram, pw, h, c);
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int m = 0; m < 4; ++m) pw[tt][m] = (h + 4 * m == c ? 1.0 : 0.0) - pw[tt][m];
      lds_fence();
      put_m(S0, h, c, pw);
      lds_fence();
    }
    double w[NN];
    get_rows<NN>(S0, t, i, w);
    sfor<0, NN>([&](auto J) { w[HD_K(J)] *= msk; });
    // t1 = R Sd + S+
    double t1 = spl;
    sfor<0, NN>([&](auto K) { t1 = fma(rl[HD_K(K)], bc<HD_K(K)>(sd), t1); });
    // LU without pivoting; reciprocal pivots on the diagonal
    sfor<0, NN>([&](auto K) {
      constexpr int k = HD_K(K);
      const double piv = bc<k>(w[k]);
      if (!(fabs(piv) > 1.0e-12)) st |= kStPivot;
      const double rp = rcp_nr(piv);
      const double lik = w[k] * rp;
      const double mm = i > k ? lik : 0.0;
      w[k] = i == k ? rp : (i > k ? lik : w[k]);
      sfor<k + 1, NN>([&](auto J) {
        constexpr int j = HD_K(J);
        w[j] = fma(-mm, bc<k>(w[j]), w[j]);
      });
    });
    // t1 <- W1^-1 t1
    sfor<0, NN>([&](auto K) {
      constexpr int k = HD_K(K);
      const double tk = bc<k>(t1);
      if (i > k) t1 = fma(-w[k], tk, t1);
    });
    sfor_rev<0, NN>([&](auto K) {
      constexpr int k = HD_K(K);
      if (i == k) t1 *= w[k];
      const double tk = bc<k>(t1);
      if (i < k) t1 = fma(-w[k], tk, t1);
    });
    // u = A t1 + Sd
    double u = sd;
    sfor<0, NN>([&](auto K) { u = fma(ra[HD_K(K)], bc<HD_K(K)>(t1), u); });
    bw[NN * NN + ii] = t1;
    // ZT = W1^-1 T = U^-1 (L^-1 T) on the matrix core: the team forms the columns
    // of L^-1 (unit lower) and U^-1 from the LU rows -- lane i holds column i, i.e.
    // row i of the transposed inverse, the operand the M-layout product wants --
    // instead of sixteen row-sequential triangular solves with T's sixteen columns
    // (NN(NN-1) broadcasts per lane against 2 x NN(NN-1)/2 here)
    {
      double zl[NN], zu[NN];
      sfor<0, NN>([&](auto R) {  // column i of L^-1: z_r = delta_ri - sum_{k<r} L_rk z_k
        constexpr int r = HD_K(R);
        double v = i == r ? 1.0 : 0.0;
        sfor<0, r>([&](auto K) { v = fma(-bc<r>(w[HD_K(K)]), zl[HD_K(K)], v); });
        zl[r] = v;
        pin<NN>(w);
      });
      sfor_rev<0, NN>([&](auto R) {  // column i of U^-1: z_r = (delta_ri - sum_{k>r} U_rk z_k) / U_rr
        constexpr int r = HD_K(R);
        double v = i == r ? 1.0 : 0.0;
        sfor<r + 1, NN>([&](auto K) { v = fma(-bc<r>(w[HD_K(K)]), zu[HD_K(K)], v); });
        zu[r] = v * bc<r>(w[r]);  // reciprocal pivot on the diagonal
        pin<NN>(w);
      });
      sfor<0, NN>([&](auto J) {
        zl[HD_K(J)] *= msk;
        zu[HD_K(J)] *= msk;
      });
      lds_fence();
      put_rows<NN>(S0, t, i, zl);  // L^-T, row-major
      put_rows<NN>(S1, t, i, zu);  // U^-T, row-major
    }
    // Sd <- T u + S-
    {
      double tq = sml;
      sfor<0, NN>([&](auto K) { tq = fma(tr[HD_K(K)], bc<HD_K(K)>(u), tq); });
      sd = tq * msk;
    }
    lds_fence();
    // ZT = U^-1 (L^-1 T); record (M layout: rows h + 4m, column c); A <- R + T (A ZT);
    // then A's rows to the team layout
    {
      double li[4][4], x1[4][4], zm[4][4], pm[4][4];
      get_m(S0, h, c, li);
      mprod<false>(li, tm, x1, h, c);  // L^-1 T
      get_m(S1, h, c, li);
      mprod<false>(li, x1, zm, h, c);  // ZT = U^-1 (L^-1 T)
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        double* zr = A.bsub + ((size_t)lc * nsc + slm[tt]) * ne2t<NN>();
        const bool ok = grp * 4 + tt < A.nsc;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int r = h + 4 * m;
          if (ok && r < NN && c < NN) zr[r * NN + c] = zm[tt][m];
        }
      }
      mprod<false>(ram, zm, pm, h, c);  // A ZT   (A symmetric: its own transpose)
      mprod<false>(tm, pm, ram, h, c);  // T (A ZT)
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int m = 0; m < 4; ++m) ram[tt][m] += rm[tt][m];
      lds_fence();
      put_m(S0, h, c, ram);
      lds_fence();
    }
    get_rows<NN>(S0, t, i, ra);
    sfor<0, NN>([&](auto J) { ra[HD_K(J)] *= msk; });
    tauc += rec[2 * NN * NN + 2 * NN];
  }

  // ---- Lambertian surface: I+ = g x ----
  double rgrow = 0.0;
  sfor<0, NN>([&](auto J) { rgrow = fma(ra[HD_K(J)], Qc.g[HD_K(J)], rgrow); });
  const double gsd = bc<0>(team_sum(g_i * sd));
  const double grg = bc<0>(team_sum(g_i * rgrow));
  double esurf = (1.0 - alb) * bsurf;
  const double dirsurf = f0mu0 * exp(-tauc * rmu0);
  if (beam) esurf += alb * dirsurf / kPi;
  const double x = (2.0 * alb * gsd + esurf) / (1.0 - 2.0 * alb * grg);
  double ip = g_i * x;
  double* fo = A.flux + (size_t)(A.flux_local ? (long)sl : s) * (L + 1) * 2;
  double chk = 0.0;
  {
    const double up = team_sum(g_i * ip);
    const double dn = team_sum(g_i * fma(rgrow, x, sd));
    if (i == 0 && valid) {
      fo[0] = twopi * up;
      fo[1] = twopi * dn + dirsurf;
    }
    chk += twopi * up + twopi * dn;
  }
  // ---- back-substitution bottom -> top ----
  for (int lc = L - 1; lc >= 0; --lc) {
    const double* bp = A.bsub + ((size_t)lc * nsc + sl) * ne2t<NN>();
    double nip = bp[NN * NN + ii] * msk;
    sfor<0, NN>([&](auto J) {
      const double z = bp[ii * NN + HD_K(J)] * msk;
      nip = fma(z, bc<HD_K(J)>(ip), nip);
    });
    const double rc = bp[NN * NN + NN + ii] * msk;
    const double up = team_sum(g_i * nip);
    const double dn = team_sum(rc * nip);
    ip = nip;
    if (i == 0 && valid) {
      const int lev = L - lc;
      fo[2 * lev] = twopi * up;
      fo[2 * lev + 1] = bp[NN * NN + 2 * NN] + dn;
    }
    chk += twopi * up + dn;
  }
  if (!isfinite(chk)) st |= kStNonFinite;
  if (valid && st) {
    atomicOr(&A.status[s], st);
    if (st & 0x0F) atomicOr(A.anyerr, 1);
  }
}
#endif  // HD_AB_VARIANTS

// ============================================================================
// K2 (team, MFMA), lean: the same sweep and back-substitution as
// hd_team_mfma_sweep_kernel in at most 256 registers, so that two waves share a
// SIMD (and one can run beside a 240-register layer-kernel wave) instead of one.
// What changes is only where the operands live between their uses:
//   * A's team rows (for the level's rc, and u = A t1 + Sd) stay in LDS tile set
//     S0 from the end of one layer to the middle of the next, not in registers;
//     W1 = I - R A goes through tile set S1 instead;
//   * R~ and T~ are read from the layer record where they are needed -- R~ (M
//     layout) for W1 and again for A <- R~ + T~ (A ZT), R~'s team row for v1, T~'s
//     team row for Sd, T~ (M layout) for the ZT products -- instead of all at the
//     top of the layer (second reads of a record are L2 hits);
//   * per-element record offsets are recomputed where they are used (laundered
//     lane indices), not hoisted out of the layer loop.
// The arithmetic and its order are hd_team_mfma_sweep_kernel's, so the records
// and fluxes are bitwise the same (tests/test_gpu_parity.py: lean vs default).
// ============================================================================
template <int NN, bool NT>
__global__ __launch_bounds__(64, 2) void hd_team_mfma_sweep_lean_kernel(SweepArgs A) {
  __shared__ double lds[2 * kSet];
  double* S0 = lds;
  double* S1 = lds + kSet;
  const Quad<NN>& Qc = tquad<NN>(c_qt);
  const int lane = (int)threadIdx.x;
  const int h = lane >> 4, c = lane & 15;  // M layout
  const int t = h, i = c;                  // T layout: team t, row i
  const bool act = i < NN;
  const int ii = act ? i : 0;
  const int grp = (int)blockIdx.x;
  const bool valid = grp * 4 + t < A.nsc;
  const int sl = valid ? grp * 4 + t : grp * 4;
  const long s = solve_of(A.s0 + sl, A.cmaj, A.nwave, A.ncol);
  const int L = A.nlyr;
  const size_t nsc = A.nsc;
  int st = 0;
  const double msk = act ? 1.0 : 0.0;
  const double g_i = Qc.g[ii] * msk;

  for (int k = lane; k < 2 * kSet; k += 64) lds[k] = 0.0;  // A = 0 in S0
  lds_fence();

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
  const int g0 = grp * 4;  // the wave's first solve (uniform)

  // problem tt's record element (r, c) of the matrix at offset off, M layout
  auto load_m = [&](int lc, int off, double (&x)[4][4]) {
    __builtin_amdgcn_sched_barrier(0);  // issued here, not hoisted into an earlier phase
    int hl = h, cl = c;
    asm volatile("" : "+v"(hl), "+v"(cl));
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const int slt = g0 + tt < A.nsc ? g0 + tt : g0;
      const double* rt = A.scr + ((size_t)lc * nsc + slt) * ne1t<NN>() + off;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int r = hl + 4 * m;
        const bool in = r < NN && cl < NN;
        x[tt][m] = in ? rt[in ? r * NN + cl : 0] : 0.0;
      }
    }
  };
  // this problem's team row of the matrix at offset off
  auto load_row = [&](const double* rec, int off, double (&x)[NN]) {
    __builtin_amdgcn_sched_barrier(0);
    int il = ii;
    asm volatile("" : "+v"(il));
    sfor<0, NN>([&](auto J) { x[HD_K(J)] = rec[off + il * NN + HD_K(J)] * msk; });
  };

  double ram[4][4];  // A (M layout)
#pragma unroll
  for (int tt = 0; tt < 4; ++tt)
#pragma unroll
    for (int m = 0; m < 4; ++m) ram[tt][m] = 0.0;
  double sd = g_i * top;
  double tauc = 0.0;

  for (int lc = 0; lc < L; ++lc) {
    // the lane indices, laundered per layer: every lane-dependent constant below
    // (identity entries, triangle masks) is then formed where it is used instead
    // of all being hoisted out of the loop into live (and spilled) registers
    int i_ = i, h_ = h, c_ = c;
    asm volatile("" : "+v"(i_), "+v"(h_), "+v"(c_));
    const int i = i_, h = h_, c = c_;
    const double* rec = A.scr + ((size_t)lc * nsc + sl) * ne1t<NN>();
    double* bp = A.bsub + ((size_t)lc * nsc + sl) * ne2t<NN>();
    double* bw = (act && valid) ? bp : A.sink;
    // direct beam at the layer top; a unit-beam record's sources scale with it
    const double eb = exp(-tauc * rmu0);
    const double sscale = A.beam_scale ? eb : 1.0;
    const double spl = rec[2 * NN * NN + ii] * msk * sscale;

    // level lc (top of layer lc): F_dn = rc . I+ + cs; A's row i from S0
    {
      double ar[NN];
      get_rows<NN>(S0, t, i, ar);
      double tq = 0.0;
      sfor<0, NN>([&](auto J) { tq = fma(ar[HD_K(J)] * msk, Qc.g[HD_K(J)], tq); });
      bw[NN * NN + NN + ii] = twopi * tq;
      const double cs = team_sum(g_i * sd);
      if (i == 0 && valid) bp[NN * NN + 2 * NN] = fma(twopi, cs, f0mu0 * eb);
    }
    // W1 = I - R A on the matrix core, to team rows through S1
    double w[NN];
    {
      double rm[4][4], pw[4][4];
      load_m(lc, 0, rm);
      mprod<false>(rm, ram, pw, h, c);
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int m = 0; m < 4; ++m) pw[tt][m] = (h + 4 * m == c ? 1.0 : 0.0) - pw[tt][m];
      lds_fence();
      put_m(S1, h, c, pw);
      lds_fence();
    }
    get_rows<NN>(S1, t, i, w);
    sfor<0, NN>([&](auto J) { w[HD_K(J)] *= msk; });
    // t1 = R Sd + S+ (R's team row read here)
    double t1 = spl;
    {
      double rl[NN];
      load_row(rec, 0, rl);
      sfor<0, NN>([&](auto K) { t1 = fma(rl[HD_K(K)], bc<HD_K(K)>(sd), t1); });
    }
    // LU without pivoting; reciprocal pivots on the diagonal
    sfor<0, NN>([&](auto K) {
      constexpr int k = HD_K(K);
      const double piv = bc<k>(w[k]);
      if (!(fabs(piv) > 1.0e-12)) st |= kStPivot;
      const double rp = rcp_nr(piv);
      const double lik = w[k] * rp;
      const double mm = i > k ? lik : 0.0;
      w[k] = i == k ? rp : (i > k ? lik : w[k]);
      sfor<k + 1, NN>([&](auto J) {
        constexpr int j = HD_K(J);
        w[j] = fma(-mm, bc<k>(w[j]), w[j]);
      });
      pin<NN>(w);  // this step's broadcasts stay in this step
    });
    // t1 <- W1^-1 t1
    sfor<0, NN>([&](auto K) {
      constexpr int k = HD_K(K);
      const double tk = bc<k>(t1);
      if (i > k) t1 = fma(-w[k], tk, t1);
    });
    sfor_rev<0, NN>([&](auto K) {
      constexpr int k = HD_K(K);
      if (i == k) t1 *= w[k];
      const double tk = bc<k>(t1);
      if (i < k) t1 = fma(-w[k], tk, t1);
    });
    // u = A t1 + Sd (A's row i from S0)
    double u = sd;
    {
      double ar[NN];
      get_rows<NN>(S0, t, i, ar);
      sfor<0, NN>([&](auto K) { u = fma(ar[HD_K(K)] * msk, bc<HD_K(K)>(t1), u); });
    }
    bw[NN * NN + ii] = t1;
    // columns of L^-1 and U^-1 from the LU rows (hd_team_mfma_sweep_kernel)
    {
      double zl[NN], zu[NN];
      sfor<0, NN>([&](auto R) {
        constexpr int r = HD_K(R);
        double v = i == r ? 1.0 : 0.0;
        sfor<0, r>([&](auto K) { v = fma(-bc<r>(w[HD_K(K)]), zl[HD_K(K)], v); });
        zl[r] = v;
        pin<NN>(w);
      });
      sfor_rev<0, NN>([&](auto R) {
        constexpr int r = HD_K(R);
        double v = i == r ? 1.0 : 0.0;
        sfor<r + 1, NN>([&](auto K) { v = fma(-bc<r>(w[HD_K(K)]), zu[HD_K(K)], v); });
        zu[r] = v * bc<r>(w[r]);
        pin<NN>(w);
      });
      sfor<0, NN>([&](auto J) {
        zl[HD_K(J)] *= msk;
        zu[HD_K(J)] *= msk;
      });
      lds_fence();
      put_rows<NN>(S0, t, i, zl);  // L^-T, row-major (A's rows in S0 are done)
      put_rows<NN>(S1, t, i, zu);  // U^-T, row-major
    }
    // Sd <- T u + S- (T's team row read here)
    {
      double tr[NN];
      load_row(rec, NN * NN, tr);
      double tq = rec[2 * NN * NN + NN + ii] * msk * sscale;
      sfor<0, NN>([&](auto K) { tq = fma(tr[HD_K(K)], bc<HD_K(K)>(u), tq); });
      sd = tq * msk;
    }
    lds_fence();
    // ZT = U^-1 (L^-1 T); record; A <- R + T (A ZT); A's rows to S0 for the next layer
    {
      double li[4][4], x1[4][4], zm[4][4];
      {
        double tm[4][4];
        load_m(lc, NN * NN, tm);
        get_m(S0, h, c, li);
        mprod<false>(li, tm, x1, h, c);  // L^-1 T
      }
      get_m(S1, h, c, li);
      mprod<false>(li, x1, zm, h, c);  // ZT = U^-1 (L^-1 T)
      // The second reads of T~ and R~ and tau' go out before ZT's stores: a load
      // issued after a store also waits for that store to retire (one in-order
      // memory counter), so read after them each waited out 16 store round trips
      const double taul = rec[2 * NN * NN + 2 * NN];
      double pm[4][4];
      mprod<false>(ram, zm, pm, h, c);  // A ZT   (A symmetric: its own transpose)
      {
        double tm[4][4];
        load_m(lc, NN * NN, tm);
        mprod<false>(tm, pm, ram, h, c);  // T (A ZT)
      }
      double rm[4][4];
      load_m(lc, 0, rm);
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        double* zr = A.bsub + ((size_t)lc * nsc + (g0 + tt < A.nsc ? g0 + tt : g0)) * ne2t<NN>();
        const bool ok = g0 + tt < A.nsc;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int r = h + 4 * m;
          // branch-free: an element the lane does not own goes to the sink
          rec_st<NT>((ok && r < NN && c < NN) ? zr + r * NN + c : A.sink + lane, zm[tt][m]);
        }
      }
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int m = 0; m < 4; ++m) ram[tt][m] += rm[tt][m];
      lds_fence();
      put_m(S0, h, c, ram);
      lds_fence();
      tauc += taul;
    }
  }

  // ---- Lambertian surface: I+ = g x ----
  double rgrow = 0.0;
  {
    double ar[NN];
    get_rows<NN>(S0, t, i, ar);
    sfor<0, NN>([&](auto J) { rgrow = fma(ar[HD_K(J)] * msk, Qc.g[HD_K(J)], rgrow); });
  }
  const double gsd = bc<0>(team_sum(g_i * sd));
  const double grg = bc<0>(team_sum(g_i * rgrow));
  double esurf = (1.0 - alb) * bsurf;
  const double dirsurf = f0mu0 * exp(-tauc * rmu0);
  if (beam) esurf += alb * dirsurf / kPi;
  const double x = (2.0 * alb * gsd + esurf) / (1.0 - 2.0 * alb * grg);
  double ip = g_i * x;
  double* fo = A.flux + (size_t)(A.flux_local ? (long)sl : s) * (L + 1) * 2;
  double chk = 0.0;
  {
    const double up = team_sum(g_i * ip);
    const double dn = team_sum(g_i * fma(rgrow, x, sd));
    if (i == 0 && valid) {
      fo[0] = twopi * up;
      fo[1] = twopi * dn + dirsurf;
    }
    chk += twopi * up + twopi * dn;
  }
  // ---- back-substitution bottom -> top ----
  for (int lc = L - 1; lc >= 0; --lc) {
    const double* bp = A.bsub + ((size_t)lc * nsc + sl) * ne2t<NN>();
    double nip = bp[NN * NN + ii] * msk;
    sfor<0, NN>([&](auto J) {
      const double z = bp[ii * NN + HD_K(J)] * msk;
      nip = fma(z, bc<HD_K(J)>(ip), nip);
    });
    const double rc = bp[NN * NN + NN + ii] * msk;
    const double up = team_sum(g_i * nip);
    const double dn = team_sum(rc * nip);
    ip = nip;
    if (i == 0 && valid) {
      const int lev = L - lc;
      fo[2 * lev] = twopi * up;
      fo[2 * lev + 1] = bp[NN * NN + 2 * NN] + dn;
    }
    chk += twopi * up + dn;
  }
  if (!isfinite(chk)) st |= kStNonFinite;
  if (valid && st) {
    atomicOr(&A.status[s], st);
    if (st & 0x0F) atomicOr(A.anyerr, 1);
  }
}

// ============================================================================
// Intensity path, nstr 18..32: hd_rad.hip's per-(unit, layer) setup
// (hd_rad_layer_kernel: the flux layer setup for azimuthal mode m with the
// Y_l^m(mu_i) tables, parity of l+m, beam source x (2 - delta_m0), thermal only
// at m = 0, plus L, V, k, the particular solution and the exponentials kept for
// the radiance kernels) on the team layout with the dense products on the matrix
// core: hd_team_mfma_layer_kernel's algebra, four units per wave.  Writes the
// radiance records unit-contiguous ([layer][unit][element]): rsw (R~/T~ packed
// upper, S~+-, tau') for the team sweep, rrd (L packed, V, k, Z+-, h, B_top,
// dB/dtau', tau', omega', e^{-k tau'}, e^{-tau'/mu0}) for the team user-angle kernel
// and the rolled flux / const / user kernels (hd_rad.hip's HD_RREC at these sizes).
// ============================================================================
template <int NN>
__global__ __launch_bounds__(64, 2) void hd_rad_team_layer_kernel(RadArgs A) {
  __shared__ double lds[2 * kSet + 4 * 2 * 16];
  double* S0 = lds;
  double* S1 = lds + kSet;
  double* G = lds + 2 * kSet;  // [t][dsq | gsq][16]
  constexpr int N = 2 * NN;
  constexpr int nsym = NN * (NN + 1) / 2;
  constexpr int NE1 = rad_layer_record_doubles(NN);
  constexpr int NR = rad_rec_doubles(NN);
  constexpr int oV = nsym, oK = nsym + NN * NN, oZp = oK + NN, oZm = oZp + NN, oH = oZm + NN;
  constexpr int oBt = oH + NN, oSl = oBt + 1, oTp = oSl + 1, oOm = oTp + 1, oEk = oOm + 1;
  constexpr int oE0 = oEk + NN;
  const Quad<NN>& Qc = tquad<NN>(c_qt);
  const int lane = (int)threadIdx.x;
  const int h = lane >> 4, c = lane & 15;  // M layout
  const int t = h, i = c;                  // T layout: team t, row i
  const bool act = i < NN;
  const int ii = act ? i : 0;
  const int L = A.nlyr;
  const size_t nu = A.nu;
  // block = 4 consecutive units of one layer, blocks numbered layer-fastest and
  // XCD-aware as in the flux kernel
  const int grp = block_group(L);
  const int lc = block_layer(L);
  const bool valid = grp * 4 + t < A.nu;
  const int u = valid ? grp * 4 + t : grp * 4;
  const int m = u / A.ns;
  const int sl = u - m * A.ns;
  const long s = A.s0 + sl;
  const int nm = A.nmom;
  const int np = A.nprop;
  const bool wr = valid && act;
  int st = 0;
  int um[4];
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) um[tt] = grp * 4 + tt < A.nu ? grp * 4 + tt : grp * 4;
  double* rr = A.rrd + ((size_t)lc * nu + u) * NR;   // element e: rr[e]
  double* out = A.rsw + (size_t)lc * NE1 * nu;    // element e of unit v: out[v * NE1 + e]

  for (int k = lane; k < 2 * kSet; k += 64) lds[k] = 0.0;
  lds_fence();

  const double msk = act ? 1.0 : 0.0;
  const double mu_i = fma(msk, Qc.mu[ii] - 1.0, 1.0);
  const double sd_i = Qc.sd[ii] * msk;
  const double g_i = Qc.g[ii] * msk;
  const double rmu_i = Qc.rmu[ii] * msk;
  const double rg_i = Qc.rg[ii] * msk;

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
  const bool therm = A.planck && m == 0;

  // ---- mode-m phase-matrix rows (parity of l+m): S+ (ap), S- (lch); beam sums ----
  double ap[NN], lch[NN];
  double xs = 0.0, xd = 0.0;
  sfor<0, NN>([&](auto J) { ap[HD_K(J)] = lch[HD_K(J)] = 0.0; });
  {
    const int mp = m & 1;
    const double* lam = rad_lam<NN>(m);
    const double sx = sqrt(fmax(0.0, 1.0 - mub * mub));
    double seed = c_rtt.seed[m];
    for (int a = 0; a < m; ++a) seed *= sx;  // Y_m^m(mu0)
    double y1 = 0.0, y2 = 0.0;                // Y_{l-1}^m(mu0), Y_{l-2}^m(mu0)
#pragma nounroll
    for (int l2 = 0; l2 < NN; ++l2) {
      const int la = 2 * l2, lb = la + 1;
      const double ya =
          la < m ? 0.0 : (la == m ? seed : fma(c_rtt.ra[m][la] * mub, y1, -c_rtt.rb[m][la] * y2));
      y2 = y1;
      y1 = ya;
      const double yb =
          lb < m ? 0.0 : (lb == m ? seed : fma(c_rtt.ra[m][lb] * mub, y1, -c_rtt.rb[m][lb] * y2));
      y2 = y1;
      y1 = yb;
      const int le = mp ? lb : la, lo = mp ? la : lb;
      const double pe0 = mp ? yb : ya, po0 = mp ? ya : yb;
      const double che = le == 0 ? 1.0 : (le <= nm ? q[1 + le] : 0.0);
      const double cho = lo == 0 ? 1.0 : (lo <= nm ? q[1 + lo] : 0.0);
      const double ge = (2 * le + 1) * (che - f) * rf;
      const double go = (2 * lo + 1) * (cho - f) * rf;
      const double te = lam[le * NN + ii] * msk;  // Y_le^m(mu_i), this lane's node
      const double to = lam[lo * NN + ii] * msk;
      const double ue = ge * te;
      const double uo = go * to;
      xs = fma(ue, pe0, xs);
      xd = fma(uo, po0, xd);
      sfor<0, NN>([&](auto J) {
        constexpr int j = HD_K(J);
        ap[j] = fma(ue, bc<j>(te), ap[j]);
        lch[j] = fma(uo, bc<j>(to), lch[j]);
      });
    }
  }
  sfor<0, NN>([&](auto J) {
    constexpr int j = HD_K(J);
    const double diag = i == j ? rmu_i : 0.0;
    const double sij = sd_i * Qc.sd[j];
    lch[j] = fma(-sij, lch[j], diag);
    ap[j] = fma(-sij, ap[j], diag);
  });
  // L L^T = S-
  double lt[NN], rdl;
  if (!team_chol<NN, true>(lch, lt, rdl)) st |= kStEigen;
  {  // L, packed lower row-major: row i holds lch[k], k <= i.  Branch-free: the
     // elements a lane does not own go to the sink.  Stores under a lane-dependent
     // condition inside the unrolled loop cost 1 KB of spill at two waves per SIMD
    double* lrow = rr + i * (i + 1) / 2;
    sfor<0, NN>([&](auto K) {
      constexpr int k = HD_K(K);
      double* dst = (wr && k <= i) ? &lrow[k] : A.sink + lane;
      *dst = lch[k];
    });
  }

  // ---- pre-Jacobi vectors (depend on L only) ----
  double w2 = 0.0, lxd = 0.0;
  const double fb2 = fb * ((m == 0 ? 0.5 : 1.0) / kPi);
  if (beam) {
    const double y = sd_i * (fb2 * xs);
    double z = 0.0;  // z = L^T y
    sfor<0, NN>([&](auto K) { z = fma(lt[HD_K(K)], bc<HD_K(K)>(y), z); });
    const double yl = team_matvec<NN>(lch, z);  // L z
    const double xdi = -fb2 * xd;
    const double rv = fma(-yl, rg_i, xdi * rmu0 * rmu_i);
    w2 = g_i * rv;
    lxd = sd_i * xdi;
    team_lsolve<NN>(lch, rdl, w2);
    team_usolve<NN>(lt, rdl, w2);
    team_lsolve<NN>(lch, rdl, lxd);
    team_usolve<NN>(lt, rdl, lxd);
  }
  double cvec = 0.0, db = 0.0, bsum = 0.0;
  if (therm) {
    const double bt = A.planckv[(size_t)(L - lc) * A.ns + sl];
    const double bb = taup > 0.0 ? A.planckv[(size_t)(L - lc - 1) * A.ns + sl] : bt;
    db = bb - bt;
    bsum = bt + bb;
    const double b1 = taup > 0.0 ? 2.0 * db / taup : 0.0;
    cvec = sd_i * mu_i;
    team_lsolve<NN>(lch, rdl, cvec);
    team_usolve<NN>(lt, rdl, cvec);
    if (wr) rr[oH + i] = rg_i * cvec;
    cvec = fma(b1 * rg_i, cvec, db) * msk;
    if (valid && i == 0) {
      rr[oBt] = bt;
      rr[oSl] = 0.5 * b1;
    }
  } else {
    if (wr) rr[oH + i] = 0.0;
    if (valid && i == 0) {
      rr[oBt] = 0.0;
      rr[oSl] = 0.0;
    }
  }
  if (valid && i == 0) {
    rr[oTp] = taup;
    rr[oOm] = om;
  }
  {
    double z[NN];
    team_tri_inverse_col<NN>(lch, rdl, z);  // row i of L^-T -> S0 (lch dies here)
    put_rows<NN>(S0, t, i, z);
  }

  // ---- C C^T = S+ ; B0 = C^T L (lane j: column j) ; C^-1 to LDS ----
  double bcol[NN];
  {
    double unused[NN], rdc;
    if (!team_chol<NN, false>(ap, unused, rdc)) st |= kStEigen;
    sfor<0, NN>([&](auto I) {
      constexpr int r = HD_K(I);
      double uu = 0.0;
      sfor<r, NN>([&](auto K) { uu = fma(bc<HD_K(K)>(ap[r]), lt[HD_K(K)], uu); });
      bcol[r] = uu;
      pin<NN>(ap);
    });
    double z[NN];
    team_tri_inverse_col<NN>(ap, rdc, z);  // row i of C^-T -> S1
    put_rows<NN>(S1, t, i, z);
  }

  // ---- eigenpairs: Sym = L^T S+ L = B0^T B0 = V diag(k^2) V^T ----
  lds_fence();
  if (!team_jacobi<NN>(bcol, A.max_sweeps)) st |= kStEigen;
  lds_fence();
  double kk;
  {
    double k2 = 0.0;
    sfor<0, NN>([&](auto K) { k2 = fma(bcol[HD_K(K)], bcol[HD_K(K)], k2); });
    if (act && !(k2 > 0.0)) st |= kStEigen;
    kk = sqrt(k2 > 0.0 ? k2 : 0.0) * msk;
    const double x = kk * taup;
    const double mm = -expm1(-x);
    const double th = mm * rcp_nr(2.0 - mm);
    const double delta = x > 1.0e-8 ? th * rcp_nr(kk > 0.0 ? kk : 1.0) : 0.5 * taup;
    G[t * 32 + i] = sqrt(delta) * msk;
    G[t * 32 + 16 + i] = sqrt(kk * th) * msk;
    if (wr) {
      rr[oK + i] = kk;
      rr[oEk + i] = 1.0 - mm;  // exp(-k tau')
    }
  }

  // ---- the dense products on the matrix core; V = L^-1 U; the beam solution ----
  double zp = 0.0, zm = 0.0, e0 = 0.0;
  {
    double X[4][4], Y[4][4], U[4][4], UT[4][4];
    {
      // L^-T stays in S0 until V = L^-1 U is formed; W = L^-T L^-1 is formed after
      // it from the same rows (no M-layout copy of L^-T or W held across the products)
      get_mt(S1, h, c, X);           // C^-1 (M)
      lds_fence();
      put_rows<NN>(S1, t, i, bcol);  // rows of B^T
      lds_fence();
      get_mt(S1, h, c, Y);           // B (M)
      mprod<false>(X, Y, U, h, c);   // U = C^-T B
      mprod<false>(Y, X, UT, h, c);  // U^T = B^T C^-1
      get_m(S0, h, c, Y);            // L^-T (M): the A^T operand of L^-1 (.)
      mprod<false>(Y, U, X, h, c);   // V = L^-1 U (M) -> the record, row-major
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const bool ok = grp * 4 + tt < A.nu;
        double* rv = A.rrd + ((size_t)lc * nu + um[tt]) * NR;
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) {
          const int r = h + 4 * q2;
          if (ok && r < NN && c < NN) rv[oV + r * NN + c] = X[tt][q2];
        }
      }
      get_mt(S0, h, c, X);          // L^-1 (M)
      mprod<false>(X, X, Y, h, c);  // W = L^-T L^-1
      lds_fence();
      put_m(S0, h, c, Y);           // W, row-major
    }
    lds_fence();
    put_m(S1, h, c, UT);
    lds_fence();
    if (beam) {
      double r_[NN];
      get_rows<NN>(S1, t, i, r_);
      const double r2 = rmu0 * rmu0;
      const double tv = team_matvec<NN>(r_, w2);
      double den = fma(-kk, kk, r2);
      if (act && fabs(den) < 1.0e-9 * r2) {
        st |= kStResonance;
        den = den < 0.0 ? -1.0e-9 * r2 : 1.0e-9 * r2;
      }
      const double ttv = tv / den * msk;
      get_cols<NN>(S1, t, i, r_);
      const double sv = team_matvec<NN>(r_, ttv) * rg_i;
      get_rows<NN>(S0, t, i, r_);
      const double yy = team_matvec<NN>(r_, sd_i * mu_i * sv);
      const double tauc = A.tauc[(size_t)lc * A.ns + sl];
      const double att = 0.5 * exp(-tauc * rmu0);
      const double dd = rg_i * fma(-yy, rmu0, lxd);
      zp = (sv + dd) * att;
      zm = (sv - dd) * att;
      e0 = exp(-taup * rmu0);
    }
    if (wr) {
      rr[oZp + i] = zp;
      rr[oZm + i] = zm;
    }
    if (valid && i == 0) rr[oE0] = e0;
    get_m(S0, h, c, Y);            // W (M)
    mprod<false>(U, Y, X, h, c);   // U^T W
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
#pragma unroll
      for (int q2 = 0; q2 < 4; ++q2) {
        X[tt][q2] *= G[tt * 32 + 16 + h + 4 * q2];
        UT[tt][q2] *= G[tt * 32 + h + 4 * q2];
      }
    mprod<true>(UT, UT, U, h, c);  // I + Omega Omega^T
    mprod<true>(X, X, Y, h, c);    // I + Psi^T Psi
    lds_fence();
    put_m(S0, h, c, U);
    put_m(S1, h, c, Y);
    lds_fence();
  }
  const double ga = g_i * (cvec - fma(-zp, e0, zm));
  const double gb = g_i * (fma(zp, e0, zm) + bsum);

  // ---- A- = (I + Omega Omega^T)^-1, A+ = (I + Psi^T Psi)^-1 ----
  double Am[4][4], Ap[4][4];
  double pv, qv;
  {
    double hr[NN], unused[NN], z[NN], jrd, X[4][4];
    get_rows<NN>(S0, t, i, hr);
    if (!team_chol<NN, false>(hr, unused, jrd)) st |= kStEigen;
    team_tri_inverse_col<NN>(hr, jrd, z);
    lds_fence();
    put_rows<NN>(S0, t, i, z);
    lds_fence();
    get_mt(S0, h, c, X);
    mprod<false>(X, X, Am, h, c);
    lds_fence();
    put_m(S0, h, c, Am);
    lds_fence();
    get_rows<NN>(S0, t, i, hr);
    pv = ga - team_matvec<NN>(hr, ga);
    get_rows<NN>(S1, t, i, hr);
    if (!team_chol<NN, false>(hr, unused, jrd)) st |= kStEigen;
    team_tri_inverse_col<NN>(hr, jrd, z);
    lds_fence();
    put_rows<NN>(S1, t, i, z);
    lds_fence();
    get_mt(S1, h, c, X);
    mprod<false>(X, X, Ap, h, c);
    lds_fence();
    put_m(S1, h, c, Ap);
    lds_fence();
    get_rows<NN>(S1, t, i, hr);
    qv = team_matvec<NN>(hr, gb) - gb;
  }

  // ---- store: R~ = A+ - A-, T~ = A- + A+ - I packed upper (M layout), S~+-, tau' ----
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) {
    double chk = 0.0;
    const bool ok = grp * 4 + tt < A.nu;
#pragma unroll
    for (int q2 = 0; q2 < 4; ++q2) {
      const int r = h + 4 * q2;
      const double rrv = Ap[tt][q2] - Am[tt][q2];
      const double trv = (Am[tt][q2] + Ap[tt][q2]) - (r == c ? 1.0 : 0.0);
      if (ok && r <= c && c < NN) {
        const int e = sym_index<NN>(r, c);
        out[(size_t)um[tt] * NE1 + e] = rrv;
        out[(size_t)um[tt] * NE1 + nsym + e] = trv;
      }
      chk += rrv + trv;
    }
    if (ok && !isfinite(chk)) {
      const int vt = um[tt];
      atomicOr(&A.status[A.s0 + (vt - (vt / A.ns) * A.ns)], kStNonFinite);
      atomicOr(A.anyerr, 1);
    }
  }
  double chk = 0.0;
  const double sp = g_i * (zp * (1.0 - e0) - db) + pv - qv;
  const double sm = g_i * (-zm * (1.0 - e0) + db) - pv - qv;
  if (wr) {
    out[(size_t)u * NE1 + 2 * nsym + i] = sp;
    out[(size_t)u * NE1 + 2 * nsym + NN + i] = sm;
  }
  chk += sp + sm;
  if (valid && i == 0) out[(size_t)u * NE1 + 2 * nsym + 2 * NN] = taup;
  if (act && !isfinite(chk + taup)) st |= kStNonFinite;
  if (valid && st) {
    atomicOr(&A.status[s], st);
    if (st & 0x0F) atomicOr(A.anyerr, 1);
  }
}

// ============================================================================
// Intensity path, nstr 18..32: hd_rad.hip's per-unit adding sweep +
// back-substitution (hd_rad_sweep_kernel: the stack state R_above/S_down and
// I+/I- kept at every level) on the team layout with the dense products on the
// matrix core -- four units (solve, azimuthal mode) per wave, the arithmetic of
// hd_team_mfma_sweep_kernel above.  The layer-operator and back-substitution
// records (rsw, bsub) are unit-contiguous at these sizes ([layer][unit][element]:
// a team's loads and stores of one unit's record hit neighbouring lines, where the
// unit-fastest layout the one-lane kernels use put every lane on its own line);
// lev keeps the unit-fastest layout the per-lane kernels read.  Replaces a
// one-lane-per-unit loop whose 16 x 16 matrices lived in private memory
// (62% of the nstr-32 radiance time, profiles/r03/).
// ============================================================================
template <int NN>
__global__ __launch_bounds__(64, 1) void hd_rad_team_sweep_kernel(RadArgs A) {
  __shared__ double lds[2 * kSet];
  double* S0 = lds;
  double* S1 = lds + kSet;
  const Quad<NN>& Qc = tquad<NN>(c_qt);
  constexpr int nsym = NN * (NN + 1) / 2;
  constexpr int NE1 = rad_layer_record_doubles(NN);
  constexpr int NB = rad_bsub_doubles(NN);
  const int lane = (int)threadIdx.x;
  const int h = lane >> 4, c = lane & 15;  // M layout
  const int t = h, i = c;                  // T layout: team t, row i
  const bool act = i < NN;
  const int ii = act ? i : 0;
  const int grp = (int)blockIdx.x;
  // every lane takes part in the MFMA / LDS / DPP exchanges: a team past the end
  // repeats the block's first unit and stores nothing
  const bool valid = grp * 4 + t < A.nu;
  const int u = valid ? grp * 4 + t : grp * 4;
  const int m = u / A.ns;
  const int sl = u - m * A.ns;
  const long s = A.s0 + sl;
  const int L = A.nlyr;
  const size_t nu = A.nu;
  int st = 0;
  const double msk = act ? 1.0 : 0.0;
  const double g_i = Qc.g[ii] * msk;
  const double rg_i = Qc.rg[ii] * msk;
  const bool wr = valid && act;

  for (int k = lane; k < 2 * kSet; k += 64) lds[k] = 0.0;
  lds_fence();

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

  int um[4];  // the wave's four units (M layout)
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) um[tt] = grp * 4 + tt < A.nu ? grp * 4 + tt : grp * 4;

  double ram[4][4];  // R_above (M layout)
  double ra[NN];     // R_above row i (T layout)
  double sd = g_i * top;
#pragma unroll
  for (int tt = 0; tt < 4; ++tt)
#pragma unroll
    for (int q = 0; q < 4; ++q) ram[tt][q] = 0.0;
  sfor<0, NN>([&](auto J) { ra[HD_K(J)] = 0.0; });
  double tauc = 0.0;

  for (int lc = 0; lc < L; ++lc) {
    const double* lp = A.rsw + (size_t)lc * NE1 * nu;  // element e of unit v: lp[v*NE1 + e]
    double* bp = A.bsub + (size_t)lc * NB * nu;
    // the stack above this layer: R_above (packed upper, row i from j = i) and S_down
    {  // branch-free: the elements a lane does not own go to the sink
      double* urow = bp + (size_t)u * NB + NN * NN + NN + sym_index<NN>(ii, ii) - ii;
      sfor<0, NN>([&](auto J) {
        constexpr int j = HD_K(J);
        double* dst = (wr && j >= i) ? urow + j : A.sink + lane;
        *dst = ra[j];
      });
      *(wr ? bp + (size_t)u * NB + NN * NN + NN + nsym + i : A.sink + lane) = sd;
    }
    // R~, T~ (packed upper) of the four units in M layout; this unit's rows (T layout)
    double rm[4][4], tm[4][4];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = h + 4 * q;
        const bool in = r < NN && c < NN;
        const int e = in ? sym_index<NN>(r, c) : 0;
        rm[tt][q] = in ? lp[(size_t)um[tt] * NE1 + e] : 0.0;
        tm[tt][q] = in ? lp[(size_t)um[tt] * NE1 + nsym + e] : 0.0;
      }
    double rl[NN], tr[NN];
    sfor<0, NN>([&](auto J) {
      const int e = sym_index<NN>(ii, HD_K(J));
      rl[HD_K(J)] = lp[(size_t)u * NE1 + e] * msk;
      tr[HD_K(J)] = lp[(size_t)u * NE1 + nsym + e] * msk;
    });
    const double spl = lp[(size_t)u * NE1 + 2 * nsym + ii] * msk;
    const double sml = lp[(size_t)u * NE1 + 2 * nsym + NN + ii] * msk;
    // W1 = I - R A on the matrix core, to team rows through LDS
    {
      double pw[4][4];
      mprod<false>(rm, ram, pw, h, c);
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int q = 0; q < 4; ++q) pw[tt][q] = (h + 4 * q == c ? 1.0 : 0.0) - pw[tt][q];
      lds_fence();
      put_m(S0, h, c, pw);
      lds_fence();
    }
    double w[NN];
    get_rows<NN>(S0, t, i, w);
    sfor<0, NN>([&](auto J) { w[HD_K(J)] *= msk; });
    // t1 = R Sd + S+
    double t1 = spl;
    sfor<0, NN>([&](auto K) { t1 = fma(rl[HD_K(K)], bc<HD_K(K)>(sd), t1); });
    // LU without pivoting; reciprocal pivots on the diagonal
    sfor<0, NN>([&](auto K) {
      constexpr int k = HD_K(K);
      const double piv = bc<k>(w[k]);
      if (!(fabs(piv) > 1.0e-12)) st |= kStPivot;
      const double rp = rcp_nr(piv);
      const double lik = w[k] * rp;
      const double mm = i > k ? lik : 0.0;
      w[k] = i == k ? rp : (i > k ? lik : w[k]);
      sfor<k + 1, NN>([&](auto J) {
        constexpr int j = HD_K(J);
        w[j] = fma(-mm, bc<k>(w[j]), w[j]);
      });
    });
    // t1 <- W1^-1 t1
    sfor<0, NN>([&](auto K) {
      constexpr int k = HD_K(K);
      const double tk = bc<k>(t1);
      if (i > k) t1 = fma(-w[k], tk, t1);
    });
    sfor_rev<0, NN>([&](auto K) {
      constexpr int k = HD_K(K);
      if (i == k) t1 *= w[k];
      const double tk = bc<k>(t1);
      if (i < k) t1 = fma(-w[k], tk, t1);
    });
    // u = A t1 + Sd
    double uv = sd;
    sfor<0, NN>([&](auto K) { uv = fma(ra[HD_K(K)], bc<HD_K(K)>(t1), uv); });
    *(wr ? bp + (size_t)u * NB + NN * NN + i : A.sink + lane) = t1;
    // ZT = W1^-1 T = U^-1 (L^-1 T): columns of the triangular inverses on the team
    // (lane i: row i of the transposed inverse), the products on the matrix core
    {
      double zl[NN], zu[NN];
      sfor<0, NN>([&](auto R) {
        constexpr int r = HD_K(R);
        double v = i == r ? 1.0 : 0.0;
        sfor<0, r>([&](auto K) { v = fma(-bc<r>(w[HD_K(K)]), zl[HD_K(K)], v); });
        zl[r] = v;
        pin<NN>(w);
      });
      sfor_rev<0, NN>([&](auto R) {
        constexpr int r = HD_K(R);
        double v = i == r ? 1.0 : 0.0;
        sfor<r + 1, NN>([&](auto K) { v = fma(-bc<r>(w[HD_K(K)]), zu[HD_K(K)], v); });
        zu[r] = v * bc<r>(w[r]);
        pin<NN>(w);
      });
      sfor<0, NN>([&](auto J) {
        zl[HD_K(J)] *= msk;
        zu[HD_K(J)] *= msk;
      });
      lds_fence();
      put_rows<NN>(S0, t, i, zl);  // L^-T
      put_rows<NN>(S1, t, i, zu);  // U^-T
    }
    // Sd <- T u + S-
    {
      double tq = sml;
      sfor<0, NN>([&](auto K) { tq = fma(tr[HD_K(K)], bc<HD_K(K)>(uv), tq); });
      sd = tq * msk;
    }
    lds_fence();
    {
      double li[4][4], x1[4][4], zm[4][4], pm[4][4];
      get_m(S0, h, c, li);
      mprod<false>(li, tm, x1, h, c);  // L^-1 T
      get_m(S1, h, c, li);
      mprod<false>(li, x1, zm, h, c);  // ZT
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const bool ok = grp * 4 + tt < A.nu;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = h + 4 * q;
          const bool own = ok && r < NN && c < NN;
          *(own ? bp + (size_t)um[tt] * NB + r * NN + c : A.sink + lane) = zm[tt][q];
        }
      }
      mprod<false>(ram, zm, pm, h, c);  // A ZT
      mprod<false>(tm, pm, ram, h, c);  // T (A ZT)
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int q = 0; q < 4; ++q) ram[tt][q] += rm[tt][q];
      lds_fence();
      put_m(S0, h, c, ram);
      lds_fence();
    }
    get_rows<NN>(S0, t, i, ra);
    sfor<0, NN>([&](auto J) { ra[HD_K(J)] *= msk; });
    tauc += lp[(size_t)u * NE1 + 2 * nsym + 2 * NN];
  }

  // ---- Lambertian surface (mode 0): I+ = g x ----
  double rgrow = 0.0;
  sfor<0, NN>([&](auto J) { rgrow = fma(ra[HD_K(J)], Qc.g[HD_K(J)], rgrow); });
  const double gsd = bc<0>(team_sum(g_i * sd));
  const double grg = bc<0>(team_sum(g_i * rgrow));
  double esurf = (1.0 - alb) * bsurf;
  if (beam) esurf += alb * f0mu0 * exp(-tauc * rmu0) / kPi;
  const double x = (2.0 * alb * gsd + esurf) / (1.0 - 2.0 * alb * grg);
  double ip = g_i * x;
  double chk = 0.0;
  {
    double dn = sd;
    sfor<0, NN>([&](auto J) { dn = fma(ra[HD_K(J)], bc<HD_K(J)>(ip), dn); });
    double* lv = A.lev + (size_t)L * 2 * NN * nu;
    if (wr) {
      lv[(size_t)i * nu + u] = x;
      lv[(size_t)(NN + i) * nu + u] = dn * rg_i;
    }
    chk += dn * msk;
  }
  // ---- back-substitution bottom -> top, I+ and I- at every level ----
  for (int lc = L - 1; lc >= 0; --lc) {
    const double* bp = A.bsub + (size_t)lc * NB * nu;
    double nip = bp[(size_t)u * NB + NN * NN + ii] * msk;
    sfor<0, NN>([&](auto J) {
      nip = fma(bp[(size_t)u * NB + ii * NN + HD_K(J)] * msk, bc<HD_K(J)>(ip), nip);
    });
    ip = nip;
    double dn = bp[(size_t)u * NB + NN * NN + NN + nsym + ii] * msk;
    sfor<0, NN>([&](auto J) {
      const double r = bp[(size_t)u * NB + NN * NN + NN + sym_index<NN>(ii, HD_K(J))] * msk;
      dn = fma(r, bc<HD_K(J)>(ip), dn);
    });
    double* lv = A.lev + (size_t)lc * 2 * NN * nu;
    if (wr) {
      lv[(size_t)i * nu + u] = ip * rg_i;
      lv[(size_t)(NN + i) * nu + u] = dn * rg_i;
    }
    chk += ip + dn;
  }
  if (act && !isfinite(chk)) st |= kStNonFinite;
  if (valid && st) {
    atomicOr(&A.status[s], st);
    if (st & 0x0F) atomicOr(A.anyerr, 1);
  }
}

hipError_t upload_warm_tables_team(const QuadHost* per_nn) {
  // the host tables (a long-double Jacobi per entry) are built once per process;
  // each device only receives the copy
  static std::vector<double> all;
  static std::once_flag once;
  std::call_once(once, [per_nn] {
    all.assign((size_t)(kMaxNN - kMaxRegNN) * kWarmEntries * kWarmTeam, 0.0);
    for (int nn = kMaxRegNN + 1; nn <= kMaxNN; ++nn) {
      double* tab = all.data() + (size_t)(nn - kMaxRegNN - 1) * kWarmEntries * kWarmTeam;
      for (int e = 0; e < kWarmEntries; ++e) {
        double v[kMaxNN * kMaxNN];
        if (e < kWarmG * kWarmG) {
          warm_eigvecs(nn, per_nn[nn - 1], e / kWarmG, e % kWarmG, v);
        } else {
          for (int k = 0; k < nn * nn; ++k) v[k] = k % (nn + 1) == 0 ? 1.0 : 0.0;
        }
        double* ent = tab + (size_t)e * kWarmTeam;
        for (int r = 0; r < nn; ++r)
          for (int c = 0; c < nn; ++c) ent[(4 * c + r % 4) * 4 + r / 4] = v[r * nn + c];
      }
    }
  });
  return hipMemcpyToSymbol(HIP_SYMBOL(d_warm_team), all.data(), sizeof(double) * all.size(), 0,
                           hipMemcpyHostToDevice);
}

hipError_t upload_quad_tables_team_mfma(const QuadTablesTeam& t) {
  return hipMemcpyToSymbol(HIP_SYMBOL(c_qt), &t, sizeof(t), 0, hipMemcpyHostToDevice);
}

template <int NN>
static hipError_t launch_layer(const LayerArgs& la, hipStream_t stream) {
  const unsigned nb1 = (unsigned)(((la.nsc + 3) / 4) * (long)la.nlyr);
  if (la.nsc >= kNtMinSolves)
    hipLaunchKernelGGL((hd_team_mfma_layer_kernel<NN, true>), dim3(nb1), dim3(64), 0, stream, la);
  else
    hipLaunchKernelGGL((hd_team_mfma_layer_kernel<NN, false>), dim3(nb1), dim3(64), 0, stream, la);
  return hipGetLastError();
}

template <int NN>
static hipError_t launch_sweep(const SweepArgs& sa, hipStream_t stream) {
  const dim3 gl((unsigned)((sa.nsc + 3) / 4));
  if (sa.lean && sa.nsc >= kNtMinSolves)
    hipLaunchKernelGGL((hd_team_mfma_sweep_lean_kernel<NN, true>), gl, dim3(64), 0, stream, sa);
  else if (sa.lean)
    hipLaunchKernelGGL((hd_team_mfma_sweep_lean_kernel<NN, false>), gl, dim3(64), 0, stream, sa);
#if HD_AB_VARIANTS
  else
    hipLaunchKernelGGL(hd_team_mfma_sweep_kernel<NN>, dim3((unsigned)((sa.nsc + 3) / 4)), dim3(64),
                       0, stream, sa);
#endif
  return hipGetLastError();
}

hipError_t launch_team_sweep_mfma(int nn, const SweepArgs& sa, hipStream_t stream) {
  switch (nn) {
    case 9: return launch_sweep<9>(sa, stream);
    case 10: return launch_sweep<10>(sa, stream);
    case 11: return launch_sweep<11>(sa, stream);
    case 12: return launch_sweep<12>(sa, stream);
    case 13: return launch_sweep<13>(sa, stream);
    case 14: return launch_sweep<14>(sa, stream);
    case 15: return launch_sweep<15>(sa, stream);
    case 16: return launch_sweep<16>(sa, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_team_layer_mfma(int nn, const LayerArgs& la, hipStream_t stream) {
  switch (nn) {
    case 9: return launch_layer<9>(la, stream);
    case 10: return launch_layer<10>(la, stream);
    case 11: return launch_layer<11>(la, stream);
    case 12: return launch_layer<12>(la, stream);
    case 13: return launch_layer<13>(la, stream);
    case 14: return launch_layer<14>(la, stream);
    case 15: return launch_layer<15>(la, stream);
    case 16: return launch_layer<16>(la, stream);
    default: return hipErrorInvalidValue;
  }
}


// ============================================================================
// Intensity path, nstr 18..32: the user-angle source-function integration
// (hd_rad.hip's hd_rad_user_kernel, c_usrint) in two kernels.
//
// hd_rad_team_user_kernel: one wave = four (unit, layer) problems.  The mode-m
// phase row at a user angle enters only through H(+-k) = c_e X +- c_o Y (DESIGN.md
// section 3b), linear in the angle's Y_l^m row, so per problem the two maps
//     P^T = diag(sd) L V,   Q^T = -diag(sd) L^-T V K
// are formed once on the matrix core and applied to eight user angles at a time:
// [ce | cx] = [P | Q] . blockdiag(C_e, C_o), a 16 x 16 x 32 product whose B operand
// (the angles' c_e/c_o columns, lane (h, c): angle c & 7, parity c >> 3, rows
// h + 4s) each lane builds from the Y_l^m recurrences -- instead of one lane per
// (unit, angle) streaming L and V and solving with L for every angle (private
// memory at NN 9..16: 60 % of the nstr-32 radiance time, profiles/r03/rad/).
// Each lane then sums its four eigen-terms of the whole-layer integral (the
// decaying and the 1 - k|mu| -> 0 family through dexp), the team sums go through
// LDS, and 32 lanes add the beam and thermal terms: the layer's source term
// "lay" per (unit, angle) -> rsw (free after the sweep), and for user depths
// strictly inside the layer the partial integral from the depth to the ray's
// entry -> radm.
// hd_rad_team_user_scan_kernel: one lane per (unit, angle): the boundary value,
// then I_exit = I_entry e^{-tau'/|mu|} + lay layer by layer along the ray, the
// radiance at each user depth (interior: I_entry e^{-|t_in - t|/|mu|} + partial).
// ============================================================================
template <int NN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3)))
void hd_rad_team_user_kernel(RadArgs A) {
  // 11.5 KB: three waves per SIMD (L^T's M layout comes straight from the record)
  __shared__ double lds[kSet + 8 * 32 + 8 * 4 + 8 * 8];
  double* S0 = lds;          // rows of L^-T
  constexpr int N = 2 * NN;
  constexpr int nsym = NN * (NN + 1) / 2;
  constexpr int NE1 = rad_layer_record_doubles(NN);
  constexpr int NR = rad_rec_doubles(NN);
  constexpr int oV = nsym, oK = nsym + NN * NN, oZp = oK + NN, oZm = oZp + NN, oH = oZm + NN;
  constexpr int oBt = oH + NN, oSl = oBt + 1, oTp = oSl + 1, oOm = oTp + 1, oEk = oOm + 1;
  constexpr int oE0 = oEk + NN;
  const Quad<NN>& Qc = tquad<NN>(c_qt);
  const int lane = (int)threadIdx.x;
  const int h = lane >> 4, c = lane & 15;  // M layout
  const int t = h, i = c;                  // T layout: team t, row i
  const bool act = i < NN;
  const int ii = act ? i : 0;
  const int L = A.nlyr;
  const size_t nu = A.nu;
  const int grp = block_group(L);
  const int lc = block_layer(L);
  int um[4];
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) um[tt] = grp * 4 + tt < A.nu ? grp * 4 + tt : grp * 4;
  const double* rec = A.rrd + (size_t)lc * nu * NR;  // element e of unit v: rec[v * NR + e]
  auto rv = [&](int e, int tt) { return rec[(size_t)um[tt] * NR + e]; };

  for (int k = lane; k < kSet; k += 64) lds[k] = 0.0;
  lds_fence();

  // ---- L's rows (T layout) and L^-T's rows by the team's forward substitution ----
  {
    const int u = um[t];
    const int r0 = ii * (ii + 1) / 2;
    double lrow[NN];
    sfor<0, NN>([&](auto K) {
      constexpr int k = HD_K(K);
      lrow[k] = (act && k <= ii) ? rec[(size_t)u * NR + r0 + (k <= ii ? k : 0)] : 0.0;
    });
    double rdl = act ? 1.0 / rec[(size_t)u * NR + r0 + ii] : 0.0;
    double z[NN];
    team_tri_inverse_col<NN>(lrow, rdl, z);  // row i of L^-T
    put_rows<NN>(S0, t, i, z);
  }
  lds_fence();
  lds_fence();
  // ---- per problem: the layer's delta-M scalars (c_setdis, as hd_rad_user_kernel) ----
  int mt[4];
  double ft[4], rft[4], taupt[4];
  const double* qt[4];
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) {
    mt[tt] = um[tt] / A.ns;
    const int sl = um[tt] - mt[tt] * A.ns;
    qt[tt] = A.prop + ((size_t)(A.s0 + sl) * L + (L - 1 - lc)) * A.nprop;
    double ssa = A.nprop > 1 ? qt[tt][1] : 0.0;
    if (ssa == 1.0) ssa = 1.0 - kDither;
    const double f = A.nmom >= N ? qt[tt][1 + N] : 0.0;
    const double om = ssa * (1.0 - f) / (1.0 - ssa * f);
    ft[tt] = f;
    rft[tt] = om / (1.0 - f);
    taupt[tt] = rv(oTp, tt);
  }
  double* red = lds + kSet;      // [angle][lay | sc | x0 | th][h, parity]
  double* aux = red + 8 * 32;     // [angle][ab | a0 | a1t | -]
  double* red2 = aux + 8 * 4;     // [angle][h, parity]
  const int a = c & 7, fam = c >> 3;
  const int nmom = A.nmom;

  for (int ab0 = 0; ab0 < A.numu; ab0 += 8) {
    // the units laundered per angle block: the record loads below are then issued
    // where they are used instead of all being hoisted out of this loop (192 VGPRs)
    int uml[4];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      uml[tt] = um[tt];
      asm volatile("" : "+s"(uml[tt]));
    }
    auto rl = [&](int e, int tt) { return rec[(size_t)uml[tt] * NR + e]; };
    const int iu = ab0 + a;
    const bool aok = iu < A.numu;
    const double muu = aok ? A.umu[iu] : 1.0;
    const bool up = muu > 0.0;
    const double anu = fabs(muu);
    const double sxu = sqrt(fmax(0.0, 1.0 - muu * muu));
    // one problem at a time (compile-time tt: its PT/QT registers), fenced so that
    // only PT, QT and this problem's values are live
    sfor<0, 4>([&](auto TT) {
      constexpr int tt = HD_K(TT);
      asm volatile("" : "+s"(uml[tt]));  // this problem's loads stay in its phase
      int h_ = h, c_ = c;                 // as do its LDS reads and lane constants
      asm volatile("" : "+v"(h_), "+v"(c_));
      const int h = h_, c = c_;
      const int v = grp * 4 + tt;  // this problem's unit (>= nu: a repeat, not stored)
      const int m = mt[tt];
      const int sl = um[tt] - m * A.ns;
      const long s = A.s0 + sl;
      const double mu0 = A.umu0 ? A.umu0[s] : 1.0;
      const double fb = A.fbeam ? A.fbeam[s] : 0.0;
      const bool beam = fb > 0.0 && mu0 > 0.0;
      const double rmu0 = beam ? 1.0 / mu0 : 0.0;
      const bool therm = A.planck && m == 0;
      const double taup = taupt[tt];
      // ---- P^T = diag(sd) L V and Q^T = -diag(sd) L^-T V K, this problem's M layout
      // (the A^T operand of the next product) ----
      double PT[4], QT[4], cpl[4], cmi[4];
      {
        double vm[4], x[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = h + 4 * q;
          const bool in = r < NN && c < NN;
          vm[q] = in ? rl(oV + (in ? r * NN + c : 0), tt) : 0.0;
        }
        d4 p = {0.0, 0.0, 0.0, 0.0}, gq = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // L^T (M): L[c][h + 4q], packed lower in the record
          const int r = h + 4 * q;
          const bool in = r <= c && c < NN;
          x[q] = in ? rl(in ? c * (c + 1) / 2 + r : 0, tt) : 0.0;
        }
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) p = __builtin_amdgcn_mfma_f64_16x16x4f64(x[s4], vm[s4], p, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = S0[tt * kTile + c * kS + h + 4 * q];  // L^-1 (M)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) gq = __builtin_amdgcn_mfma_f64_16x16x4f64(x[s4], vm[s4], gq, 0, 0, 0);
        // ---- the layer's homogeneous constants from its level intensities
        // (hd_rad_const_kernel): C+ = (X^-1 s_top + Y^-1 d_top)/2, C- = (X^-1 s_bot -
        // Y^-1 d_bot)/2 with X^-1 = (L^-T V)^T diag(g), Y^-1 = -K^-1 (L V)^T diag(g):
        // one more product, B's columns 0/1 = g(s_top / s_bot) against L^-T V and
        // 2/3 = g(d_top / d_bot) against L V ----
        {
          const int side = c & 1;
          const double tsd = side ? taup : 0.0;
          const double ebs = exp(-tsd * rmu0);
          const double bt = rl(oBt, tt), slope = rl(oSl, tt);
          const double b2 = 2.0 * fma(slope, tsd, bt);
          const double* lv = A.lev + (size_t)(lc + side) * 2 * NN * nu + uml[tt];
          double bx[4], by[4];
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            const int r = h + 4 * s4;
            const bool in = r < NN && c < 4;
            const int rr_ = in ? r : 0;
            const double ipl = in ? lv[(size_t)rr_ * nu] : 0.0;
            const double imi = in ? lv[(size_t)(NN + rr_) * nu] : 0.0;
            const double zp = in ? rl(oZp + rr_, tt) : 0.0, zm = in ? rl(oZm + rr_, tt) : 0.0;
            const double hr = in ? rl(oH + rr_, tt) : 0.0;
            const double gr = Qc.g[rr_];
            bx[s4] = (in && c < 2) ? gr * (ipl + imi - (zp + zm) * ebs - b2) : 0.0;
            by[s4] = (in && c >= 2) ? gr * (ipl - imi - (zp - zm) * ebs - 2.0 * slope * hr) : 0.0;
          }
          d4 cacc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) cacc = __builtin_amdgcn_mfma_f64_16x16x4f64(gq[s4], bx[s4], cacc, 0, 0, 0);
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) cacc = __builtin_amdgcn_mfma_f64_16x16x4f64(p[s4], by[s4], cacc, 0, 0, 0);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int j = h + 4 * q;
            const double kj = j < NN ? rl(oK + (j < NN ? j : 0), tt) : 0.0;
            const double at_ = bc<0>(cacc[q]), ab_ = bc<1>(cacc[q]);
            const double bt_ = bc<2>(cacc[q]), bb_ = bc<3>(cacc[q]);
            cpl[q] = 0.5 * (at_ + (kj > 0.0 ? -bt_ / kj : 0.0));
            cmi[q] = 0.5 * (ab_ - (kj > 0.0 ? -bb_ / kj : 0.0));
            if (ab0 == 0 && v < A.nu && j < NN && c < 2)
              A.cst[((size_t)lc * 2 * NN + c * NN + j) * nu + v] = c ? cmi[q] : cpl[q];
          }
        }
        const double kc = c < NN ? rl(oK + (c < NN ? c : 0), tt) : 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = h + 4 * q;
          const double sdr = r < NN ? Qc.sd[r < NN ? r : 0] : 0.0;
          PT[q] = p[q] * sdr;
          QT[q] = gq[q] * (-kc * sdr);
        }
      }
      // ---- this lane's rows of the angle's c_e (c < 8) or c_o (c >= 8) column, and
      // its share of x0 = sum_l g_l Y_l^m(mu) Y_l^m(-mu0) ----
      double cu[4] = {0.0, 0.0, 0.0, 0.0};
      double xp = 0.0;
      {
        const int lpar = (m & 1) ^ fam;  // this lane's parity of l
        const double mub = beam ? mu0 : 0.0;
        const double sx0 = sqrt(fmax(0.0, 1.0 - mub * mub));
        const double* lam = rad_lam<NN>(m);
        double su = c_rtt.seed[m], s0v = su;
        for (int k = 0; k < m; ++k) {
          su *= sxu;
          s0v *= sx0;
        }
        double y1u = 0.0, y2u = 0.0, y10 = 0.0, y20 = 0.0;
        const double* q = qt[tt];
        const double f = ft[tt], rf = rft[tt];
#pragma nounroll
        for (int l2 = 0; l2 < NN; ++l2) {
          double yv = 0.0, y0v = 0.0;
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const int l = 2 * l2 + p;
            const double cra = c_rtt.ra[m][l], crb = c_rtt.rb[m][l];
            const double yu = l < m ? 0.0 : (l == m ? su : fma(cra * muu, y1u, -crb * y2u));
            const double y0 = l < m ? 0.0 : (l == m ? s0v : fma(cra * mub, y10, -crb * y20));
            y2u = y1u;
            y1u = yu;
            y20 = y10;
            y10 = y0;
            yv = p == lpar ? yu : yv;
            y0v = p == lpar ? y0 : y0v;
          }
          const int l = 2 * l2 + lpar;
          const double chi = l == 0 ? 1.0 : (l <= nmom ? q[1 + l] : 0.0);
          const double gl = (2 * l + 1) * (chi - f) * rf;
          const double gy = 0.5 * gl * yv;
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            const int r = h + 4 * s4;
            cu[s4] = fma(gy, r < NN ? lam[l * NN + (r < NN ? r : 0)] : 0.0, cu[s4]);
          }
          const double y0s = ((l + m) & 1) ? -y0v : y0v;
          xp = fma((l2 & 3) == h ? gl * yv : 0.0, y0s, xp);
        }
      }
      // ---- [ce | cx] = [P | Q] . blockdiag(C_e, C_o) on the matrix core ----
      d4 hacc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
        hacc = __builtin_amdgcn_mfma_f64_16x16x4f64(PT[s4], fam == 0 ? cu[s4] : 0.0, hacc, 0, 0, 0);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
        hacc = __builtin_amdgcn_mfma_f64_16x16x4f64(QT[s4], fam == 1 ? cu[s4] : 0.0, hacc, 0, 0, 0);
      // ---- this lane's four eigen-terms of the whole-layer integral; beam/thermal sums ----
      const double lmu = taup / anu;
      const double emu = exp(-lmu);
      double amp[4], kq[4];
      double lp = 0.0, sc = 0.0, th = 0.0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = h + 4 * q;
        const bool jok = j < NN;
        const int jj = jok ? j : 0;
        // lane c holds ce (c < 8) or cx (c >= 8) of angle c & 7; its partner c ^ 8 the other
        const double own = hacc[q];
        const double oth = xperm<8>(own);
        const double ce = fam ? oth : own, cx = fam ? own : oth;
        const double cc = jok ? (fam ? cmi[q] : cpl[q]) : 0.0;
        const double am = cc * (fam ? ce - cx : ce + cx);  // hpl_j (c < 8), hmi_j (c >= 8)
        const double kj = jok ? rl(oK + jj, tt) : 0.0;
        const double ek = jok ? rl(oEk + jj, tt) : 1.0;
        // hpl's +k family decays along upward rays, hmi's along downward ones; the
        // other meets 1 - k|mu| -> 0
        const bool dec = (fam == 0) == up;
        const double term = dec ? dexp(1.0, ek * emu, fma(kj, anu, 1.0), lmu)
                                : dexp(ek, emu, fma(-kj, anu, 1.0), lmu);
        lp = fma(am, term, lp);
        amp[q] = am;
        kq[q] = kj;
        const double wi = jok ? Qc.w[jj] : 0.0;
        const double zp = jok ? rl(oZp + jj, tt) : 0.0, zm = jok ? rl(oZm + jj, tt) : 0.0;
        const double hr = jok ? rl(oH + jj, tt) : 0.0;
        sc = fma(wi * cu[q], fam ? zp - zm : zp + zm, sc);
        th = fma(wi, cu[q] * (fam ? hr : 1.0), th);
      }
      {
        double* rp = red + a * 32 + h * 2 + fam;
        rp[0] = lp;
        rp[8] = sc;
        rp[16] = xp;
        rp[24] = th;
      }
      lds_fence();
      // ---- lanes 0..7, one per angle: team sums, the beam and thermal terms; lay -> rsw ----
      if (lane < 8) {
        const int iv = ab0 + lane;
        const double* rp = red + lane * 32;
        double lay = 0.0, scs = 0.0, x0 = 0.0, we = 0.0, wo = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          lay += rp[k];
          scs += rp[8 + k];
          x0 += rp[16 + k];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          we += rp[24 + 2 * k];
          wo += rp[25 + 2 * k];
        }
        const double mv = iv < A.numu ? A.umu[iv] : 1.0;
        const bool upv = mv > 0.0;
        const double av = fabs(mv);
        const double lmv = taup / av;
        const double emv = exp(-lmv);
        double ab = 0.0, a0 = 0.0, a1t = 0.0;
        if (beam) {
          const double fac = (m == 0 ? 1.0 : 2.0) * fb / (4.0 * kPi);
          ab = fma(fac * x0, exp(-A.tauc[(size_t)lc * A.ns + sl] * rmu0), scs);
          const double e0l = rl(oE0, tt);
          lay += upv ? ab * (1.0 - e0l * emv) / fma(av, rmu0, 1.0)
                     : ab * dexp(e0l, emv, fma(-av, rmu0, 1.0), lmv);
        }
        if (therm) {
          const double* q = qt[tt];
          double ssa = A.nprop > 1 ? q[1] : 0.0;
          if (ssa == 1.0) ssa = 1.0 - kDither;
          const double f = ft[tt];
          const double om = ssa * (1.0 - f) / (1.0 - ssa * f);
          const double bt = rl(oBt, tt), slope = rl(oSl, tt);
          const double ce0 = (1.0 - om) + 2.0 * we;
          a1t = slope * ce0;
          a0 = fma(bt, ce0, 2.0 * slope * wo);
          lay += upv ? (a0 + a1t * mv) - (a0 + a1t * taup + a1t * mv) * emv
                     : (a0 + a1t * taup + a1t * mv) - (a0 + a1t * mv) * emv;
        }
        if (iv < A.numu && v < A.nu) A.rsw[((size_t)lc * nu + v) * NE1 + iv] = lay;
        double* ap = aux + lane * 4;
        ap[0] = ab;
        ap[1] = a0;
        ap[2] = a1t;
      }
      lds_fence();
      // ---- user depths inside the layer: the partial integral from the depth to the
      // ray's entry (the scan adds the entry value's attenuated share) ----
      {
        const double ttop = A.taus[(size_t)lc * A.ns + sl];
        const double tbot = A.taus[(size_t)(lc + 1) * A.ns + sl];
        const double tau = tbot - ttop;
        const double scale = tau > 0.0 ? taup / tau : 0.0;
        // candidates: the caller's depths, or the layer's two levels -- whose scaled
        // depth (tbot - ttop) tau'/tau can miss tau' by an ulp, and the scan then
        // takes the interior branch for them as hd_rad_user_kernel does
        const int k0 = A.utau ? 0 : lc, k1 = A.utau ? A.ntau : lc + 2;
        for (int k = k0; k < k1; ++k) {
          const double tu = user_tau(A, k, sl);
          if (tu < ttop || tu > tbot) continue;  // uniform
          const double tl = fmin(fmax((tu - ttop) * scale, 0.0), taup);
          // the depth's layer along this ray: hd_rad_team_user_scan_kernel's walk
          const bool mine = up ? (tu >= ttop && (lc == L - 1 || tu < tbot))
                               : (tu <= tbot && (lc == 0 || tu > ttop));
          const double tin = up ? taup : 0.0;
          const bool need = aok && mine && tl != tin && tl != taup - tin;
          if (!__any(need)) continue;  // uniform
          double r = 0.0;
          if (need) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
              r += seg_exp(amp[q], fam ? -kq[q] : kq[q], tl, tin, fam ? taup : 0.0, muu);
          }
          red2[a * 8 + h * 2 + fam] = r;
          lds_fence();
          if (lane < 8 && ab0 + lane < A.numu && v < A.nu) {
            const int iv = ab0 + lane;
            const double mv = A.umu[iv];
            const bool upv = mv > 0.0;
            const bool minev = upv ? (tu >= ttop && (lc == L - 1 || tu < tbot))
                                   : (tu <= tbot && (lc == 0 || tu > ttop));
            const double tinv = upv ? taup : 0.0;
            if (minev && tl != tinv && tl != taup - tinv) {
              double rs = 0.0;
#pragma unroll
              for (int k2 = 0; k2 < 8; ++k2) rs += red2[lane * 8 + k2];
              const double* ap = aux + lane * 4;
              if (beam) rs += seg_exp(ap[0], rmu0, tl, tinv, 0.0, mv);
              if (therm) {
                const double e2 = exp(-(tinv - tl) / mv);
                rs += (ap[1] + ap[2] * tl + ap[2] * mv) - (ap[1] + ap[2] * tinv + ap[2] * mv) * e2;
              }
              A.radm[((size_t)k * A.numu + iv) * nu + v] = rs;
            }
          }
          lds_fence();
        }
      }
    });
  }
}

template <int NN>
__global__ __launch_bounds__(256) void hd_rad_team_user_scan_kernel(RadArgs A) {
  constexpr int nsym = NN * (NN + 1) / 2;
  constexpr int NE1 = rad_layer_record_doubles(NN);
  constexpr int NR = rad_rec_doubles(NN);
  constexpr int oTp = nsym + NN * NN + 4 * NN + 2;
  const Quad<NN>& Qc = tquad<NN>(c_qt);
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nu = A.nu;
  if (id >= (long)nu * A.numu) return;
  const int iu = (int)(id / (long)nu);
  const int u = (int)(id - (long)iu * (long)nu);  // unit fastest: coalesced records
  const int m = u / A.ns;
  const int sl = u - m * A.ns;
  const long s = A.s0 + sl;
  const int L = A.nlyr;
  const double muu = A.umu[iu];
  const bool up = muu > 0.0;
  const double anu = fabs(muu);
  const double mu0 = A.umu0 ? A.umu0[s] : 1.0;
  const double fb = A.fbeam ? A.fbeam[s] : 0.0;
  const bool beam = fb > 0.0 && mu0 > 0.0;
  const double rmu0 = beam ? 1.0 / mu0 : 0.0;
  double cur = 0.0;
  if (m == 0) {
    if (up) {
      const double* lv = A.lev + (size_t)L * 2 * NN * nu + u;
      double fdn = 0.0;
      for (int i = 0; i < NN; ++i) fdn = fma(Qc.g[i] * Qc.g[i], lv[(NN + i) * nu], fdn);
      fdn *= 2.0 * kPi;
      const double alb = A.albedo ? A.albedo[s] : 0.0;
      if (beam) {
        const double tb = A.tauc[(size_t)(L - 1) * A.ns + sl] +
                          A.rrd[((size_t)(L - 1) * nu + u) * NR + oTp];
        fdn += fb * mu0 * exp(-tb * rmu0);
      }
      cur = alb / kPi * fdn + (A.planck ? (1.0 - alb) * A.planckv[(size_t)(L + 1) * A.ns + sl]
                                        : 0.0);
    } else {
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
    const double taup = A.rrd[((size_t)lc * nu + u) * NR + oTp];
    const double emu = exp(-(taup / anu));
    const double lay = A.rsw[((size_t)lc * nu + u) * NE1 + iu];
    const double cin = cur;
    const double cout = fma(cin, emu, lay);
    const double tau = tbot - ttop;
    const double scale = tau > 0.0 ? taup / tau : 0.0;
    const double tin = up ? taup : 0.0;
    auto put = [&](int kk) {
      const double t = fmin(fmax((user_tau(A, kk, sl) - ttop) * scale, 0.0), taup);
      double* o = A.radm + ((size_t)kk * A.numu + iu) * nu + u;
      const double val = t == tin ? cin
                       : t == taup - tin ? cout
                       : fma(cin, exp(-fabs(tin - t) / anu), *o);  // *o: the partial integral
      *o = val;
      chk += val;
    };
    if (up) {
      while (k >= 0 && user_tau(A, k, sl) >= ttop) put(k--);
    } else {
      while (k < A.ntau && user_tau(A, k, sl) <= tbot) put(k++);
    }
    cur = cout;
  }
  for (; k < A.ntau && !up; ++k) A.radm[((size_t)k * A.numu + iu) * nu + u] = cur;
  if (!isfinite(chk)) {
    atomicOr(&A.status[s], kStNonFinite);
    atomicOr(A.anyerr, 1);
  }
}

template <int NN>
static hipError_t launch_rad_user(const RadArgs& a, hipStream_t stream) {
  const unsigned nb = (unsigned)(((a.nu + 3) / 4) * (long)a.nlyr);
  hipLaunchKernelGGL(hd_rad_team_user_kernel<NN>, dim3(nb), dim3(64), 0, stream, a);
  const long nr = (long)a.nu * a.numu;
  hipLaunchKernelGGL(hd_rad_team_user_scan_kernel<NN>, dim3((unsigned)((nr + 255) / 256)),
                     dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_rad_team_user(int nn, const RadArgs& a, hipStream_t stream) {
  if (a.numu > rad_layer_record_doubles(nn)) return hipErrorInvalidValue;
  switch (nn) {
    case 9: return launch_rad_user<9>(a, stream);
    case 10: return launch_rad_user<10>(a, stream);
    case 11: return launch_rad_user<11>(a, stream);
    case 12: return launch_rad_user<12>(a, stream);
    case 13: return launch_rad_user<13>(a, stream);
    case 14: return launch_rad_user<14>(a, stream);
    case 15: return launch_rad_user<15>(a, stream);
    case 16: return launch_rad_user<16>(a, stream);
    default: return hipErrorInvalidValue;
  }
}

template <int NN>
static hipError_t launch_rad_sweep(const RadArgs& a, hipStream_t stream) {
  hipLaunchKernelGGL(hd_rad_team_sweep_kernel<NN>, dim3((unsigned)((a.nu + 3) / 4)), dim3(64), 0,
                     stream, a);
  return hipGetLastError();
}

hipError_t launch_rad_team_sweep(int nn, const RadArgs& a, hipStream_t stream) {
  switch (nn) {
    case 9: return launch_rad_sweep<9>(a, stream);
    case 10: return launch_rad_sweep<10>(a, stream);
    case 11: return launch_rad_sweep<11>(a, stream);
    case 12: return launch_rad_sweep<12>(a, stream);
    case 13: return launch_rad_sweep<13>(a, stream);
    case 14: return launch_rad_sweep<14>(a, stream);
    case 15: return launch_rad_sweep<15>(a, stream);
    case 16: return launch_rad_sweep<16>(a, stream);
    default: return hipErrorInvalidValue;
  }
}


template <int NN>
static hipError_t launch_rad_layer(const RadArgs& a, hipStream_t stream) {
  const unsigned nb = (unsigned)(((a.nu + 3) / 4) * (long)a.nlyr);
  hipLaunchKernelGGL(hd_rad_team_layer_kernel<NN>, dim3(nb), dim3(64), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_rad_team_layer(int nn, const RadArgs& a, hipStream_t stream) {
  switch (nn) {
    case 9: return launch_rad_layer<9>(a, stream);
    case 10: return launch_rad_layer<10>(a, stream);
    case 11: return launch_rad_layer<11>(a, stream);
    case 12: return launch_rad_layer<12>(a, stream);
    case 13: return launch_rad_layer<13>(a, stream);
    case 14: return launch_rad_layer<14>(a, stream);
    case 15: return launch_rad_layer<15>(a, stream);
    case 16: return launch_rad_layer<16>(a, stream);
    default: return hipErrorInvalidValue;
  }
}

template <int NN>
static void fill_rad_team(RadTabTeam<NN>& t, const QuadHost& h) {
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

// the Y_l^m tables of the team intensity kernels (hd_rad.hip's recurrence); called
// once per device under hd_api.cpp's global table lock
hipError_t upload_rad_tables_team(const QuadHost* per_nn) {
  static RadTabsTeam c;  // ~570 KB: keep off the stack
  fill_rad_team<9>(c.t9, per_nn[8]);
  fill_rad_team<10>(c.t10, per_nn[9]);
  fill_rad_team<11>(c.t11, per_nn[10]);
  fill_rad_team<12>(c.t12, per_nn[11]);
  fill_rad_team<13>(c.t13, per_nn[12]);
  fill_rad_team<14>(c.t14, per_nn[13]);
  fill_rad_team<15>(c.t15, per_nn[14]);
  fill_rad_team<16>(c.t16, per_nn[15]);
  for (int m = 0; m < 2 * kMaxNN; ++m) {
    double sd = 1.0;
    for (int a = 1; a <= m; ++a) sd *= std::sqrt((2.0 * a - 1) / (2.0 * a));
    c.seed[m] = sd;
    for (int l = 0; l < 2 * kMaxNN; ++l) {
      if (l > m) {
        const double den = std::sqrt((double)l * l - (double)m * m);
        c.ra[m][l] = (2.0 * l - 1) / den;
        c.rb[m][l] = std::sqrt((double)(l - 1) * (l - 1) - (double)m * m) / den;
      } else {
        c.ra[m][l] = c.rb[m][l] = 0.0;
      }
    }
  }
  return hipMemcpyToSymbol(HIP_SYMBOL(c_rtt), &c, sizeof(RadTabsTeam), 0, hipMemcpyHostToDevice);
}

}  // namespace hd
