// hd_team.hip -- gfx950 kernels of the flux-only discrete-ordinate solve for
// nstr 18..32 (NN = nstr/2 in 9..16), where one problem's NN x NN matrices no
// longer fit one lane's registers.
//
//   hd_team_layer_kernel<NN>  one 16-lane team per (solve, layer): the same
//                             per-layer setup as hd_layer_kernel (delta-M,
//                             phase-matrix assembly, Cholesky + Jacobi
//                             symmetric eigenproblem, beam/thermal particular
//                             solutions, R~/T~/S~ in the flux-weighted basis;
//                             DESIGN.md section 3)        [c_setdis, c_soleig,
//                             c_upbeam, c_upisot]
//   hd_team_sweep_kernel<NN>  one team per solve: adding sweep top->bottom,
//                             Lambertian surface, back-substitution, level
//                             fluxes in harp layout     [c_setmtx, c_solve0,
//                             c_fluxes]
//
// Team layout: a team is one DPP row (16 lanes of a wave64); lane i owns row i
// of every NN x NN matrix and element i of every vector (lanes i >= NN carry
// zeros).  All cross-lane traffic is DPP inside the row -- row_newbcast:k
// (one v_mov_b64_dpp) hands lane k's value to the whole team, row_ror and the
// quad/half/full mirrors give the XOR permutations of the parallel Jacobi
// ordering and the team sums.  No LDS, no barriers: a team is always wholly
// active or wholly inactive, so every DPP source lane is live.
//
// Scratch records, solve-major inside a layer (a team's record is contiguous):
//   layer ops [lc][s][2NN^2+2NN+2]  R~ rows | T~ rows | S~+ | S~- | tau' | pad
//   back-sub  [lc][s][NN^2+2NN+1 -> even]  ZT rows | t | rc | cs | pad
#include <cstdlib>
#include <cstring>

#include "hd_team_prims.hpp"

namespace hd {

namespace {
__constant__ QuadTablesTeam c_quad_team;
}  // namespace

using namespace team;

#if HD_AB_VARIANTS  // the VALU team kernels: A/B build only (the product runs hd_team_mfma.hip)
// ============================================================================
// K1 (team): per-(solve, layer) setup
// ============================================================================
template <int NN>
__global__ __launch_bounds__(kTeamBlock) void hd_team_layer_kernel(LayerArgs A) {
  __shared__ double tr_lds[kTeamsPerBlock * kTeam * (kTeam + 1)];  // 16 transpose tiles
  constexpr int N = 2 * NN;
  const Quad<NN>& Qc = tquad<NN>(c_quad_team);
  const int i = tlane();
  const bool act = i < NN;
  const int ii = act ? i : 0;
  const long team = (long)blockIdx.x * kTeamsPerBlock + (threadIdx.x >> 4);
  const int L = A.nlyr;
  if (team >= (long)A.nsc * L) return;  // whole team
  // consecutive teams = consecutive solves of one layer -> contiguous records
  const int sl = (int)(team % A.nsc);
  const int lc = (int)(team / A.nsc);
  const long s = A.s0 + sl;
  const int nm = A.nmom;
  const int np = A.nprop;
  int st = 0;

  // lanes >= NN carry zeros; masks are arithmetic (x * msk on clamped, finite
  // loads) rather than selects around loads, which cost registers at NN < 16
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

  // ---- phase-matrix rows: -A+ (ap), -A- (lch); beam source elements ----
  double ap[NN], lch[NN];
  double xs = 0.0, xd = 0.0;
  sfor<0, NN>([&](auto J) { ap[HD_K(J)] = lch[HD_K(J)] = 0.0; });
  {
    double pprev = 0.0, pcur = 1.0;
#pragma nounroll
    for (int l2 = 0; l2 < NN; ++l2) {
      const int le = 2 * l2, lo = le + 1;
      const double che = le == 0 ? 1.0 : (le <= nm ? q[1 + le] : 0.0);
      const double cho = lo <= nm ? q[1 + lo] : 0.0;
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
  // L L^T = -A-
  double lt[NN], rdl;
  if (!team_chol<NN, true>(lch, lt, rdl)) st |= kStEigen;

  // ---- pre-Jacobi vectors (depend on L only) ----
  double y2 = 0.0, lxd = 0.0;
  const double fb2 = fb * (0.5 / kPi);
  if (beam) {
    const double y = sd_i * (fb2 * xs);
    double z = 0.0;  // z = L^T y
    sfor<0, NN>([&](auto K) { z = fma(lt[HD_K(K)], bc<HD_K(K)>(y), z); });
    double yl = 0.0;  // L z
    sfor<0, NN>([&](auto K) { yl = fma(lch[HD_K(K)], bc<HD_K(K)>(z), yl); });
    const double xdi = -fb2 * xd;
    const double rv = fma(-yl, rg_i, xdi * rmu0 * rmu_i);
    y2 = g_i * rv;
    lxd = sd_i * xdi;
    team_lsolve<NN>(lch, rdl, y2);
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

  // ---- eigenpairs (c_soleig): Sym = L^T (-A+) L = V diag(k^2) V^T ----
  // With C C^T = -A+ (SPD because Sym is), Sym = B^T B for B = C^T L; the
  // one-sided Jacobi on B's columns yields k^2 = |b_j|^2 and B = B0 V, so
  // U = L V = C^-T B and V = L^-1 U.  Each of V, V^T y2 and U is consumed as
  // soon as it exists (V rows -> Psi^T rows, then the beam, then U rows ->
  // Omega rows), which keeps the live set to one team row-set at a time.
  double kk;        // lane j: k_j
  double pst[NN];   // lane i: row i of Psi^T = L^-T V Gamma^1/2
  double omr[NN];   // lane i: row i of Omega = U Delta^1/2
  double zp = 0.0, zm = 0.0, e0 = 0.0;
  {
    double unused[NN], rdc;
    if (!team_chol<NN, false>(ap, unused, rdc)) st |= kStEigen;  // ap <- rows of C
    double bcol[NN];  // lane j: B_ij = sum_k C_ki L_kj
    sfor<0, NN>([&](auto I) {
      constexpr int r = HD_K(I);
      double t = 0.0;
      sfor<r, NN>([&](auto K) { t = fma(bc<HD_K(K)>(ap[r]), lt[HD_K(K)], t); });
      bcol[r] = t;
    });
    if (!team_jacobi<NN>(bcol, A.max_sweeps)) st |= kStEigen;
    double k2 = 0.0;
    sfor<0, NN>([&](auto K) { k2 = fma(bcol[HD_K(K)], bcol[HD_K(K)], k2); });
    if (act && !(k2 > 0.0)) st |= kStEigen;
    kk = sqrt(k2 > 0.0 ? k2 : 0.0) * msk;
    // Delta = tanh(k tau'/2)/k, Gamma = k tanh(k tau'/2) (lane j)
    double dsq, gsq;
    {
      const double x = kk * taup;
      const double m = -expm1(-x);
      const double th = m * rcp_nr(2.0 - m);
      const double delta = x > 1.0e-8 ? th * rcp_nr(kk > 0.0 ? kk : 1.0) : 0.5 * taup;
      dsq = sqrt(delta);
      gsq = sqrt(kk * th);
    }
    // columns (lane j) of U = C^-T b_j and V = L^-1 U: lane-local solves with
    // the matrix entries broadcast
    sfor_rev<0, NN>([&](auto I) {  // C^T y = b
      constexpr int r = HD_K(I);
      double t = bcol[r];
      sfor<r + 1, NN>([&](auto K) { t = fma(-bc<HD_K(K)>(ap[r]), bcol[HD_K(K)], t); });
      bcol[r] = t * bc<r>(rdc) * msk;
    });
    double vt[NN];  // lane j: column j of V (row j of V^T)
    sfor<0, NN>([&](auto I) {  // L x = y
      constexpr int r = HD_K(I);
      double t = bcol[r];
      sfor<0, r>([&](auto K) { t = fma(-bc<r>(lch[HD_K(K)]), vt[HD_K(K)], t); });
      vt[r] = t * bc<r>(rdl) * msk;
    });
    // rows of V and U: transposes through this team's LDS tile (a team lives
    // in one wave and LDS operations of a wave complete in order, so no
    // barrier; the row stride kTeam+1 keeps both passes conflict-free)
    double* tile = tr_lds + (threadIdx.x >> 4) * (kTeam * (kTeam + 1));
    sfor<0, NN>([&](auto I) { tile[HD_K(I) * (kTeam + 1) + i] = vt[HD_K(I)]; });
    __builtin_amdgcn_wave_barrier();
    sfor<0, NN>([&](auto J) {
      pst[HD_K(J)] = tile[ii * (kTeam + 1) + HD_K(J)] * msk * bc<HD_K(J)>(gsq);
    });
    __builtin_amdgcn_wave_barrier();
    team_umsolve<NN>(lt, rdl, pst);  // Psi^T rows = L^-T V Gamma^1/2
    // ---- beam particular solution Z+/- (c_upbeam) ----
    double tt = 0.0;  // lane j: (V^T y2)_j / (1/mu0^2 - k_j^2)
    if (beam) {
      const double r2 = rmu0 * rmu0;
      double t = 0.0;
      sfor<0, NN>([&](auto K) { t = fma(vt[HD_K(K)], bc<HD_K(K)>(y2), t); });
      double den = fma(-kk, kk, r2);
      if (act && fabs(den) < 1.0e-9 * r2) {
        st |= kStResonance;
        den = den < 0.0 ? -1.0e-9 * r2 : 1.0e-9 * r2;
      }
      tt = t / den * msk;
    }
    sfor<0, NN>([&](auto I) { tile[HD_K(I) * (kTeam + 1) + i] = bcol[HD_K(I)]; });
    __builtin_amdgcn_wave_barrier();
    double u[NN];  // lane i: row i of U
    sfor<0, NN>([&](auto J) { u[HD_K(J)] = tile[ii * (kTeam + 1) + HD_K(J)] * msk; });
    __builtin_amdgcn_wave_barrier();
    if (beam) {
      double sv = 0.0;  // W^-1 D^1/2 L V tt = W^-1 D^1/2 U tt
      sfor<0, NN>([&](auto J) { sv = fma(u[HD_K(J)], bc<HD_K(J)>(tt), sv); });
      sv *= rg_i;
      double yy = sd_i * mu_i * sv;
      team_lsolve<NN>(lch, rdl, yy);
      team_usolve<NN>(lt, rdl, yy);
      // tauc null: sources for a unit beam at the layer top (the sweep scales them)
      const double tauc = A.tauc ? A.tauc[(size_t)lc * A.nsc + sl] : 0.0;
      const double att = 0.5 * exp(-tauc * rmu0);
      const double dd = rg_i * fma(-yy, rmu0, lxd);
      zp = (sv + dd) * att;
      zm = (sv - dd) * att;
      e0 = exp(-taup * rmu0);
    }
    // ---- layer operators in the flux-weighted basis: Omega rows ----
    sfor<0, NN>([&](auto J) { omr[HD_K(J)] = u[HD_K(J)] * bc<HD_K(J)>(dsq); });
  }
  const double ga = g_i * (cvec - fma(-zp, e0, zm));
  const double gb = g_i * (fma(zp, e0, zm) + bsum);
  // By Woodbury, Q~- = I - A- and Q~+ = A+ - I with A- = (I + Omega Omega^T)^-1,
  // A+ = (I + Psi^T Psi)^-1 (SPD, eigenvalues in (0, 1]); lane i gets row i of
  // each inverse from the Cholesky rows J by two lane-local triangular solves
  // with broadcast J entries:  z J^T = e_i, then a J = z  (a = e_i (J J^T)^-1).
  double am_[NN], ap_[NN];
  auto spd_inverse_row = [&](double (&h)[NN], double (&arow)[NN]) {
    double unused[NN], jrd;
    if (!team_chol<NN, false>(h, unused, jrd)) st |= kStEigen;  // h <- row i of J
    double z[NN];
    sfor<0, NN>([&](auto R) {
      constexpr int r = HD_K(R);
      double t = i == r ? 1.0 : 0.0;
      sfor<0, r>([&](auto K) { t = fma(-bc<r>(h[HD_K(K)]), z[HD_K(K)], t); });
      z[r] = t * bc<r>(jrd);
    });
    // both solves broadcast the same J entries; without this the compiler
    // would keep all NN(NN-1)/2 broadcast values live from one solve to the next
#pragma unroll
    for (int k = 0; k < NN; ++k) asm volatile("" : "+v"(h[k]));
    asm volatile("" : "+v"(jrd));
    sfor_rev<0, NN>([&](auto C) {
      constexpr int c = HD_K(C);
      double t = z[c];
      sfor<c + 1, NN>([&](auto K) { t = fma(-arow[HD_K(K)], bc<HD_K(K)>(h[c]), t); });
      arow[c] = t * bc<c>(jrd);
    });
  };
  {
    double hm[NN];  // row i of I + Omega Omega^T
    sfor<0, NN>([&](auto J) {
      constexpr int j = HD_K(J);
      double t = i == j ? 1.0 : 0.0;
      sfor<0, NN>([&](auto K) { t = fma(omr[HD_K(K)], bc<j>(omr[HD_K(K)]), t); });
      hm[j] = t;
    });
    spd_inverse_row(hm, am_);
  }
  {
    double hp[NN];  // row i of I + Psi^T Psi
    sfor<0, NN>([&](auto J) {
      constexpr int j = HD_K(J);
      double t = i == j ? 1.0 : 0.0;
      sfor<0, NN>([&](auto K) { t = fma(pst[HD_K(K)], bc<j>(pst[HD_K(K)]), t); });
      hp[j] = t;
    });
    spd_inverse_row(hp, ap_);
  }
  double pv = ga, qv = -gb;  // Q~- ga = ga - A- ga,  Q~+ gb = A+ gb - gb
  sfor<0, NN>([&](auto J) {
    constexpr int j = HD_K(J);
    pv = fma(-am_[j], bc<j>(ga), pv);
    qv = fma(ap_[j], bc<j>(gb), qv);
  });

  // ---- store: R~ = A+ - A-, T~ = A- + A+ - I (rows), S~+, S~-, tau' ----
  // lanes >= NN store into a sink instead of branching around the stores (a
  // branch here costs the whole kernel's register allocation at NN < 16)
  double* rec = A.scr + ((size_t)lc * A.nsc + sl) * ne1t<NN>();
  double* out = act ? rec : A.sink;
  double chk = 0.0;
  sfor<0, NN>([&](auto J) {
    constexpr int j = HD_K(J);
    const double r = ap_[j] - am_[j];
    const double t = (am_[j] + ap_[j]) - (i == j ? 1.0 : 0.0);
    out[ii * NN + j] = r;
    out[NN * NN + ii * NN + j] = t;
    chk += r + t;
  });
  const double sp = g_i * (zp * (1.0 - e0) - db) + pv - qv;
  const double sm = g_i * (-zm * (1.0 - e0) + db) - pv - qv;
  out[2 * NN * NN + ii] = sp;
  out[2 * NN * NN + NN + ii] = sm;
  chk += sp + sm;
  if (i == 0) rec[2 * NN * NN + 2 * NN] = taup;
  if (act && !isfinite(chk + taup)) st |= kStNonFinite;
  if (st) {
    atomicOr(&A.status[s], st);
    if (st & 0x0F) atomicOr(A.anyerr, 1);
  }
}

// ============================================================================
// K2 (team): per-solve adding sweep + back-substitution
// ============================================================================
template <int NN>
__global__ __launch_bounds__(kTeamBlock) void hd_team_sweep_kernel(SweepArgs A) {
  const Quad<NN>& Qc = tquad<NN>(c_quad_team);
  const int i = tlane();
  const bool act = i < NN;
  const int ii = act ? i : 0;
  const long team = (long)blockIdx.x * kTeamsPerBlock + (threadIdx.x >> 4);
  if (team >= A.nsc) return;  // whole team
  const int sl = (int)team;
  const long s = A.s0 + sl;
  const int L = A.nlyr;
  const size_t nsc = A.nsc;
  int st = 0;
  const double msk = act ? 1.0 : 0.0;  // arithmetic lane mask (see the layer kernel)
  const double g_i = Qc.g[ii] * msk;

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

  double ra[NN];  // reflection of the stack above (row i)
  double sd = g_i * top;  // diffuse downward source at the current interface
  sfor<0, NN>([&](auto J) { ra[HD_K(J)] = 0.0; });
  double tauc = 0.0;

  for (int lc = 0; lc < L; ++lc) {
    const double* rec = A.scr + ((size_t)lc * nsc + sl) * ne1t<NN>();
    double* bp = A.bsub + ((size_t)lc * nsc + sl) * ne2t<NN>();
    double* bw = act ? bp : A.sink;  // lanes >= NN store into the sink (no branches)
    double rl[NN];
    sfor<0, NN>([&](auto J) { rl[HD_K(J)] = rec[ii * NN + HD_K(J)] * msk; });
    // direct beam at the layer top; a unit-beam record's sources scale with it
    const double eb = exp(-tauc * rmu0);
    const double sscale = A.beam_scale ? eb : 1.0;
    const double spl = rec[2 * NN * NN + ii] * msk * sscale;
    const double sml = rec[2 * NN * NN + NN + ii] * msk * sscale;

    // level lc (top of layer lc): F_dn = rc . I+ + cs
    {
      double t = 0.0;
      sfor<0, NN>([&](auto J) { t = fma(ra[HD_K(J)], Qc.g[HD_K(J)], t); });
      bw[NN * NN + NN + ii] = twopi * t;
      const double cs = team_sum(g_i * sd);
      if (i == 0) bp[NN * NN + 2 * NN] = fma(twopi, cs, f0mu0 * eb);
    }
    // W1 = I - R_l A ; t1 = R_l Sd + S+
    double w[NN];
    sfor<0, NN>([&](auto J) {
      constexpr int j = HD_K(J);
      double t = i == j ? 1.0 : 0.0;
      sfor<0, NN>([&](auto K) { t = fma(-rl[HD_K(K)], bc<HD_K(K)>(ra[j]), t); });
      w[j] = t;
    });
    double t1 = spl;
    sfor<0, NN>([&](auto K) { t1 = fma(rl[HD_K(K)], bc<HD_K(K)>(sd), t1); });
    // LU without pivoting; reciprocal pivots on the diagonal
    sfor<0, NN>([&](auto K) {
      constexpr int k = HD_K(K);
      const double piv = bc<k>(w[k]);
      if (!(fabs(piv) > 1.0e-12)) st |= kStPivot;
      const double rp = rcp_nr(piv);
      const double lik = w[k] * rp;
      const double m = i > k ? lik : 0.0;
      w[k] = i == k ? rp : (i > k ? lik : w[k]);
      sfor<k + 1, NN>([&](auto J) {
        constexpr int j = HD_K(J);
        w[j] = fma(-m, bc<k>(w[j]), w[j]);
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
    // M1 = A W1^-1 (row-local): z U = a, then x L = z
    double am[NN];
    sfor<0, NN>([&](auto J) {
      constexpr int j = HD_K(J);
      double t = ra[j];
      sfor<0, j>([&](auto K) { t = fma(-am[HD_K(K)], bc<HD_K(K)>(w[j]), t); });
      am[j] = t * bc<j>(w[j]);
    });
    sfor_rev<0, NN>([&](auto J) {
      constexpr int j = HD_K(J);
      double t = am[j];
      sfor<j + 1, NN>([&](auto K) { t = fma(-am[HD_K(K)], bc<HD_K(K)>(w[j]), t); });
      am[j] = t;
    });
    // T~ rows; ZT = W1^-1 T (row-sequential solves)
    double tr[NN], zt[NN];
    sfor<0, NN>([&](auto J) {
      constexpr int j = HD_K(J);
      tr[j] = rec[NN * NN + ii * NN + j] * msk;
      zt[j] = tr[j];
    });
    sfor<0, NN>([&](auto K) {
      constexpr int k = HD_K(K);
      const double m = i > k ? w[k] : 0.0;
      sfor<0, NN>([&](auto J) { zt[HD_K(J)] = fma(-m, bc<k>(zt[HD_K(J)]), zt[HD_K(J)]); });
    });
    sfor_rev<0, NN>([&](auto K) {
      constexpr int k = HD_K(K);
      const double sc = i == k ? w[k] : 1.0;
      sfor<0, NN>([&](auto J) { zt[HD_K(J)] *= sc; });
      const double m = i < k ? w[k] : 0.0;
      sfor<0, NN>([&](auto J) { zt[HD_K(J)] = fma(-m, bc<k>(zt[HD_K(J)]), zt[HD_K(J)]); });
    });
    sfor<0, NN>([&](auto J) { bw[ii * NN + HD_K(J)] = zt[HD_K(J)]; });
    // P = M1 T ; Ra <- R_l + T P ; Sd <- T u + S-
    double pm[NN];
    sfor<0, NN>([&](auto J) {
      constexpr int j = HD_K(J);
      double t = 0.0;
      sfor<0, NN>([&](auto K) { t = fma(am[HD_K(K)], bc<HD_K(K)>(tr[j]), t); });
      pm[j] = t;
    });
    sfor<0, NN>([&](auto J) {
      constexpr int j = HD_K(J);
      double t = rl[j];
      sfor<0, NN>([&](auto K) { t = fma(tr[HD_K(K)], bc<HD_K(K)>(pm[j]), t); });
      ra[j] = t;
    });
    {
      double t = sml;
      sfor<0, NN>([&](auto K) { t = fma(tr[HD_K(K)], bc<HD_K(K)>(u), t); });
      sd = t;
    }
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
  // flux_local: the band epilogue's chunk buffer (hd_solve_band without per-point fluxes)
  double* fo = A.flux + (size_t)(A.flux_local ? (long)sl : s) * (L + 1) * 2;
  double chk = 0.0;
  {
    const double up = team_sum(g_i * ip);
    const double dn = team_sum(g_i * fma(rgrow, x, sd));
    if (i == 0) {
      fo[0] = twopi * up;
      fo[1] = twopi * dn + dirsurf;
      chk += fo[0] + fo[1];
    }
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
    if (i == 0) {
      const int lev = L - lc;
      fo[2 * lev] = twopi * up;
      fo[2 * lev + 1] = bp[NN * NN + 2 * NN] + dn;
      chk += fo[2 * lev] + fo[2 * lev + 1];
    }
  }
  if (!isfinite(chk)) st |= kStNonFinite;
  if (st) {
    atomicOr(&A.status[s], st);
    if (st & 0x0F) atomicOr(A.anyerr, 1);
  }
}

#endif  // HD_AB_VARIANTS

// ============================================================================
// host side
// ============================================================================
template <int NN>
static void fill_quad_team(Quad<NN>& q, const QuadHost& h) {
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

void fill_quad_tables_team(const QuadHost* per_nn, QuadTablesTeam& t) {
  fill_quad_team<9>(t.q9, per_nn[8]);
  fill_quad_team<10>(t.q10, per_nn[9]);
  fill_quad_team<11>(t.q11, per_nn[10]);
  fill_quad_team<12>(t.q12, per_nn[11]);
  fill_quad_team<13>(t.q13, per_nn[12]);
  fill_quad_team<14>(t.q14, per_nn[13]);
  fill_quad_team<15>(t.q15, per_nn[14]);
  fill_quad_team<16>(t.q16, per_nn[15]);
}

hipError_t upload_quad_tables_team(const QuadHost* per_nn /* [kMaxNN], index nn-1 */) {
  QuadTablesTeam t;
  fill_quad_tables_team(per_nn, t);
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_quad_team), &t, sizeof(t), 0, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = upload_quad_tables_team_mfma(t);
  return e;
}

// HD_TEAM_LAYER=valu selects the VALU-product layer kernel (A/B runs); the
// default is the MFMA one (hd_team_mfma.hip)
static bool team_layer_valu() {
#if HD_AB_VARIANTS
  static const bool v = [] {
    const char* e = ab_env("HD_TEAM_LAYER");
    return e && std::strcmp(e, "valu") == 0;
  }();
  return v;
#else
  return false;
#endif
}

// HD_TEAM_SWEEP=valu selects the VALU-product sweep (A/B runs); the default is
// the MFMA one (hd_team_mfma.hip)
static bool team_sweep_valu() {
#if HD_AB_VARIANTS
  static const bool v = [] {
    const char* e = ab_env("HD_TEAM_SWEEP");
    return e && std::strcmp(e, "valu") == 0;
  }();
  return v;
#else
  return false;
#endif
}

template <int NN>
static hipError_t launch_team(const PlanckArgs* pa, const TaucArgs* ta, const LayerArgs& la,
                              const SweepArgs& sa, hipStream_t stream, hipEvent_t* ev) {
  static_assert(ne1t<NN>() % 2 == 0 && ne2t<NN>() % 2 == 0, "16-byte aligned records");
  launch_prologue(pa, ta, stream);
  const long nt1 = (long)la.nsc * la.nlyr;
  const unsigned nb1 = (unsigned)((nt1 + kTeamsPerBlock - 1) / kTeamsPerBlock);
  const unsigned nb2 = (unsigned)((sa.nsc + kTeamsPerBlock - 1) / kTeamsPerBlock);
  // timing quadruple: layer start / end, sweep start / end
  if (ev) (void)hipEventRecord(ev[0], stream);
  if (team_layer_valu()) {
#if HD_AB_VARIANTS
    hipLaunchKernelGGL(hd_team_layer_kernel<NN>, dim3(nb1), dim3(kTeamBlock), 0, stream, la);
#endif
  } else {
    const hipError_t e = launch_team_layer_mfma(NN, la, stream);
    if (e != hipSuccess) return e;
  }
  if (ev) (void)hipEventRecord(ev[1], stream);
  if (ev) (void)hipEventRecord(ev[2], stream);
  if (!team_sweep_valu()) {
    const hipError_t e = launch_team_sweep_mfma(NN, sa, stream);
    if (ev) (void)hipEventRecord(ev[3], stream);
    return e;
  }
#if HD_AB_VARIANTS
  hipLaunchKernelGGL(hd_team_sweep_kernel<NN>, dim3(nb2), dim3(kTeamBlock), 0, stream, sa);
#else
  (void)nb2;
#endif
  if (ev) (void)hipEventRecord(ev[3], stream);
  return hipGetLastError();
}

// the two halves of launch_team, for the pipelined multi-chunk path of hd_solve
// (chunk k+1's layer kernel on one stream beside chunk k's sweep on another)
template <int NN>
static hipError_t launch_team_layer(const LayerArgs& la, hipStream_t stream) {
#if HD_AB_VARIANTS
  if (team_layer_valu()) {
    const long nt1 = (long)la.nsc * la.nlyr;
    const unsigned nb1 = (unsigned)((nt1 + kTeamsPerBlock - 1) / kTeamsPerBlock);
    hipLaunchKernelGGL(hd_team_layer_kernel<NN>, dim3(nb1), dim3(kTeamBlock), 0, stream, la);
    return hipGetLastError();
  }
#endif
  return launch_team_layer_mfma(NN, la, stream);
}
template <int NN>
static hipError_t launch_team_sweep(const SweepArgs& sa, hipStream_t stream) {
  if (!team_sweep_valu()) return launch_team_sweep_mfma(NN, sa, stream);
#if HD_AB_VARIANTS
  const unsigned nb2 = (unsigned)((sa.nsc + kTeamsPerBlock - 1) / kTeamsPerBlock);
  hipLaunchKernelGGL(hd_team_sweep_kernel<NN>, dim3(nb2), dim3(kTeamBlock), 0, stream, sa);
#endif
  return hipGetLastError();
}

hipError_t launch_team_layer_nn(int nn, const LayerArgs& la, hipStream_t stream) {
  switch (nn) {
    case 9: return launch_team_layer<9>(la, stream);
    case 10: return launch_team_layer<10>(la, stream);
    case 11: return launch_team_layer<11>(la, stream);
    case 12: return launch_team_layer<12>(la, stream);
    case 13: return launch_team_layer<13>(la, stream);
    case 14: return launch_team_layer<14>(la, stream);
    case 15: return launch_team_layer<15>(la, stream);
    case 16: return launch_team_layer<16>(la, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_team_sweep_nn(int nn, const SweepArgs& sa, hipStream_t stream) {
  switch (nn) {
    case 9: return launch_team_sweep<9>(sa, stream);
    case 10: return launch_team_sweep<10>(sa, stream);
    case 11: return launch_team_sweep<11>(sa, stream);
    case 12: return launch_team_sweep<12>(sa, stream);
    case 13: return launch_team_sweep<13>(sa, stream);
    case 14: return launch_team_sweep<14>(sa, stream);
    case 15: return launch_team_sweep<15>(sa, stream);
    case 16: return launch_team_sweep<16>(sa, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_solve_chunk_team(int nn, const PlanckArgs* pa, const TaucArgs* ta,
                                   const LayerArgs& la, const SweepArgs& sa, hipStream_t stream,
                                   hipEvent_t* ev) {
  switch (nn) {
    case 9: return launch_team<9>(pa, ta, la, sa, stream, ev);
    case 10: return launch_team<10>(pa, ta, la, sa, stream, ev);
    case 11: return launch_team<11>(pa, ta, la, sa, stream, ev);
    case 12: return launch_team<12>(pa, ta, la, sa, stream, ev);
    case 13: return launch_team<13>(pa, ta, la, sa, stream, ev);
    case 14: return launch_team<14>(pa, ta, la, sa, stream, ev);
    case 15: return launch_team<15>(pa, ta, la, sa, stream, ev);
    case 16: return launch_team<16>(pa, ta, la, sa, stream, ev);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace hd
