// hd_kernels.hpp -- kernel argument blocks and launcher declarations.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>

#include "hd_device.hpp"

namespace hd {

constexpr int kMaxNN = 16;    // nstr <= 32
constexpr int kMaxRegNN = 8;  // one-lane-per-problem kernels (hd_kernels.hip) up to nstr 16;
                              // 16-lane team kernels (hd_team.hip) for nstr 18..32

template <int NN>
__host__ __device__ constexpr int ne1() {  // per-layer operator record (doubles)
  return NN * (NN + 1) + 2 * NN + 1;
}
template <int NN>
__host__ __device__ constexpr int ne2() {  // per-level back-substitution record
  return NN * NN + 2 * NN + 1;
}
// Register-path flux records in 16-byte element pairs: [lc][pair][nsc] of
// double2, so each lane moves two record elements per memory instruction (a
// wave's 64 lanes: 1 KB contiguous).  Every group of elements starts at an even
// element (padded), so a pair never spans two groups.
__host__ __device__ constexpr int even_up(int n) { return (n + 1) & ~1; }
template <int NN>
struct RecL {  // layer record: R~ upper | T~ upper | S~+ | S~- | tau'
  static constexpr int nsym = NN * (NN + 1) / 2;
  static constexpr int R = 0;
  static constexpr int T = R + even_up(nsym);
  static constexpr int Sp = T + even_up(nsym);
  static constexpr int Sm = Sp + even_up(NN);
  static constexpr int Tau = Sm + even_up(NN);
  static constexpr int pairs = (Tau + 2) / 2;
};
template <int NN>
struct RecB {  // back-substitution record: ZT (column-major) | t | rc | cs
  static constexpr int Z = 0;
  static constexpr int Tv = Z + even_up(NN * NN);
  static constexpr int Rc = Tv + even_up(NN);
  static constexpr int Cs = Rc + even_up(NN);
  static constexpr int pairs = (Cs + 2) / 2;
};
// Record traffic (layer records, back-substitution records) of a large chunk is written
// once and read once, a whole kernel later, far beyond what the caches hold: there the
// kernels use nontemporal loads and stores (the `nt` bit, NT = true) so that it does not
// displace anything else -- C4 +2 %, the 8-GPU rank shape +1.6 % in interleaved runs.  A
// small chunk's records stay in L2 between its kernels and plain accesses keep them there
// (C1: 146 k vs 137 k solves/s with nt).  The team path (nstr 18..32) uses nt for its
// whole-row record stores only (C5 +1.3 %): its record reads are 8-byte pieces of a
// team's lanes, and with nt on them C5 ran 1.07 M solves/s against 1.33 M.
// profiles/r05/record_nt_ab.txt
#ifndef HD_NT_MIN_SOLVES
#define HD_NT_MIN_SOLVES 4096  // records of >= ~230 MB per chunk: far beyond the 32 MB of L2
#endif
constexpr int kNtMinSolves = HD_NT_MIN_SOLVES;  // chunks of at least this many solves use NT
typedef double hd_d2v __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ void rec_store(double2* p, double2 v) {
  if constexpr (NT) {
    hd_d2v w = {v.x, v.y};
    __builtin_nontemporal_store(w, reinterpret_cast<hd_d2v*>(p));
  } else {
    *p = v;
  }
}
template <bool NT>
__device__ __forceinline__ double2 rec_load(const double2* p) {
  if constexpr (NT) {
    const hd_d2v w = __builtin_nontemporal_load(reinterpret_cast<const hd_d2v*>(p));
    return make_double2(w.x, w.y);
  } else {
    return *p;
  }
}
template <bool NT>
__device__ __forceinline__ void rec_st(double* p, double v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <bool NT>
__device__ __forceinline__ double rec_ld(const double* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
// writes record elements in increasing order within a group as 16-byte pairs
template <bool NT>
struct PairOutT {
  double2* p;
  size_t stride;  // pairs -> double2 stride (nsc)
  double pend;
  __device__ __forceinline__ void put(int e, double v) {
    if (e & 1) rec_store<NT>(p + (size_t)(e >> 1) * stride, make_double2(pend, v));
    else pend = v;
  }
  // after the group's last element e: a lone even element goes out with a zero pad
  __device__ __forceinline__ void close(int e) {
    if (!(e & 1)) rec_store<NT>(p + (size_t)(e >> 1) * stride, make_double2(pend, 0.0));
  }
};
using PairOut = PairOutT<false>;
template <bool NT = false>
__device__ __forceinline__ double pair_get(const double2* p, size_t stride, int e) {
  const double2 q = rec_load<NT>(p + (size_t)(e >> 1) * stride);
  return (e & 1) ? q.y : q.x;
}

// packed row-major upper-triangle index of (i, j) in either order
template <int NN>
__host__ __device__ constexpr int sym_index(int i, int j) {
  return i <= j ? i * NN - i * (i - 1) / 2 + (j - i) : j * NN - j * (j - 1) / 2 + (i - j);
}

// Chunk lane -> solve.  A call's solves are processed in chunks of consecutive
// indices q = s0 + sl.  Normally q is the caller's solve s = wave*ncol + col;
// with the fused band epilogue (hd_solve_band) the order is column-major,
// q = col*nwave + wave, so that the wave-points of one column sit in
// neighbouring lanes and their weighted fluxes are summed across lanes.
// (32-bit arithmetic: hd_solve limits nwave*ncol to 2^31 - 1)
__host__ __device__ inline long solve_of(long q, int cmaj, int nwave, int ncol) {
  if (!cmaj) return q;
  const unsigned qu = (unsigned)q, c = qu / (unsigned)nwave;
  return (long)(qu - c * (unsigned)nwave) * ncol + c;
}

struct PlanckArgs {
  const double* temf;   // [ncol][nlyr+1], level 0 = bottom
  const double* btemp;  // [S] or null
  const double* ttemp;  // [S] or null
  const double* temis;  // [S] or null
  const double* wlo;    // [nwave]
  const double* whi;    // [nwave]
  double* out;          // [nlyr+3][nsc]
  long s0;
  int nsc;
  int ncol;
  int nlyr;
  int cmaj;   // column-major chunk order (solve_of)
  int nwave;
};

struct TaucArgs {
  const double* prop;
  double* out;  // [nlyr][nsc] scaled optical depth at the top of each solver layer
  long s0;
  int nsc;
  int nlyr;
  int nprop;
  int use_f;    // delta-M active (moments >= nstr available)
  int f_slot;   // prop slot of chi_nstr = 1 + nstr
  int cmaj;     // column-major chunk order (solve_of)
  int nwave;
  int ncol;
};

struct LayerArgs {
  const double* prop;
  const double* tauc;     // [nlyr][nsc] (beam) or null: unit beam at every layer top
  const double* fbeam;
  const double* umu0;
  const double* planckv;  // [nlyr+3][nsc] (planck) or null
  double* scr;
  int* status;
  int* anyerr;
  long s0;    // first solve of this chunk (flattened wave*ncol + col)
  int nsc;    // solves in this chunk (= scratch stride)
  int ncol;
  int nlyr;
  int nprop;
  int nmom;   // moments used = min(nmom, nprop-2)
  int planck;
  int max_sweeps;
  double* sink;  // team path: store target of lanes >= NN (>= 2*16^2+2*16+2 doubles)
  int cmaj;      // column-major chunk order (solve_of)
  int nwave;
  int warm;      // team path: start the Jacobi from the (ssa, chi_1) bin's eigenvectors
};

// Up to this many solves per chunk the nstr 4 / 8 sweep runs in NN-lane teams: there
// the one-lane sweep leaves most SIMDs idle or at one wave (C1 16 solves, C3 19 990:
// +25 % and +9 % a step); at 1e5 solves it fills the chip and the teams' redundant
// work (2x the one-lane flops) cancels their shorter chains (C3l within noise).
constexpr int kQuadMaxSolves = 32768;

struct SweepArgs {
  const double* scr;
  double* bsub;
  double* xsurf;  // [nsc] Lambert-surface amplitude x (I+ = g x), down -> up kernel
  double* flux;
  const double* fbeam;
  const double* umu0;
  const double* albedo;
  const double* fisot;
  const double* planckv;
  int* status;
  int* anyerr;
  long s0;
  int nsc;
  int ncol;
  int nlyr;
  int planck;
  double* sink;  // team path: store target of lanes >= NN
  int cmaj;      // column-major chunk order (solve_of)
  int nwave;
  // fused band epilogue (hd_solve_band); part == nullptr: off.  Register path:
  // the back-substitution sums wts[w] F over the lanes of a column (segmented,
  // fixed order) and a wave's segment heads store [wave][slot][lev][2] partials;
  // fsurf [2][nsc] carries the sweep's surface fluxes to it.  flux may then be null.
  const double* wts;
  double* part;
  double* fsurf;
  int nslot;       // column slots per wave
  int rsteps;      // ceil(log2(min(nwave, 64))) shuffle steps
  int flux_local;  // team path: flux is a chunk buffer [nsc][L+1][2]
  // register path: the layer records' sources are for a unit beam at each layer
  // top (LayerArgs.tauc null); the sweep scales them by exp(-tau_c/mu0)
  int beam_scale;
  // team path (nstr 18..32): the lean sweep (hd_team_mfma_sweep_lean_kernel, two waves
  // per SIMD) instead of the one-wave-per-SIMD sweep
  int lean;
  // register path, nstr 4 / 8: the sweep in NN-lane teams (hd_sweep_quad_kernel):
  // 1 on, 0 off, -1 for chunks of at most kQuadMaxSolves solves
  int quad;
  // register path, nstr 16: the adding sweep with the stack state in LDS
  // (hd_sweep_lean_kernel, two waves per SIMD) instead of hd_sweep_kernel
  int lean8;
};

// chunk epilogue of the fused band sum: bflux[c] (=|+=) sum of the chunk's
// partials of column c, in wave order (cmaj: register-path partials; else the
// chunk flux buffer of the team path in wave-point order)
struct BandArgs {
  const double* part;   // register path: [wave][nslot][nlev][2]
  const double* fchunk; // team path: [nsc][nlev][2]
  const double* wts;    // [nwave]
  double* bflux;        // [ncol][nlev][2]
  long s0;
  int nsc;
  int ncol;
  int nwave;
  int nlev;
  int nslot;
};

struct QuadHost {
  double mu[kMaxNN], w[kMaxNN], sd[kMaxNN], g[kMaxNN];
  double pt[2 * kMaxNN][kMaxNN];
};

// Warm start of the team layer kernel's Jacobi (hd_team_mfma.hip, nstr 18..32):
// for every (ssa, chi_1) bin of a kWarmG x kWarmG grid on [0,1]^2, the
// eigenvectors V0 of Sym = B0^T B0 of a Henyey-Greenstein layer at the bin
// centre (B0 = C^T L, the layer kernel's factors).  The kernel runs the Jacobi
// on B0 V0, whose columns are already close to orthogonal (any orthogonal V0
// gives the same eigenpairs; the table only saves sweeps: 5 -> 3 per wave at
// nstr 32, profiles/r03_warm/).  Entry kWarmG^2 is the identity
// (non-scattering layers: Sym is diagonal).  The register path (nstr <= 16)
// saves one sweep of four, which does not pay for the rotations
// (profiles/r03_warm_reg_notkept/).
constexpr int kWarmG = 16;
constexpr int kWarmEntries = kWarmG * kWarmG + 1;
__host__ __device__ constexpr int warm_bin(double x) {
  // x in [0,1] -> 0..kWarmG-1 (NaN and out-of-range values clamp)
  return x > 0.0 ? (x < 1.0 ? (int)(x * kWarmG) : kWarmG - 1) : 0;
}
// host: the eigenvectors (row-major nn x nn, columns = vectors) of bin (ia, ib)
void warm_eigvecs(int nn, const QuadHost& q, int ia, int ib, double* v);

// copy the quadrature tables (index nn-1) into the current device's constant memory
hipError_t upload_quad_tables(const QuadHost* per_nn);       // nn 1..kMaxRegNN
hipError_t upload_quad_tables_team(const QuadHost* per_nn);  // nn kMaxRegNN+1..kMaxNN
// cumulative scaled depth (beam) and level Planck radiances (planck) of a chunk
void launch_prologue(const PlanckArgs* pa, const TaucArgs* ta, hipStream_t stream);
// ev: 3 events (before K1, between, after K2) or nullptr; pa null when planck is off
hipError_t launch_solve_chunk_nn(int nn, const PlanckArgs* pa, const TaucArgs* ta,
                                 const LayerArgs& la, const SweepArgs& sa, hipStream_t stream,
                                 hipEvent_t* ev);
// back-substitution of a register-path chunk (reads sa.bsub / sa.xsurf)
hipError_t launch_backsub_nn(int nn, const SweepArgs& sa, hipStream_t stream, bool tail);
// register path, separately: the layer kernel and the adding sweep of one chunk
hipError_t launch_layer_nn(int nn, const LayerArgs& la, hipStream_t stream);
hipError_t launch_sweep_nn(int nn, const SweepArgs& sa, hipStream_t stream);
// register path, nstr 16: layer setup + adding sweep + back-substitution of one chunk in
// one kernel (hd_column_kernel; la.scr unused -- no layer records)
hipError_t launch_column_nn(int nn, const LayerArgs& la, const SweepArgs& sa, hipStream_t stream);
hipError_t launch_solve_chunk_team(int nn, const PlanckArgs* pa, const TaucArgs* ta,
                                   const LayerArgs& la, const SweepArgs& sa, hipStream_t stream,
                                   hipEvent_t* ev);
// team path, separately: the layer kernel and the sweep of one chunk
hipError_t launch_team_layer_nn(int nn, const LayerArgs& la, hipStream_t stream);
hipError_t launch_team_sweep_nn(int nn, const SweepArgs& sa, hipStream_t stream);
size_t scratch_doubles_per_solve(int nn, int nlyr, bool planck);
// the chunk epilogue of hd_solve_band (after the chunk's back-substitution)
hipError_t launch_band_reduce(const BandArgs& ba, hipStream_t stream);
// column slots a 64-lane wave of consecutive column-major solves can touch
inline int band_slots(int nwave) { return nwave >= 64 ? 2 : (63 / nwave + 2 < 64 ? 63 / nwave + 2 : 64); }
inline int band_steps(int nwave) {
  int k = 0;
  while ((1 << k) < (nwave < 64 ? nwave : 64)) ++k;
  return k;
}
// Kernel variants that were measured and not kept (the column
// kernel, the LDS-state nstr-16 sweep, the one-wave team sweep, the VALU team layer
// and sweep kernels, the per-angle radiance user kernel at nstr <= 16) are compiled
// only into the A/B build (scripts/ab/build_variant.sh defines HD_AB_VARIANTS=1):
// the product library carries only the kernels its dispatch can select.
#ifndef HD_AB_VARIANTS
#define HD_AB_VARIANTS 0
#endif
// A/B switches of the kernel variants (HD_JACOBI_WARM, HD_TEAM_SWEEP_LEAN, HD_SWEEP_QUAD,
// HD_SWEEP_LEAN8, HD_RAD_USER, HD_TEAM_LAYER, HD_TEAM_SWEEP) are read only when the
// single opt-in HD_AB=1 is set too: a stray variable in a user's environment never
// changes which kernel runs (or the bits of the result).  Tests and the A/B scripts set it.
inline const char* ab_env(const char* name) {
  const char* on = std::getenv("HD_AB");
  if (!on || on[0] != '1' || on[1] != '\0') return nullptr;
  return std::getenv(name);
}
// record an error for hd_last_error(NULL) (entry points without a context); returns code
int set_global_error(int code, const char* fmt, ...);
// doubles per (layer, solve) of the layer-operator and back-substitution records
size_t layer_record_doubles(int nn);
size_t bsub_record_doubles(int nn);

}  // namespace hd
