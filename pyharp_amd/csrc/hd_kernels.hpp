// hd_kernels.hpp -- kernel argument blocks and launcher declarations.
#pragma once

#include <hip/hip_runtime.h>

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
// packed row-major upper-triangle index of (i, j) in either order
template <int NN>
__host__ __device__ constexpr int sym_index(int i, int j) {
  return i <= j ? i * NN - i * (i - 1) / 2 + (j - i) : j * NN - j * (j - 1) / 2 + (i - j);
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
};

struct LayerArgs {
  const double* prop;
  const double* tauc;     // [nlyr][nsc] (beam) or null
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
};

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
};

struct QuadHost {
  double mu[kMaxNN], w[kMaxNN], sd[kMaxNN], g[kMaxNN];
  double pt[2 * kMaxNN][kMaxNN];
};

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
hipError_t launch_solve_chunk_team(int nn, const PlanckArgs* pa, const TaucArgs* ta,
                                   const LayerArgs& la, const SweepArgs& sa, hipStream_t stream,
                                   hipEvent_t* ev);
size_t scratch_doubles_per_solve(int nn, int nlyr, bool planck);
// record an error for hd_last_error(NULL) (entry points without a context); returns code
int set_global_error(int code, const char* fmt, ...);
// doubles per (layer, solve) of the layer-operator and back-substitution records
size_t layer_record_doubles(int nn);
size_t bsub_record_doubles(int nn);

}  // namespace hd
