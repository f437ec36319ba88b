// hd_rad.hpp -- argument block and launchers of the intensity path
// (hd_rad.hip): every azimuthal mode, user optical depths and user angles,
// nstr <= 32 (one lane per (solve, mode) problem).
#pragma once

#include <hip/hip_runtime.h>

#include "hd_kernels.hpp"

namespace hd {

constexpr int kRadMaxNN = kMaxNN;  // nstr <= 32 (NN > 8: rolled loops, private memory)

template <int NN>
__host__ __device__ constexpr int rad_nsym() {
  return NN * (NN + 1) / 2;
}
// per-(unit, layer) layer-operator record of the intensity kernels: the register
// path's layout (R~, T~ upper, S~+, S~-, tau') at every nstr
__host__ __device__ constexpr int rad_layer_record_doubles(int nn) {
  return nn * (nn + 1) + 2 * nn + 1;
}
// per-(unit, layer) radiance record: L (packed lower), V, k, Z+, Z-, h, B_top,
// dB/dtau', tau', omega', exp(-k tau'), exp(-tau'/mu0)
__host__ __device__ constexpr int rad_rec_doubles(int nn) {
  return nn * (nn + 1) / 2 + nn * nn + 5 * nn + 5;
}
// per-(unit, layer) sweep record for the back-substitution: ZT, t, R_above (packed), S_down
__host__ __device__ constexpr int rad_bsub_doubles(int nn) {
  return nn * nn + 2 * nn + nn * (nn + 1) / 2;
}

struct RadArgs {
  // inputs (per solve, index s = s0 + sl)
  const double* prop;
  const double* fbeam;
  const double* umu0;
  const double* albedo;
  const double* fisot;
  const double* phi0;     // [S] degrees or null
  const double* planckv;  // [nlyr+3][ns] or null
  const double* tauc;     // [nlyr][ns] scaled depth of every layer top (beam) or null
  double* taus;           // [nlyr+1][ns] unscaled depth of every level (written by the taus kernel)
  // user grid (device)
  const double* umu;   // [numu]
  const double* phi;   // [nphi] degrees
  const double* utau;  // [ntau] unscaled, ascending; null = the nlyr+1 levels
  // scratch (unit u = m*ns + sl is the fastest index)
  double* rsw;   // [nlyr][ne1][nu]   layer operators (flux-kernel layout)
  double* rrd;   // [nlyr][rad_rec][nu]
  double* bsub;  // [nlyr][rad_bsub][nu]
  double* lev;   // [nlyr+1][2NN][nu]   I+ (NN) then I- (NN) per level, solver order
  double* cst;   // [nlyr][2NN][nu]     C+ then C-
  double* radm;  // [ntau*numu][nu]     radiance per mode
  // outputs
  double* flux;  // [S][ntau][2], index 0 = deepest user depth
  double* uu;    // [S][nphi][ntau][numu]
  int* status;
  int* anyerr;
  long s0;
  int ns;     // solves in this chunk
  int nm;     // azimuthal modes (nstr with a beam and radiances, else 1)
  int nu;     // ns * nm
  int ncol;
  int nlyr;
  int nprop;
  int nmom;
  int planck;
  int max_sweeps;
  int numu, nphi, ntau;
  int corint;  // Nakajima-Tanaka TMS correction of the single scattering
};

hipError_t upload_rad_tables(const QuadHost* per_nn);  // nn 1..kRadMaxNN
// tauc/planck prologue must have run (launch_prologue) for the chunk's solves;
// radiances = false: fluxes at the user depths only (mode 0, no uu)
hipError_t launch_rad_chunk(int nn, const RadArgs& a, bool radiances, hipStream_t stream);
size_t rad_scratch_doubles_per_unit(int nn, int nlyr);
// nstr 18..32: the adding sweep + back-substitution on the team layout with the
// dense products on FP64 MFMA, four units per wave (hd_team_mfma.hip)
hipError_t launch_rad_team_sweep(int nn, const RadArgs& a, hipStream_t stream);
// nstr 18..32: the per-(unit, layer) setup on the team layout + FP64 MFMA, and its
// Y_l^m tables (uploaded with the other intensity-path tables)
hipError_t launch_rad_team_layer(int nn, const RadArgs& a, hipStream_t stream);
hipError_t upload_rad_tables_team(const QuadHost* per_nn);
// nstr 18..32: the same kernels compiled with rolled NN-loops (hd_rad_wide.hip)
namespace wide {
hipError_t upload_rad_tables(const QuadHost* per_nn);
hipError_t launch_rad_chunk(int nn, const RadArgs& a, bool radiances, hipStream_t stream);
}  // namespace wide

}  // namespace hd
