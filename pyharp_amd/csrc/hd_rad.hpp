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
  double* rsw;   // [nlyr][ne1][nu]   layer operators (flux-kernel layout); nstr > 16:
                 //   [nlyr][nu][ne1] (team kernels, unit-contiguous)
  double* rrd;   // [nlyr][rad_rec][nu]; nstr > 16: [nlyr][nu][rad_rec]
  double* bsub;  // [nlyr][rad_bsub][nu]; nstr > 16: [nlyr][nu][rad_bsub]
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
  // nstr <= 16 with radiances: the const kernel also writes each (unit, layer)'s
  // angle-independent maps into the rsw / bsub regions (dead after the sweep) and the
  // user-angle integration runs hd_rad_user_map_kernel
  int umap;
  double* sink;  // team kernels: target of the stores a lane does not own (>= 64 doubles)
};

// int_{t1}^{t2} a exp(-c (t - tref)) exp(-(t - t1)/mu) dt/mu, t1 = evaluation
// depth, (t2 - t1)/mu >= 0; the 1 + c mu -> 0 limit through (1 - e^-x)/x
__device__ __forceinline__ double seg_exp(double a, double c, double t1, double t2, double tref,
                                          double mu) {
  const double p1 = exp(-c * (t1 - tref));
  const double den = fma(c, mu, 1.0);
  const double dt = (t2 - t1) / mu;
  const double x = den * dt;
  if (fabs(x) < 0.5) {
    const double ph = x == 0.0 ? 1.0 : -expm1(-x) / x;
    return a * p1 * dt * ph;
  }
  const double p2 = exp(-c * (t2 - tref) - dt);
  return a * (p1 - p2) / den;
}

// (pa - pb)/den where pb = pa e^{-y}, y = den * len: the direct quotient, or
// pa * len * (1 - e^-y)/y by its Taylor series when |y| < 1/2 (den -> 0)
__device__ __forceinline__ double dexp(double pa, double pb, double den, double len) {
  const double y = den * len;
  // sum_{n<=13} (-y)^n/(n+1)!: |y|^14/15! < 5e-17 for |y| < 1/2
  double ph = 1.0 / 87178291200.0;  // 1/14!
  ph = fma(ph, -y, 1.0 / 6227020800.0);
  ph = fma(ph, -y, 1.0 / 479001600.0);
  ph = fma(ph, -y, 1.0 / 39916800.0);
  ph = fma(ph, -y, 1.0 / 3628800.0);
  ph = fma(ph, -y, 1.0 / 362880.0);
  ph = fma(ph, -y, 1.0 / 40320.0);
  ph = fma(ph, -y, 1.0 / 5040.0);
  ph = fma(ph, -y, 1.0 / 720.0);
  ph = fma(ph, -y, 1.0 / 120.0);
  ph = fma(ph, -y, 1.0 / 24.0);
  ph = fma(ph, -y, 1.0 / 6.0);
  ph = fma(ph, -y, 0.5);
  ph = fma(ph, -y, 1.0);
  return fabs(y) < 0.5 ? pa * len * ph : (pa - pb) / den;
}

// user depth lu of solve sl: the caller's utau or the level depths
__device__ __forceinline__ double user_tau(const RadArgs& A, int lu, int sl) {
  return A.utau ? A.utau[lu] : A.taus[(size_t)lu * A.ns + sl];
}

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
// nstr 18..32: the user-angle integration in two kernels -- per (unit, layer) on the
// team layout + FP64 MFMA (every user angle's whole-layer source term and the
// interior user depths' partial integrals), then a per-(unit, angle) scan over the
// layers.  Needs numu <= rad_layer_record_doubles(nn) (the whole-layer terms reuse
// the layer-operator records, free after the sweep)
hipError_t launch_rad_team_user(int nn, const RadArgs& a, hipStream_t stream);
hipError_t upload_rad_tables_team(const QuadHost* per_nn);
// nstr 18..32: the same kernels compiled with rolled NN-loops (hd_rad_wide.hip)
namespace wide {
hipError_t upload_rad_tables(const QuadHost* per_nn);
hipError_t launch_rad_chunk(int nn, const RadArgs& a, bool radiances, hipStream_t stream);
}  // namespace wide

}  // namespace hd
