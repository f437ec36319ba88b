// hd_harp.hip -- gfx950 kernels of the harp-side steps around the solve
// (include/hdharp.h): optics assembly into the solver layout, band flux,
// heating rate, spherical flux correction.  All of it is HBM-bound streaming
// work: one lane per output element, consecutive lanes on consecutive
// doubles, no LDS.
//
//   hd_att_coef_kernel     per (attenuator, wave): locate + linear interpolation
//                          of (k_ext, ssa) in wavelength, clamped at the table
//                          ends  [interpn.h:34-76 with locate.h:15-42, ndim=1]
//   hd_attenuate_kernel    per (wave, col, layer): k c, ssa k c
//                          [s8_fuller.cpp:109-115, h2so4_simple.cpp:109-115]
//   hd_band_optics_kernel  per (wave, col, layer, prop): tau = dz sum k c,
//                          ssa = sum ssa k c / sum k c, moments 0
//                          [amars_sw.cpp:261-271]
//   hd_band_loop_kernel    per (wave, col, layer, prop): the band loop's mixing,
//                          tau-weighted ssa, tau*ssa-weighted HG moments, +1e-10
//                          [radiation_band.cpp:86-116]
//
// Floating-point contraction is off in this file's kernels: every product and
// sum rounds as in the reference's (and the numpy restatement's) expression order,
// so the optics are bit-identical to oracle/harp_np.py (they are bandwidth-bound,
// the FMAs would buy nothing).
//   hd_band_flux_kernel    per (col, level, dir): sum_w weight_w F_w in w order
//                          [amars_lw.cpp:84-88]; hd_band_flux_wave_kernel: a
//                          wave per output when outputs are few and bins many
//   hd_heating_kernel      per (col, layer)  [amars_sw.cpp:291-302]
//   hd_spherical_kernel    per (col, dir): top-down recurrence
//                          [spherical_flux_correction.cpp:3-17]
#include <hip/hip_runtime.h>

#include "../../include/hdharp.h"
#include "../../include/hdisort.h"
#include "hd_kernels.hpp"

#pragma clang fp contract(off)

namespace hd {
namespace {

constexpr int kMaxAtt = 16;

struct AttTables {
  int nrow[kMaxAtt];
  const double* wl[kMaxAtt];
  const double* k[kMaxAtt];
  const double* s[kMaxAtt];
  const double* g[kMaxAtt];  // HG asymmetry (band loop), or null
  int species[kMaxAtt];
  int natt;
  int nv;  // values per (attenuator, wave) in coef: 2 {k, ssa} or 3 {k, ssa, g}
};

// zero-offset j with xx[j] <= x < xx[j+1] for ascending or descending xx,
// -1 below / n-1 above the range (Numerical Recipes locate, as locate.h)
__device__ int locate_dev(const double* xx, double x, int n) {
  int jl = 0, ju = n + 1;  // unit offsets
  const bool ascnd = xx[n - 1] >= xx[0];
  while (ju - jl > 1) {
    const int jm = (ju + jl) >> 1;
    if ((x >= xx[jm - 1]) == ascnd) jl = jm;
    else ju = jm;
  }
  int j;
  if (x == xx[0]) j = 1;
  else if (x == xx[n - 1]) j = n;
  else j = jl;
  return j - 1;
}

// coef[a][w] = {k(lambda_w), ssa(lambda_w)[, g(lambda_w)]}
__global__ __launch_bounds__(256) void hd_att_coef_kernel(AttTables T, const double* coord,
                                                          int kind, int nwave, double* coef) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T.natt * nwave) return;
  const int a = t / nwave, w = t - a * nwave;
  const double x = kind == HD_COORD_WAVENUMBER ? 1.0e4 / coord[w] : coord[w];
  const int n = T.nrow[a];
  const double* ax = T.wl[a];
  int i1 = locate_dev(ax, x, n), i2;
  if (i1 == -1) {
    i1 = 0;
    i2 = 0;
  } else if (i1 == n - 1) {
    i2 = n - 1;
  } else {
    i2 = i1 + 1;
  }
  const double x1 = ax[i1], x2 = ax[i2];
  const double k1 = T.k[a][i1], k2 = T.k[a][i2];
  const double s1 = T.s[a][i1], s2 = T.s[a][i2];
  const double g1 = T.g[a] ? T.g[a][i1] : 0.0, g2 = T.g[a] ? T.g[a][i2] : 0.0;
  double k, s, g;
  if (x2 != x1) {
    k = ((x - x1) * k2 + (x2 - x) * k1) / (x2 - x1);
    s = ((x - x1) * s2 + (x2 - x) * s1) / (x2 - x1);
    g = ((x - x1) * g2 + (x2 - x) * g1) / (x2 - x1);
  } else {
    k = (k1 + k2) / 2.;
    s = (s1 + s2) / 2.;
    g = (g1 + g2) / 2.;
  }
  coef[(size_t)t * T.nv] = k;
  coef[(size_t)t * T.nv + 1] = s;
  if (T.nv > 2) coef[(size_t)t * T.nv + 2] = g;
}

__global__ __launch_bounds__(256) void hd_attenuate_kernel(const double* coef, int species,
                                                           const double* conc, int ncol,
                                                           int nlyr, int nspecies, long n,
                                                           double* out) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const long cl = t % ((long)ncol * nlyr);
  const int w = (int)(t / ((long)ncol * nlyr));
  const double c = conc[cl * nspecies + species];
  const double kc = coef[(size_t)w * 2] * c;
  out[t * 2] = kc;
  out[t * 2 + 1] = coef[(size_t)w * 2 + 1] * kc;  // ssa (k c), the reference's order
}

// one lane per output double of prop: consecutive lanes write consecutive
// doubles whatever nprop is
__global__ __launch_bounds__(256) void hd_band_optics_kernel(const double* coef, AttTables T,
                                                             int nwave, const double* conc,
                                                             int ncol, int nlyr, int nspecies,
                                                             const double* dz, int nprop,
                                                             long n, double* prop) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int p = (int)(t % nprop);
  const long e = t / nprop;  // (w, c, l)
  double v = 0.0;
  if (p < 2) {
    const long cl = e % ((long)ncol * nlyr);
    const int w = (int)(e / ((long)ncol * nlyr));
    double ext = 0.0, sca = 0.0;
    for (int a = 0; a < T.natt; ++a) {
      const double c = conc[cl * nspecies + T.species[a]];
      const double* cf = coef + ((size_t)a * nwave + w) * 2;
      const double kc = cf[0] * c;
      ext += kc;
      sca += cf[1] * kc;
    }
    v = p == 0 ? ext * dz[cl] : (ext != 0.0 ? (sca * dz[cl]) / (ext * dz[cl]) : 0.0);
  }
  prop[t] = v;
}

// the band loop (radiation_band.cpp:86-116), one lane per output double of
// prop [w][c][l][2+nmom]; coef stride 3 {k, ssa, g}
__global__ __launch_bounds__(256) void hd_band_loop_kernel(const double* coef, AttTables T,
                                                           const double* ext0, int nwave,
                                                           const double* conc, int ncol, int nlyr,
                                                           int nspecies, const double* dz,
                                                           int nprop, long n, double* prop) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int p = (int)(t % nprop);
  const long e = t / nprop;  // (w, c, l)
  const long cl = e % ((long)ncol * nlyr);
  const int w = (int)(e / ((long)ncol * nlyr));
  double ext = 0.0, sca = 0.0, mom = 0.0;
  if (ext0) ext += ext0[e];
  for (int a = 0; a < T.natt; ++a) {
    const double c = conc[cl * nspecies + T.species[a]];
    const double* cf = coef + ((size_t)a * nwave + w) * 3;
    const double kc = cf[0] * c;
    ext += kc;
    sca += cf[1] * kc;
    if (p >= 2 && T.g[a]) {  // chi_l = g^l, l = p - 1, by repeated products
      const double g = cf[2];
      double chi = g;
      for (int l = 2; l < p; ++l) chi = chi * g;
      mom += (chi * cf[1]) * kc;
    }
  }
  double v;
  if (p == 0) v = ext * dz[cl];
  else if (p == 1) v = sca / (ext + 1e-10);
  else v = mom / (sca + 1e-10);
  prop[t] = v;
}

__global__ __launch_bounds__(256) void hd_band_flux_kernel(const double* flux,
                                                           const double* weight, int nwave,
                                                           long m, double* bflux) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= m) return;
  double s = 0.0;
  for (int w = 0; w < nwave; ++w) s = fma(weight[w], flux[(size_t)w * m + t], s);
  bflux[t] = s;
}

// few outputs, many bins (one column line-by-line: ~80 outputs x 2e4 bins): a
// wave per output, lanes stride over w, fixed-order butterfly at the end
__global__ __launch_bounds__(256) void hd_band_flux_wave_kernel(const double* flux,
                                                                const double* weight, int nwave,
                                                                long m, double* bflux) {
  const long t = (long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= m) return;  // whole wave
  double s = 0.0;
  for (int w = lane; w < nwave; w += 64) s = fma(weight[w], flux[(size_t)w * m + t], s);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) bflux[t] = s;
}

__global__ __launch_bounds__(256) void hd_heating_kernel(const double* bflux, const double* dz,
                                                         const double* rho, double cp,
                                                         int ncol, int nlyr, double* out) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)ncol * nlyr) return;
  const long c = t / nlyr;
  const int k = (int)(t - c * nlyr);
  const double* f = bflux + (size_t)c * (nlyr + 1) * 2;
  const double df = f[2 * k] - f[2 * k + 1];
  const double df1 = f[2 * (k + 1)] - f[2 * (k + 1) + 1];
  out[t] = -(1.0 / (rho[t] * cp)) * (df1 - df) / dz[t];
}

__global__ __launch_bounds__(64) void hd_spherical_kernel(double* bflux, const double* x1f,
                                                          const double* area, const double* vol,
                                                          int ncol, int nlev) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)ncol * 2) return;
  const long c = t >> 1;
  const int d = (int)(t & 1);
  double* f = bflux + (size_t)c * nlev * 2 + d;
  double fiu = f[(size_t)(nlev - 1) * 2];
  for (int i = nlev - 2; i >= 0; --i) {
    const double dx1f = x1f[i + 1] - x1f[i];
    const double fi = f[(size_t)i * 2];
    const double volh = (fiu - fi) / dx1f * vol[i];
    fiu = fi;
    f[(size_t)i * 2] = (f[(size_t)(i + 1) * 2] * area[i + 1] - volh) / area[i];
  }
}

unsigned nblk(long n, int b) { return (unsigned)((n + b - 1) / b); }

int pack_tables(const hd_attenuator* atts, int natt, AttTables& T) {
  if (natt < 1 || natt > kMaxAtt) return set_global_error(HD_EINVAL, "natt=%d not in [1, %d]", natt, kMaxAtt);
  T.natt = natt;
  T.nv = 2;
  for (int a = 0; a < natt; ++a) {
    const hd_attenuator& at = atts[a];
    T.g[a] = nullptr;
    if (at.nrow < 1 || !at.wavelength || !at.kext || !at.ssa || at.species < 0)
      return set_global_error(HD_EINVAL, "attenuator %d: bad table (nrow=%d species=%d)", a,
                              at.nrow, at.species);
    T.nrow[a] = at.nrow;
    T.wl[a] = at.wavelength;
    T.k[a] = at.kext;
    T.s[a] = at.ssa;
    T.species[a] = at.species;
  }
  return HD_OK;
}

int launched(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_global_error(HD_EHIP, "%s: launch failed: %s", what, hipGetErrorString(e));
  return HD_OK;
}

}  // namespace

// ---- RFM tables (harp::RFMImpl, src/opacity/rfm.cpp:122-225) ----------------
// interpn.h's index pair and arithmetic on one axis
__device__ __forceinline__ void bracket(const double* ax, int n, double x, int& i1, int& i2) {
  i1 = locate_dev(ax, x, n);
  if (i1 == -1) {
    i1 = 0;
    i2 = 0;
  } else if (i1 == n - 1) {
    i2 = n - 1;
  } else {
    i2 = i1 + 1;
  }
}
__device__ __forceinline__ double lerp_ref(const double* ax, int i1, int i2, double x, double v1,
                                           double v2) {
  const double x1 = ax[i1], x2 = ax[i2];
  return x2 != x1 ? ((x - x1) * v2 + (x2 - x) * v1) / (x2 - x1) : (v1 + v2) / 2.;
}

// per (col, lyr): ln p and the temperature anomaly T - T_ref(ln p)  [get_reftemp]
__global__ __launch_bounds__(256) void hd_rfm_state_kernel(hd_rfm_table t, const double* pres,
                                                           const double* temp, long n,
                                                           double* work) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double lnp = log(pres[i]);
  int i1, i2;
  bracket(t.lnp, t.npres, lnp, i1, i2);
  const double tref = lerp_ref(t.lnp, i1, i2, lnp, t.tref[i1], t.tref[i2]);
  work[i] = lnp;
  work[n + i] = temp[i] - tref;
}

// per (wave, col, lyr), (col, lyr) fastest: interpn over (wave, ln p, T anomaly)
// in the reference's nesting, then 1e-3 exp(k) conc
__global__ __launch_bounds__(256) void hd_rfm_kernel(hd_rfm_table t, const double* conc,
                                                     int nspecies, long ncl, long n,
                                                     const double* work, double* out) {
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= n) return;
  const int w = (int)(id / ncl);
  const long cl = id - (long)w * ncl;
  const double xw = t.wave[w], xp = work[cl], xt = work[ncl + cl];
  int w1, w2, p1, p2, q1, q2;
  bracket(t.wave, t.nwave, xw, w1, w2);
  bracket(t.lnp, t.npres, xp, p1, p2);
  bracket(t.tgrid, t.ntemp, xt, q1, q2);
  auto at_wave = [&](int iw) {
    const double* d = t.kdata + (size_t)iw * t.npres * t.ntemp;
    const double a = lerp_ref(t.tgrid, q1, q2, xt, d[(size_t)p1 * t.ntemp + q1],
                              d[(size_t)p1 * t.ntemp + q2]);
    const double b = lerp_ref(t.tgrid, q1, q2, xt, d[(size_t)p2 * t.ntemp + q1],
                              d[(size_t)p2 * t.ntemp + q2]);
    return lerp_ref(t.lnp, p1, p2, xp, a, b);
  };
  const double v = lerp_ref(t.wave, w1, w2, xw, at_wave(w1), at_wave(w2));
  out[id] = 1.E-3 * exp(v) * conc[cl * nspecies + t.species];
}
}  // namespace hd

using hd::nblk;

extern "C" {

int hd_attenuate(const hd_attenuator* att, const double* coord, int coord_kind, int nwave,
                 const double* conc, int ncol, int nlyr, int nspecies, double* out,
                 void* stream_) {
  if (!att || nwave < 0 || ncol < 0 || nlyr < 0 || nspecies < 1 ||
      (coord_kind != HD_COORD_WAVELENGTH && coord_kind != HD_COORD_WAVENUMBER))
    return hd::set_global_error(HD_EINVAL, "hd_attenuate: bad arguments");
  if (att->species >= nspecies)
    return hd::set_global_error(HD_EINVAL, "hd_attenuate: species %d >= nspecies %d",
                                att->species, nspecies);
  const long n = (long)nwave * ncol * nlyr;
  if (n == 0) return HD_OK;
  if (!coord || !conc || !out) return hd::set_global_error(HD_EINVAL, "hd_attenuate: null array");
  hd::AttTables T{};
  int rc = hd::pack_tables(att, 1, T);
  if (rc) return rc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
  double* coef = nullptr;  // per-(wave) coefficients, stream-ordered scratch
  if (hipMallocAsync((void**)&coef, (size_t)nwave * 2 * sizeof(double), s) != hipSuccess) {
    (void)hipGetLastError();
    return hd::set_global_error(HD_ENOMEM, "hd_attenuate: scratch allocation failed");
  }
  hipLaunchKernelGGL(hd::hd_att_coef_kernel, dim3(nblk(nwave, 256)), dim3(256), 0, s, T, coord,
                     coord_kind, nwave, coef);
  hipLaunchKernelGGL(hd::hd_attenuate_kernel, dim3(nblk(n, 256)), dim3(256), 0, s, coef,
                     att->species, conc, ncol, nlyr, nspecies, n, out);
  rc = hd::launched("hd_attenuate");
  (void)hipFreeAsync(coef, s);
  return rc;
}

int hd_band_optics(const hd_attenuator* atts, int natt, const double* coord, int coord_kind,
                   int nwave, const double* conc, int ncol, int nlyr, int nspecies,
                   const double* dz, int nprop, double* prop, void* stream_) {
  if (!atts || nwave < 0 || ncol < 0 || nlyr < 0 || nspecies < 1 || nprop < 2 ||
      (coord_kind != HD_COORD_WAVELENGTH && coord_kind != HD_COORD_WAVENUMBER))
    return hd::set_global_error(HD_EINVAL, "hd_band_optics: bad arguments");
  hd::AttTables T{};
  int rc = hd::pack_tables(atts, natt, T);
  if (rc) return rc;
  for (int a = 0; a < natt; ++a)
    if (atts[a].species >= nspecies)
      return hd::set_global_error(HD_EINVAL, "hd_band_optics: attenuator %d species %d >= %d",
                                  a, atts[a].species, nspecies);
  const long n = (long)nwave * ncol * nlyr * nprop;
  if (n == 0) return HD_OK;
  if (!coord || !conc || !dz || !prop)
    return hd::set_global_error(HD_EINVAL, "hd_band_optics: null array");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
  double* coef = nullptr;
  if (hipMallocAsync((void**)&coef, (size_t)natt * nwave * 2 * sizeof(double), s) != hipSuccess) {
    (void)hipGetLastError();
    return hd::set_global_error(HD_ENOMEM, "hd_band_optics: scratch allocation failed");
  }
  hipLaunchKernelGGL(hd::hd_att_coef_kernel, dim3(nblk((long)natt * nwave, 256)), dim3(256), 0,
                     s, T, coord, coord_kind, nwave, coef);
  hipLaunchKernelGGL(hd::hd_band_optics_kernel, dim3(nblk(n, 256)), dim3(256), 0, s, coef, T,
                     nwave, conc, ncol, nlyr, nspecies, dz, nprop, n, prop);
  rc = hd::launched("hd_band_optics");
  (void)hipFreeAsync(coef, s);
  return rc;
}

int hd_band_loop_optics(const hd_band_attenuator* atts, int natt, const double* ext0,
                        const double* coord, int coord_kind, int nwave, const double* conc,
                        int ncol, int nlyr, int nspecies, const double* dz, int nmom,
                        double* prop, void* stream_) {
  if (!atts || nwave < 0 || ncol < 0 || nlyr < 0 || nspecies < 1 || nmom < 0 ||
      (coord_kind != HD_COORD_WAVELENGTH && coord_kind != HD_COORD_WAVENUMBER))
    return hd::set_global_error(HD_EINVAL, "hd_band_loop_optics: bad arguments");
  if (natt < 1 || natt > hd::kMaxAtt)
    return hd::set_global_error(HD_EINVAL, "hd_band_loop_optics: natt=%d not in [1, %d]", natt,
                                hd::kMaxAtt);
  hd_attenuator tabs[hd::kMaxAtt];
  for (int a = 0; a < natt; ++a) tabs[a] = atts[a].table;
  hd::AttTables T{};
  int rc = hd::pack_tables(tabs, natt, T);
  if (rc) return rc;
  T.nv = 3;
  for (int a = 0; a < natt; ++a) {
    if (atts[a].table.species >= nspecies)
      return hd::set_global_error(HD_EINVAL,
                                  "hd_band_loop_optics: attenuator %d species %d >= %d", a,
                                  atts[a].table.species, nspecies);
    T.g[a] = atts[a].gasym;
  }
  const int nprop = 2 + nmom;
  const long n = (long)nwave * ncol * nlyr * nprop;
  if (n == 0) return HD_OK;
  if (!coord || !conc || !dz || !prop)
    return hd::set_global_error(HD_EINVAL, "hd_band_loop_optics: null array");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
  double* coef = nullptr;
  if (hipMallocAsync((void**)&coef, (size_t)natt * nwave * 3 * sizeof(double), s) != hipSuccess) {
    (void)hipGetLastError();
    return hd::set_global_error(HD_ENOMEM, "hd_band_loop_optics: scratch allocation failed");
  }
  hipLaunchKernelGGL(hd::hd_att_coef_kernel, dim3(nblk((long)natt * nwave, 256)), dim3(256), 0,
                     s, T, coord, coord_kind, nwave, coef);
  hipLaunchKernelGGL(hd::hd_band_loop_kernel, dim3(nblk(n, 256)), dim3(256), 0, s, coef, T, ext0,
                     nwave, conc, ncol, nlyr, nspecies, dz, nprop, n, prop);
  rc = hd::launched("hd_band_loop_optics");
  (void)hipFreeAsync(coef, s);
  return rc;
}

int hd_band_flux(const double* flux, const double* weight, int nwave, int ncol, int nlev,
                 double* bflux, void* stream_) {
  if (nwave < 0 || ncol < 0 || nlev < 1)
    return hd::set_global_error(HD_EINVAL, "hd_band_flux: bad sizes");
  const long m = (long)ncol * nlev * 2;
  if (m == 0) return HD_OK;
  if ((nwave > 0 && (!flux || !weight)) || !bflux)
    return hd::set_global_error(HD_EINVAL, "hd_band_flux: null array");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
  if (m >= 65536 || nwave < 256) {  // a lane per output: coalesced, w in order
    hipLaunchKernelGGL(hd::hd_band_flux_kernel, dim3(nblk(m, 256)), dim3(256), 0, s, flux,
                       weight, nwave, m, bflux);
  } else {  // a wave per output
    hipLaunchKernelGGL(hd::hd_band_flux_wave_kernel, dim3(nblk(m, 4)), dim3(256), 0, s, flux,
                       weight, nwave, m, bflux);
  }
  return hd::launched("hd_band_flux");
}

int hd_heating_rate(const double* bflux, const double* dz, const double* rho, double cp,
                    int ncol, int nlyr, double* dTdt, void* stream_) {
  if (ncol < 0 || nlyr < 1 || !(cp > 0.0))
    return hd::set_global_error(HD_EINVAL, "hd_heating_rate: bad arguments");
  if ((long)ncol * nlyr == 0) return HD_OK;
  if (!bflux || !dz || !rho || !dTdt)
    return hd::set_global_error(HD_EINVAL, "hd_heating_rate: null array");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
  hipLaunchKernelGGL(hd::hd_heating_kernel, dim3(nblk((long)ncol * nlyr, 256)), dim3(256), 0, s,
                     bflux, dz, rho, cp, ncol, nlyr, dTdt);
  return hd::launched("hd_heating_rate");
}

int hd_spherical_flux_correction(double* bflux, const double* x1f, const double* area,
                                 const double* vol, int ncol, int nlev, void* stream_) {
  if (ncol < 0 || nlev < 1) return hd::set_global_error(HD_EINVAL, "hd_spherical_flux_correction: bad sizes");
  if (ncol == 0 || nlev == 1) return HD_OK;
  if (!bflux || !x1f || !area || !vol)
    return hd::set_global_error(HD_EINVAL, "hd_spherical_flux_correction: null array");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
  hipLaunchKernelGGL(hd::hd_spherical_kernel, dim3(nblk((long)ncol * 2, 64)), dim3(64), 0, s,
                     bflux, x1f, area, vol, ncol, nlev);
  return hd::launched("hd_spherical_flux_correction");
}

int hd_rfm_attenuate(const hd_rfm_table* t, const double* conc, int ncol, int nlyr, int nspecies,
                     const double* pres, const double* temp, double* out, void* stream_) {
  if (!t || ncol < 0 || nlyr < 0 || nspecies < 1 || t->nwave < 1 || t->npres < 1 ||
      t->ntemp < 1 || t->species < 0 || t->species >= nspecies)
    return hd::set_global_error(HD_EINVAL, "hd_rfm_attenuate: bad arguments");
  if (!t->wave || !t->lnp || !t->tgrid || !t->tref || !t->kdata)
    return hd::set_global_error(HD_EINVAL, "hd_rfm_attenuate: null table array");
  const long ncl = (long)ncol * nlyr;
  const long n = ncl * t->nwave;
  if (n == 0) return HD_OK;
  if (!conc || !pres || !temp || !out)
    return hd::set_global_error(HD_EINVAL, "hd_rfm_attenuate: null array");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
  double* work = nullptr;  // ln p and the temperature anomaly per (col, lyr)
  if (hipMallocAsync((void**)&work, (size_t)ncl * 2 * sizeof(double), s) != hipSuccess) {
    (void)hipGetLastError();
    return hd::set_global_error(HD_ENOMEM, "hd_rfm_attenuate: scratch allocation failed");
  }
  hipLaunchKernelGGL(hd::hd_rfm_state_kernel, dim3(nblk(ncl, 256)), dim3(256), 0, s, *t, pres,
                     temp, ncl, work);
  hipLaunchKernelGGL(hd::hd_rfm_kernel, dim3(nblk(n, 256)), dim3(256), 0, s, *t, conc, nspecies,
                     ncl, n, work, out);
  int rc = hd::launched("hd_rfm_attenuate");
  (void)hipFreeAsync(work, s);
  return rc;
}

}  // extern "C"
