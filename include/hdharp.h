/*
 * hdharp.h -- C-ABI of the harp-side steps on either side of the DISORT flux
 * solve (part of libhdisort.so; HIP kernels for gfx950, include/hdisort.h
 * for the solve itself).  SURVEY.md section 8(f) ranks 1 and 2:
 *
 *   before the solve -- optics assembly straight into the solver layout:
 *     hd_attenuate     one attenuator's forward: S8FullerImpl::forward
 *                      (src/opacity/s8_fuller.cpp:72-117) and
 *                      H2SO4SimpleImpl::forward (src/opacity/h2so4_simple.cpp:72-117):
 *                      1-D linear interpolation of (k_ext, ssa) in wavelength
 *                      (src/math/interpn.h:34-76, locate.h:15-42, clamped at the
 *                      table ends), times the species concentration
 *     hd_band_optics   the amars_sw assembly (examples/amars_sw.cpp:261-271):
 *                      sum of attenuators, x dz, ssa = sum(ssa k c)/sum(k c),
 *                      written as prop [nwave][ncol][nlyr][nprop]
 *     hd_band_loop_optics  the library band loop's mixing (radiation_band.cpp:86-116):
 *                      tau-weighted ssa, tau*ssa-weighted phase moments, the
 *                      reference's +1e-10 regularisation
 *   after the solve -- band epilogue:
 *     hd_band_flux     sum_w weight_w F_w (examples/amars_lw.cpp:84-88;
 *                      amars_sw.cpp:169-196 with weight = d(wavenumber);
 *                      legacy src/rtsolver/rt_solver_disort.cpp_:183-184)
 *     hd_heating_rate  dT/dt = -(dF_net/dz)/(rho c_p), F_net = F_up - F_dn
 *                      (examples/amars_sw.cpp:291-302)
 *     hd_spherical_flux_correction  src/utils/spherical_flux_correction.cpp:3-17
 *                      along the level axis of the harp band flux
 *                      (legacy rt_solver_disort.cpp_:186-207)
 *
 * All array pointers are DEVICE pointers; stream = hipStream_t (NULL =
 * default).  Return codes and hd_last_error(NULL) as in hdisort.h.
 */
#ifndef HDHARP_H_
#define HDHARP_H_

#ifdef __cplusplus
extern "C" {
#endif

/* one opacity table, already in the units the reference keeps after reset():
 * k_ext multiplied by the species weight [m^2/kg -> m^2/mol]
 * (s8_fuller.cpp:64-66, h2so4_simple.cpp:64-66) */
typedef struct hd_attenuator {
  int nrow;                 /* table rows, wavelength strictly monotonic         */
  const double *wavelength; /* [nrow] um (first data column of the text table)   */
  const double *kext;       /* [nrow] extinction cross-section, m^2/mol          */
  const double *ssa;        /* [nrow] single-scattering albedo                   */
  int species;              /* index into the last dim of conc                   */
} hd_attenuator;

/* coordinate kinds: kwargs["wavelength"] [um] or kwargs["wavenumber"] [cm^-1]
 * (wavelength = 1e4 / wavenumber, s8_fuller.cpp:79-85) */
#define HD_COORD_WAVELENGTH 0
#define HD_COORD_WAVENUMBER 1

/* out [nwave][ncol][nlyr][2]: [0] = k(lambda) c, [1] = ssa(lambda) k(lambda) c
 * conc [ncol][nlyr][nspecies] mol/m^3 */
int hd_attenuate(const hd_attenuator *att, const double *coord, int coord_kind, int nwave,
                 const double *conc, int ncol, int nlyr, int nspecies, double *out,
                 void *stream);

/* prop [nwave][ncol][nlyr][nprop] (nprop >= 2): [0] = dz sum_a k_a c_a (layer
 * optical thickness), [1] = sum_a ssa_a k_a c_a / sum_a k_a c_a (0 where the
 * layer has no extinction; the reference divides 0/0 there), [2..] = 0.
 * dz [ncol][nlyr] m */
int hd_band_optics(const hd_attenuator *atts, int natt, const double *coord, int coord_kind,
                   int nwave, const double *conc, int ncol, int nlyr, int nspecies,
                   const double *dz, int nprop, double *prop, void *stream);

/* RadiationBandImpl::forward's optics mixing (src/radiation/radiation_band.cpp:86-116,
 * the "band loop") on the device, written straight into the solver layout
 *   prop [nwave][ncol][nlyr][2+nmom].
 * Each attenuator a contributes kdata_a = [k_a(lambda) c_a, ssa_a(lambda),
 * chi_a1..chi_anmom] with Henyey-Greenstein moments chi_al = g_a(lambda)^l (k, ssa and
 * g interpolated in wavelength as hd_attenuate does); per element, in this order
 * (ext0 first, then the attenuators in array order; products left to right, no
 * fused multiply-adds):
 *   ext  = ext0 + sum_a k_a c_a                     (radiation_band.cpp:91)
 *   sca  = sum_a ssa_a * (k_a c_a)                  (:94-96)
 *   m_l  = sum_{a with g} (chi_al * ssa_a) * (k_a c_a)  (:98-103)
 *   prop[2+l-1] = m_l / (sca + 1e-10)               (:108-110)
 *   prop[1]     = sca / (ext + 1e-10)               (:112-114)
 *   prop[0]     = ext * dz                          (:116)
 * ext0: [nwave][ncol][nlyr] extinction of attenuators without ssa (nprop = 1, e.g.
 * hd_rfm_attenuate's output), or NULL.  Latent reference bugs not reproduced
 * (SURVEY.md 3.3): prop there lacks the wave axis (:83-84) and the aerosol
 * modules' slot 1 is already ssa*k*c (s8_fuller.cpp:113-114), which the loop
 * would weight by k*c a second time -- here slot 1 of an attenuator is its ssa. */
typedef struct hd_band_attenuator {
  hd_attenuator table;  /* k_ext, ssa vs wavelength (as hd_attenuate)               */
  const double *gasym;  /* [table.nrow] HG asymmetry g(lambda), or NULL: no moments  */
} hd_band_attenuator;

int hd_band_loop_optics(const hd_band_attenuator *atts, int natt, const double *ext0,
                        const double *coord, int coord_kind, int nwave, const double *conc,
                        int ncol, int nlyr, int nspecies, const double *dz, int nmom,
                        double *prop, void *stream);

/* one RFM absorption table (harp::RFMImpl after reset(), src/opacity/rfm.cpp:30-120;
 * the reference reads it from netCDF: dims Wavenumber/Pressure/TempGrid, variables
 * of the same names, the reference Temperature profile and one variable per
 * species).  All arrays are DEVICE pointers. */
typedef struct hd_rfm_table {
  int nwave, npres, ntemp;
  const double *wave;  /* [nwave] wavenumber axis                                */
  const double *lnp;   /* [npres] ln(pressure [Pa]) axis (the reference's log_)   */
  const double *tgrid; /* [ntemp] temperature-anomaly axis [K]                     */
  const double *tref;  /* [npres] reference temperature profile [K]               */
  const double *kdata; /* [nwave][npres][ntemp] ln(m^2/kmol)                       */
  int species;         /* index into the last dim of conc                         */
} hd_rfm_table;

/* harp::RFMImpl::forward (rfm.cpp:122-197): out [nwave][ncol][nlyr] (nprop = 1) =
 * 1e-3 exp(interpn(kdata; wave_w, ln p, T - T_ref(ln p))) conc[..][species];
 * pres [Pa], temp [K]: [ncol][nlyr]; conc [ncol][nlyr][nspecies] mol/m^3 */
int hd_rfm_attenuate(const hd_rfm_table *t, const double *conc, int ncol, int nlyr,
                     int nspecies, const double *pres, const double *temp, double *out,
                     void *stream);

/* bflux [ncol][nlev][2] = sum_w weight[w] flux[w][ncol][nlev][2] (fixed order) */
int hd_band_flux(const double *flux, const double *weight, int nwave, int ncol, int nlev,
                 double *bflux, void *stream);

/* dTdt [ncol][nlyr] K/s from bflux [ncol][nlyr+1][2], dz and rho [ncol][nlyr] */
int hd_heating_rate(const double *bflux, const double *dz, const double *rho, double cp,
                    int ncol, int nlyr, double *dTdt, void *stream);

/* in place on bflux [ncol][nlev][2] (both directions); x1f, area [nlev],
 * vol [nlev-1], level 0 = bottom as in harp */
int hd_spherical_flux_correction(double *bflux, const double *x1f, const double *area,
                                 const double *vol, int ncol, int nlev, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* HDHARP_H_ */
