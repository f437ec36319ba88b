/*
 * hdisort.h -- C-ABI of the MI355X-native flux-only discrete-ordinate
 * radiative-transfer solver (libhdisort.so, HIP kernels for gfx950).
 *
 * This is the drop-in boundary for pyharp's RT-solver plugin path.  It
 * replaces, for the flux-only case (onlyfl, lamber, azimuthal mode m=0):
 *
 *   - pydisort's batch driver  disort::DisortImpl::forward(prop, &bc[, temf])
 *       [EXTERNAL, pydisort @ afee3ec897f, cmake/pydisort.cmake:9-11]
 *     called at examples/amars_sw.cpp:280, examples/amars_lw.cpp:80,
 *     tests/test_disort.cpp:49, src/radiation/radiation_band.cpp:124-127,
 *     behind the plugin signature RTSolverImpl::forward(prop, bc, temf)
 *     (src/rtsolver/rtsolver.hpp:25-29);
 *   - the per-column cdisort call  c_disort(&ds_, &ds_out_)
 *     (legacy site src/rtsolver/rt_solver_disort.cpp_:147,234).
 *
 * Layouts follow the harp call sites:
 *   prop  [nwave][ncol][nlyr][nprop] f64, layer 0 = bottom
 *         slot 0 = layer optical thickness, 1 = single-scattering albedo,
 *         2.. = phase moments chi_1..chi_nmom (chi_0 = 1 implicit)
 *         (src/index.h:12-18, src/radiation/radiation_band.cpp:116)
 *   bc    per-solve arrays [nwave][ncol] f64 (NULL = default): fbeam (0),
 *         umu0 (1), albedo (0), btemp (0), ttemp (0), temis (0), fisot (0);
 *         umu0 is used as given, as pydisort hands it to cdisort: with fbeam > 0
 *         a umu0 outside (0, 1] is cdisort's input error (c_chekin) and sets
 *         HD_STATUS_BAD_INPUT (harp's legacy driver floored umu0 at 1e-3 on its
 *         side, rt_solver_disort.cpp_:80; such a caller clamps umu0 itself)
 *         (src/radiation/radiation_band.hpp:74-77, amars_sw.cpp:276-278,
 *          amars_lw.cpp:73-74)
 *   temf  [ncol][nlyr+1] f64 level temperatures, level 0 = bottom (planck)
 *         (amars_lw.cpp:76, src/utils/layer2level.hpp:41)
 *   wave_lower/upper [nwave] f64 wavenumber bounds [cm^-1] (planck): one entry
 *         per wave of prop -- the kernels read index w for every w < nwave
 *   flux  [nwave][ncol][nlyr+1][2] f64, level 0 = surface,
 *         [..][0] = upward flux, [..][1] = rfldir + rfldn
 *         (src/rtsolver/rt_solver_disort.cpp_:172-181, amars_sw.cpp:185-191)
 * All array pointers are DEVICE pointers (hipMalloc / torch cuda tensors).
 *
 * Errors never cross the ABI as exceptions: every entry point returns an
 * hd_status code; hd_last_error() gives the message.
 *
 * Threading: a context may be shared by several modules, streams
 * and host threads.  Each entry point holds the context's mutex while it
 * enqueues, and every solve starts behind the previous solve on the context
 * (an event on that solve's stream), so the context's scratch is never used by
 * two solves at once.  Calls captured into a HIP graph are ordered by the
 * stream the graph is replayed on instead.  The entry points restore the
 * caller's current device.  For concurrency across host threads use one context
 * per (device, thread), as the bindings do.
 */
#ifndef HDISORT_H_
#define HDISORT_H_

#ifdef __cplusplus
extern "C" {
#endif

#define HDISORT_VERSION 100 /* 1.0.0 */

/* Flags of the pydisort flag string (bindings): lamber
 * (required), onlyfl, planck, usrtau, usrang, intensity_correction +
 * old_intensity_correction, quiet, print-* are honoured; ibcnd is refused as
 * harp's driver refuses it (src/rtsolver/rt_solver_disort.cpp_:67-68), and so
 * are spher, general_source, output_uum and the new intensity correction
 * (not implemented); unknown names are refused. */

/* return codes */
#define HD_OK 0
#define HD_EINVAL 1    /* bad argument / shape / flag                         */
#define HD_ENUMERIC 2  /* at least one solve set an error bit (see status)    */
#define HD_EHIP 3      /* HIP runtime error                                   */
#define HD_ENOMEM 4    /* device allocation failed                            */

/* hd_config.flags (subset of the pydisort flag string that this path keeps) */
#define HD_FLAG_LAMBER 0x1u /* Lambertian lower boundary (always on)          */
#define HD_FLAG_PLANCK 0x2u /* thermal emission (needs temf, wave bounds)     */
#define HD_FLAG_ONLYFL 0x4u /* fluxes only (always on: the only mode here)    */

/* per-solve status bits (int32 per solve) */
#define HD_STATUS_BAD_INPUT 0x01 /* tau<0, ssa outside [0,1], f>=1, a beam with
                                    umu0 outside (0,1], albedo outside [0,1] ... */
#define HD_STATUS_EIGEN 0x02     /* eigenvalue <= 0 / Cholesky breakdown / Jacobi
                                    not converged within the sweep cap          */
#define HD_STATUS_NONFINITE 0x04 /* NaN/Inf produced                             */
#define HD_STATUS_RESONANCE 0x10 /* warning: umu0 ~ 1/k (beam/quadrature resonance) */
#define HD_STATUS_PIVOT 0x20     /* warning: tiny pivot in the boundary sweep      */
#define HD_STATUS_ERROR_MASK 0x0F

typedef struct hd_config {
  int nstr;       /* number of streams, even, 2..32 (a limit of this boundary:
                     nstr > 32 is rejected with HD_EINVAL) */
  int nmom;       /* phase moments the module was configured with (>= 0)   */
  int nlyr;       /* layers                                                 */
  int nprop;      /* last-dim size of prop (>= 1); moments used = min(nmom, nprop-2) */
  unsigned flags; /* HD_FLAG_*                                              */
} hd_config;

typedef struct hd_inputs {
  int nwave, ncol;
  const double *prop;
  const double *fbeam, *umu0, *albedo, *btemp, *ttemp, *temis, *fisot;
  const double *temf;
  const double *wave_lower, *wave_upper;
} hd_inputs;

/* per-kernel device time accumulated since hd_context_set_timing(ctx, 1): HIP events
 * recorded on the solve stream around every launch, resolved lazily by get_timing */
typedef struct hd_timing {
  double layer_ms;  /* sum over launches of hd_layer_kernel (per-layer setup)  */
  double sweep_ms;  /* sum over launches of hd_sweep_kernel (boundary sweep)   */
  int layer_launches;
  int sweep_launches;
} hd_timing;

typedef struct hd_context hd_context;

int hd_version(void);
/* ctx may be NULL (the last error of any call).  The string is a copy owned by the
 * calling thread, valid until that thread calls hd_last_error again. */
const char *hd_last_error(const hd_context *ctx);

int hd_context_create(hd_context **ctx, int device);
int hd_context_destroy(hd_context *ctx);
/* max solves per internal chunk (scratch = chunk*nlyr*~1.4 KB); 0 = auto */
int hd_context_set_chunk(hd_context *ctx, long max_solves);
int hd_context_set_timing(hd_context *ctx, int enable);
/* debug: cap on the eigensolver's Jacobi sweeps (0 = default 16).  A solve whose
 * Jacobi is still rotating at the cap sets HD_STATUS_EIGEN. */
int hd_context_set_max_sweeps(hd_context *ctx, int max_sweeps);
int hd_context_get_timing(const hd_context *ctx, hd_timing *out);
/* pre-size scratch for graph capture / steady state: room for hd_solve and for
 * hd_solve_band (any nwave) of up to nsolve solves of this config (with its per-point
 * flux buffer when nsolve takes hd_solve_band's row-major route), and the status
 * buffer.  A call captured into a HIP graph never allocates: if scratch would
 * have to grow during capture it returns HD_EINVAL instead. */
int hd_context_reserve(hd_context *ctx, const hd_config *cfg, long nsolve);
/* solves per internal chunk of an nsolve-solve call of this config under the automatic
 * chunking (hd_context_set_chunk 0): nstr <= 16 about 32 768 when that gives five or
 * more chunks, otherwise about 40 960 (a chunk's sweep leaves SIMDs to the next chunk's
 * layer kernel), nstr 18..32 from a 16 GB scratch budget (about 16 000 at nlyr 80); a
 * call that fits one chunk stays one.  Chunk k+1's layer kernel runs beside chunk k's
 * sweep.  No device needed; -1 on bad args. */
long hd_chunk_solves(const hd_config *cfg, long nsolve);

/*
 * Solve every (wave, column) flux problem of the batch on `stream`
 * (hipStream_t passed as void*; NULL = default stream).
 * status: device int32[nwave*ncol] or NULL.  With NULL the call is
 * synchronous and returns HD_ENUMERIC if any solve set an error bit; with a
 * caller buffer the call is asynchronous and the caller inspects it.
 */
int hd_solve(hd_context *ctx, const hd_config *cfg, const hd_inputs *in, double *flux,
             int *status, void *stream);

/*
 * Fused band epilogue: the solve of hd_solve plus the
 * weighted sum over the wave axis that every harp caller applies next --
 *   bflux[c][lev][dir] = sum_w weight[w] flux[w][c][lev][dir]
 * (examples/amars_lw.cpp:84-88 `(flux * weights.view({-1,1,1,1})).sum(0)`,
 * examples/amars_sw.cpp:169-196 with weight = d(wavenumber); legacy
 * src/rtsolver/rt_solver_disort.cpp_:183-184).  For nstr <= 16 the sum is
 * formed in the back-substitution epilogue (solves taken column by column,
 * the weighted fluxes of a column summed across lanes), so the per-point
 * fluxes never reach memory; for nstr 18..32 each chunk's fluxes are summed
 * into bflux after the chunk.  Exception, for nstr <= 16 with flux NULL and
 * five or more automatic chunks (C4's regime): the solves run in hd_solve's
 * row-major chunks into a per-point flux buffer of the context (nwave*ncol*
 * (nlyr+1)*2 doubles, sized by hd_context_reserve too) and hd_band_flux sums
 * them -- faster there than the column-order epilogue, and bitwise equal to
 * hd_solve + hd_band_flux.  The summation order is fixed (deterministic
 * for a given shape and chunk size; no atomics).  Heating rates and the
 * spherical correction follow from bflux (hdharp.h) -- after the cross-rank
 * all-reduce when a band's points are sharded over GPUs.
 *   band->weight  DEVICE [nwave]
 *   band->bflux   DEVICE [ncol][nlyr+1][2], overwritten
 *   flux          DEVICE [nwave][ncol][nlyr+1][2] or NULL (per-point fluxes
 *                 are then not stored)
 * status / stream / return codes as hd_solve.
 */
typedef struct hd_band {
  const double *weight;
  double *bflux;
} hd_band;

int hd_solve_band(hd_context *ctx, const hd_config *cfg, const hd_inputs *in,
                  const hd_band *band, double *flux, int *status, void *stream);

/*
 * The same two solves on HOST arrays (pydisort's own contract: CPU tensors in,
 * a CPU tensor out -- DisortImpl::forward [EXTERNAL] at
 * examples/amars_sw.cpp:280, examples/amars_lw.cpp:80, tests/test_disort.cpp:49,
 * src/radiation/radiation_band.cpp:124-127, all with CPU tensors).  Every
 * hd_inputs pointer (and weight) is a host pointer; the arrays are copied to a
 * device staging area of the context in pieces of whole waves (~128 k solves;
 * piece j+1's copy beside piece j's solve), each piece solved on the device
 * exactly as hd_solve / hd_solve_band (the band sum: the pieces' partial sums
 * added in piece order), and flux / bflux / status copied back.  Synchronous;
 * HD_ENUMERIC if any solve set an error bit (status, host int32[nwave*ncol],
 * may be NULL).  No CPU arithmetic: without a device they fail as hd_solve does.
 *   hd_solve_band_host: weight HOST [nwave]; bflux HOST [ncol][nlyr+1][2]
 *   (required); flux HOST per-point fluxes or NULL.
 */
int hd_solve_host(hd_context *ctx, const hd_config *cfg, const hd_inputs *in, double *flux,
                  int *status);
int hd_solve_band_host(hd_context *ctx, const hd_config *cfg, const hd_inputs *in,
                       const double *weight, double *bflux, double *flux, int *status);

/*
 * Intensity path (flags usrtau / usrang, onlyfl off): pydisort's forward with
 * radiances and DisortImpl::get_rad [EXTERNAL], as called at
 * tests/test_disort.cpp:13-55 (user_mu, user_phi, user_tau; get_rad at :52)
 * and by the legacy driver src/rtsolver/rt_solver_disort.cpp_:210-286
 * (c_disort, then ds_out_.uu interpolated onto outgoing rays).  Every
 * azimuthal mode m < nstr (mode 0 only without a beam), every nstr 2..32
 * (nstr 18..32: the same kernels with their per-lane matrices in private memory).
 *
 *   utau   HOST [ntau] user optical depths (unscaled, >= 0, ascending);
 *          ntau = 0: the nlyr+1 layer boundaries of every column
 *   umu    HOST [numu] user polar cosines, nonzero, > 0 upward
 *   phi    HOST [nphi] user azimuths [deg]
 *   phi0   DEVICE [nwave*ncol] beam azimuth [deg] or NULL (0)
 *   onlyfl 1: fluxes at the user depths only (uu untouched)
 *   corint 1: Nakajima-Tanaka correction of the beam radiances (cdisort with
 *          intensity_correction AND old_intensity_correction; DISORT 2.0 INTCOR):
 *          TMS (exact single scattering, STWL eq. 68) plus, for downward
 *          directions, minus the IMS secondary-scattering term (STWL A.13-A.16);
 *          0: none.  Any other value is HD_EINVAL: cdisort's new
 *          (Buras-Emde-Dowling) correction -- intensity_correction without
 *          old_intensity_correction -- is not implemented, and the bindings
 *          refuse that flag combination when radiances are requested.
 * Not capturable into a HIP graph (HD_EINVAL under capture): the user grid is
 * copied from host arrays.
 * Outputs (device):
 *   flux [nwave][ncol][ntau][2]  index 0 = the deepest user depth (harp order,
 *        as the level fluxes of hd_solve), [..][0] up, [..][1] rfldir + rfldn
 *   uu   [nwave][ncol][nphi][ntau][numu]  radiance, user order
 *        (cdisort's uu[j][lu][iu] per solve)
 */
typedef struct hd_radiance {
  int ntau;
  const double *utau;
  int numu;
  const double *umu;
  int nphi;
  const double *phi;
  const double *phi0;
  int onlyfl;
  int corint;
} hd_radiance;

int hd_solve_radiance(hd_context *ctx, const hd_config *cfg, const hd_inputs *in,
                      const hd_radiance *rad, double *flux, double *uu, int *status,
                      void *stream);

/* host helper: the double-Gauss quadrature the kernels use (nstr/2 nodes on (0,1)) */
int hd_quadrature(int nstr, double *mu, double *w);

#ifdef __cplusplus
}
#endif
#endif /* HDISORT_H_ */
