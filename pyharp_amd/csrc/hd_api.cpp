// hd_api.cpp -- C-ABI of libhdisort.so (include/hdisort.h): argument
// validation, quadrature constants, scratch management, chunked launches,
// per-solve status, optional per-kernel timing with HIP events.
//
// Replaces pydisort's DisortImpl::forward batch loop over (nwave, ncol)
// [EXTERNAL, pydisort @ afee3ec897f] and its per-column c_disort calls
// (legacy: src/rtsolver/rt_solver_disort.cpp_:147,234; error behaviour:
// nonzero c_disort -> "DisortWrapper::Run failed.", :149-151).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hdharp.h"
#include "../../include/hdisort.h"
#include "hd_kernels.hpp"
#include "hd_team_prims.hpp"
#include "hd_rad.hpp"

struct hd_context {
  int device = 0;
  double* scratch = nullptr;
  size_t scratch_doubles = 0;
  // per-g fluxes of hd_solve_band's row-major route (band_rowmajor)
  double* pflux = nullptr;
  size_t pflux_doubles = 0;
  int band_cmaj = 0;  // A/B (HD_BAND_CMAJ=1): always the column-major fused epilogue
  int* status = nullptr;  // internal per-solve status (when caller passes NULL)
  size_t status_len = 0;
  int* anyerr = nullptr;
  long chunk = 0;  // 0 = auto
  bool timing = false;
  // timing: one event triple per launched chunk, resolved lazily in get_timing
  std::vector<hipEvent_t> pool;
  size_t pool_used = 0;
  hd_timing times{};
  int max_sweeps = 16;  // Jacobi sweep cap (debug setter: hd_context_set_max_sweeps)
  // team-path Jacobi from the tabulated (ssa, chi_1) eigenvectors
  // (hd_kernels.hpp); HD_JACOBI_WARM=0 in the environment turns it off (A/B)
  int warm = 1;
  // team path: the two-waves-per-SIMD sweep (hd_team_mfma_sweep_lean_kernel, the
  // default); HD_TEAM_SWEEP_LEAN=0 in the environment picks the one-wave sweep when
  // a context is created
  int lean = 1;
  // nstr 4 / 8: the sweep in NN-lane teams (hd_sweep_quad_kernel) for chunks of at
  // most kQuadMaxSolves solves (-1, the default), always (1) or never (0): HD_SWEEP_QUAD
  int quad = -1;
  // nstr 16: the adding sweep with the stack state in LDS (hd_sweep_lean_kernel,
  // two waves per SIMD) -- off by default: 1 024 waves per chunk spread one per SIMD
  // and each runs 1.85 ms against hd_sweep_kernel's 1.4 (C4 12.38 vs 12.77 M,
  // profiles/r05/lean8_ab.txt); HD_AB=1 HD_SWEEP_LEAN8=1 picks it
  int lean8 = 0;
  // nstr 16: layer setup, adding sweep and back-substitution of a chunk in one kernel
  // (hd_column_kernel: no layer records in HBM); HD_AB=1 HD_COLUMN=0|1
  int column = 0;
  // true while a solve enqueues into a capturing stream: scratch may not grow then
  bool capturing = false;
  std::string err;
  std::mutex err_mu;  // guards err (hd_last_error reads it without the solve lock)
  // register path: back-substitution of chunk k on `side`, beside chunk k+1's
  // layer kernel (its 44-VGPR waves fit next to the layer kernel's on a SIMD)
  hipStream_t side = nullptr;
  // register path: chunk k+1's layer kernel on its own stream, beside chunk k's
  // sweep (it takes the SIMDs a partial sweep leaves idle)
  hipStream_t lay = nullptr;
  hipEvent_t ev_layer[2] = {nullptr, nullptr};
  hipEvent_t ev_sweep[2] = {nullptr, nullptr};
  hipEvent_t ev_back[2] = {nullptr, nullptr};
  hipEvent_t ev_pro[2] = {nullptr, nullptr};  // next chunk's prologue done (side stream)
  hipEvent_t ev_fork = nullptr;                // start of a solve on the caller's stream
  double* sink = nullptr;                      // team kernels: stores of lanes >= nstr/2
  double* rad_grid = nullptr;                  // device copies of umu | phi | utau
  size_t rad_grid_len = 0;
  // Serialisation of the context's scratch (SURVEY 8(b) "Threading"): every
  // entry point holds `mu` while it enqueues, and every solve starts behind
  // `ev_done`, recorded on the caller's stream at the end of the previous
  // solve -- so two modules sharing this context from two streams (or two
  // host threads) never touch scratch/status/anyerr concurrently.
  std::mutex mu;
  hipEvent_t ev_done = nullptr;
  bool done_valid = false;
  // hd_solve_host / hd_solve_band_host: device copies of the caller's host arrays
  double* hstage = nullptr;
  size_t hstage_len = 0;  // doubles
  hipStream_t hstream = nullptr;   // host<->device copies
  hipStream_t hstream2 = nullptr;  // the pieces' solves
  hipStream_t hstream3 = nullptr;  // device->host copies (PCIe is full duplex: beside the uploads)
  hipEvent_t hev_in[2] = {nullptr, nullptr};
  hipEvent_t hev_done[2] = {nullptr, nullptr};
};

namespace {

std::mutex g_err_mu;
std::string g_err;

int fail(hd_context* ctx, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (ctx) {
    std::lock_guard<std::mutex> lk(ctx->err_mu);
    ctx->err = buf;
  }
  std::lock_guard<std::mutex> lk(g_err_mu);
  g_err = buf;
  return code;
}

#define HD_HIP(ctx, call)                                                                   \
  do {                                                                                      \
    hipError_t e_ = (call);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return fail(ctx, HD_EHIP, "%s failed: %s", #call, hipGetErrorString(e_));            \
  } while (0)

// Gauss-Legendre nodes/weights on (0,1), ascending (double-Gauss half range).
void gauss01(int nn, double* mu, double* w) {
  const double pi = 3.14159265358979323846;
  for (int i = 0; i < (nn + 1) / 2; ++i) {
    double x = std::cos(pi * (i + 0.75) / (nn + 0.5));
    double dp = 1.0;
    for (int it = 0; it < 100; ++it) {
      double p0 = 1.0, p1 = x;
      for (int l = 2; l <= nn; ++l) {
        double p2 = ((2 * l - 1) * x * p1 - (l - 1) * p0) / l;
        p0 = p1;
        p1 = p2;
      }
      dp = nn * (x * p1 - p0) / (x * x - 1.0);
      double dx = p1 / dp;
      x -= dx;
      if (std::fabs(dx) < 1e-16) break;
    }
    {
      double p0 = 1.0, p1 = x;
      for (int l = 2; l <= nn; ++l) {
        double p2 = ((2 * l - 1) * x * p1 - (l - 1) * p0) / l;
        p0 = p1;
        p1 = p2;
      }
      dp = nn * (x * p1 - p0) / (x * x - 1.0);
    }
    const double wx = 2.0 / ((1.0 - x * x) * dp * dp);
    mu[nn - 1 - i] = 0.5 * (1.0 + x);
    w[nn - 1 - i] = 0.5 * wx;
    mu[i] = 0.5 * (1.0 - x);
    w[i] = 0.5 * wx;
  }
}

void make_quad(int nn, hd::QuadHost& q) {
  std::memset(&q, 0, sizeof(q));
  gauss01(nn, q.mu, q.w);
  for (int i = 0; i < nn; ++i) {
    q.sd[i] = std::sqrt(q.w[i] / q.mu[i]);
    q.g[i] = std::sqrt(q.w[i] * q.mu[i]);
    double p0 = 1.0, p1 = q.mu[i];
    q.pt[0][i] = 1.0;
    if (2 * nn > 1) q.pt[1][i] = p1;
    for (int l = 2; l < 2 * nn; ++l) {
      double p2 = ((2 * l - 1) * q.mu[i] * p1 - (l - 1) * p0) / l;
      q.pt[l][i] = p2;
      p0 = p1;
      p1 = p2;
    }
  }
}

// The quadrature tables of every nn, built once per process; their upload into a
// device's __constant__ memory happens once per device (the module's constants
// are per device, shared by every context on it), under one global lock.
const hd::QuadHost* quad_host() {
  static hd::QuadHost all[hd::kMaxNN];
  static std::once_flag once;
  std::call_once(once, [] {
    for (int nn = 1; nn <= hd::kMaxNN; ++nn) make_quad(nn, all[nn - 1]);
  });
  return all;
}

constexpr int kMaxDevices = 64;
std::mutex g_tab_mu;
bool g_tables[kMaxDevices] = {};      // flux-path tables uploaded, per device
bool g_rad_tables[kMaxDevices] = {};  // intensity-path tables uploaded, per device

int ensure_tables(hd_context* ctx) {
  if (ctx->device < 0 || ctx->device >= kMaxDevices)
    return fail(ctx, HD_EINVAL, "hd_solve: device %d beyond the table cache", ctx->device);
  std::lock_guard<std::mutex> lk(g_tab_mu);
  if (g_tables[ctx->device]) return HD_OK;
  const hd::QuadHost* all = quad_host();
  hipError_t e = hd::upload_quad_tables(all);
  if (e == hipSuccess) e = hd::upload_quad_tables_team(all);
  if (e == hipSuccess) e = hd::upload_warm_tables_team(all);
  if (e != hipSuccess) return fail(ctx, HD_EHIP, "hd_solve: constant upload: %s", hipGetErrorString(e));
  g_tables[ctx->device] = true;
  return HD_OK;
}

int ensure_rad_tables(hd_context* ctx) {
  int rc = ensure_tables(ctx);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_tab_mu);
  if (g_rad_tables[ctx->device]) return HD_OK;
  hipError_t e = hd::upload_rad_tables(quad_host());
  if (e == hipSuccess) e = hd::upload_rad_tables_team(quad_host());
  if (e != hipSuccess)
    return fail(ctx, HD_EHIP, "hd_solve_radiance: constant upload: %s", hipGetErrorString(e));
  g_rad_tables[ctx->device] = true;
  return HD_OK;
}

constexpr long kRegChunkMax = 40960;  // the register path's largest automatic chunk

// team path: bytes of scratch for the two chunks in flight (the per-solve size counts
// both) within a 16 GB budget
long team_chunk_target(int nn, int nlyr, bool planck) {
  const double budget = 16.0 * 1024.0 * 1024.0 * 1024.0;
  const double per = 8.0 * (double)hd::scratch_doubles_per_solve(nn, nlyr, planck);
  return std::min<long>(262144, std::max<long>(16384, (long)(budget / per)));
}

long auto_chunk(long nsolve, int nn, int nlyr, bool planck) {
  // NN <= 8: the sweep runs one lane per solve at one wave per SIMD (its register
  // file is full) and cannot share a SIMD with the layer kernel.  Chunks of 32 000-
  // 40 000 solves (500-625 sweep waves) leave 40-50 % of the SIMDs to the next chunk's
  // layer kernel while a sweep runs, instead of the 1 024 waves of a 65 536-solve chunk
  // that take every SIMD: C4 12.80 -> 13.35 M solves/s at 20 chunks of 32 000 (16 of
  // 40 000: 13.27; 24-28 chunks: 12.96-13.03).  With fewer than five chunks the
  // pipeline's fill and drain dominate and the larger chunk wins: the 8-GPU rank shape
  // (80 000) runs 2 x 40 000 at 12.15 M, 3 x 26 667 at 11.78
  // (profiles/r05/chunk_sweep.txt).
  // NN > 8: one 16-lane team per solve; chunks bounded by a scratch budget
  // (the rest of the 288 GB stays the caller's).
  long target;
  if (nn <= hd::kMaxRegNN) {
    target = (nsolve + 32767) / 32768 >= 5 ? 32768 : kRegChunkMax;
  } else {
    target = team_chunk_target(nn, nlyr, planck);
  }
  // (team path: a call that fits one chunk stays one chunk.  Split in two, the 8-GPU
  // C5 rank shape -- 8 000 solves -- ran 1.155 M solves/s against 1.268 M: a 4 000-solve
  // layer kernel takes 2.57 ms alone and 3.63 ms beside the first chunk's sweep,
  // against 4.59 ms for all 8 000, profiles/r05/c5_rank_shape.txt)
  if (nsolve <= target) return nsolve;
  const long n = (nsolve + target - 1) / target;
  return (nsolve + n - 1) / n;
}

// The largest chunk auto_chunk gives any call of at most nsolve solves (the chunk
// size is not monotone in nsolve: 163 840 solves run in chunks of 32 768, 80 000 in
// chunks of 40 000), so hd_context_reserve(nsolve) covers every smaller call too.
// hd_solve_band without caller fluxes on the register path, when the call runs as the
// three-stream pipeline of five or more automatic chunks (the 32 768-solve regime): the
// row-major chunks of hd_solve into a per-g flux buffer of the context, then
// hd_band_flux.  C4: 14.80-14.92 M solves/s against 14.33-14.45 M for the column-major
// fused epilogue on one box (profiles/r06/fuse_ab.txt); the 8-GPU rank shape (two
// chunks) is equal and the small shapes keep the fused epilogue.
bool band_rowmajor(const hd_context* ctx, int nn, long nsolve) {
  return nn <= hd::kMaxRegNN && ctx->chunk <= 0 && !ctx->band_cmaj && !ctx->column &&
         (nsolve + 32767) / 32768 >= 5;
}

long max_auto_chunk(long nsolve, int nn, int nlyr, bool planck) {
  const long cap = nn <= hd::kMaxRegNN ? kRegChunkMax : team_chunk_target(nn, nlyr, planck);
  return std::min(nsolve, cap);
}

// the last solve that used the context's buffers has finished (before a free)
void drain(hd_context* ctx) {
  if (ctx->done_valid) (void)hipEventSynchronize(ctx->ev_done);
}

// Growing a buffer frees the old one, which a captured graph may still point at,
// and a free/malloc cannot be captured: during capture growth is an error (size
// the context first with hd_context_reserve, or run the call once eagerly).
int ensure_scratch(hd_context* ctx, size_t ndoubles) {
  if (ctx->scratch_doubles >= ndoubles) return HD_OK;
  if (ctx->capturing)
    return fail(ctx, HD_EINVAL,
                "hd_solve: scratch must grow to %zu bytes inside a stream capture; size the "
                "context first (hd_context_reserve, or one eager call of the same shape)",
                ndoubles * sizeof(double));
  drain(ctx);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  ctx->scratch = nullptr;
  ctx->scratch_doubles = 0;
  if (hipMalloc(&ctx->scratch, ndoubles * sizeof(double)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(ctx, HD_ENOMEM, "hd_solve: cannot allocate %zu bytes of scratch",
                ndoubles * sizeof(double));
  }
  ctx->scratch_doubles = ndoubles;
  return HD_OK;
}

int ensure_pflux(hd_context* ctx, size_t ndoubles) {
  if (ctx->pflux_doubles >= ndoubles) return HD_OK;
  if (ctx->capturing)
    return fail(ctx, HD_EINVAL,
                "hd_solve_band: the per-g flux buffer must grow to %zu bytes inside a stream "
                "capture; size the context first (hd_context_reserve, or one eager call of the "
                "same shape)", ndoubles * sizeof(double));
  drain(ctx);
  if (ctx->pflux) (void)hipFree(ctx->pflux);
  ctx->pflux = nullptr;
  ctx->pflux_doubles = 0;
  if (hipMalloc(&ctx->pflux, ndoubles * sizeof(double)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(ctx, HD_ENOMEM, "hd_solve_band: cannot allocate %zu bytes of per-g fluxes",
                ndoubles * sizeof(double));
  }
  ctx->pflux_doubles = ndoubles;
  return HD_OK;
}

int ensure_status(hd_context* ctx, size_t n) {
  if (ctx->status_len >= n) return HD_OK;
  if (ctx->capturing)
    return fail(ctx, HD_EINVAL,
                "hd_solve: the status buffer must grow inside a stream capture; pass a status "
                "buffer or size the context first (hd_context_reserve)");
  drain(ctx);
  if (ctx->status) (void)hipFree(ctx->status);
  ctx->status = nullptr;
  ctx->status_len = 0;
  if (hipMalloc(&ctx->status, std::max<size_t>(n, 1) * sizeof(int)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(ctx, HD_ENOMEM, "hd_solve: cannot allocate status buffer");
  }
  ctx->status_len = n;
  return HD_OK;
}

// fold every recorded (K1 start, K1 end, K2 start, K2 end) quadruple into the totals
int resolve_timing(hd_context* ctx) {
  for (size_t i = 0; i + 4 <= ctx->pool_used; i += 4) {
    HD_HIP(ctx, hipEventSynchronize(ctx->pool[i + 3]));
    float t1 = 0.f, t2 = 0.f;
    HD_HIP(ctx, hipEventElapsedTime(&t1, ctx->pool[i], ctx->pool[i + 1]));
    HD_HIP(ctx, hipEventElapsedTime(&t2, ctx->pool[i + 2], ctx->pool[i + 3]));
    ctx->times.layer_ms += t1;
    ctx->times.sweep_ms += t2;
    ctx->times.layer_launches += 1;
    ctx->times.sweep_launches += 1;
  }
  ctx->pool_used = 0;
  return HD_OK;
}

// restores the caller's current device on every return path (the entry points
// switch to the context's device)
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// A solve on `stream` starts after the previous solve on this context, whatever
// stream that one ran on.  Under stream capture the event is neither waited on
// nor recorded (an event recorded outside the graph cannot order a replay; a
// captured call is ordered by the stream its graph is replayed on).
int enter(hd_context* ctx, hipStream_t stream, bool* capturing) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HD_HIP(ctx, hipStreamIsCapturing(stream, &cs));
  *capturing = cs != hipStreamCaptureStatusNone;
  if (!*capturing && ctx->done_valid) HD_HIP(ctx, hipStreamWaitEvent(stream, ctx->ev_done, 0));
  return HD_OK;
}

int leave(hd_context* ctx, hipStream_t stream, bool capturing) {
  if (capturing) return HD_OK;
  HD_HIP(ctx, hipEventRecord(ctx->ev_done, stream));
  ctx->done_valid = true;
  return HD_OK;
}

int validate(hd_context* ctx, const hd_config* cfg, const hd_inputs* in, const double* flux) {
  if (!cfg || !in) return fail(ctx, HD_EINVAL, "hd_solve: null config/inputs");
  if (cfg->nstr < 2 || cfg->nstr % 2 || cfg->nstr / 2 > hd::kMaxNN)
    return fail(ctx, HD_EINVAL, "hd_solve: nstr=%d must be even and in [2, %d]", cfg->nstr,
                2 * hd::kMaxNN);
  if (cfg->nlyr < 1) return fail(ctx, HD_EINVAL, "hd_solve: nlyr=%d < 1", cfg->nlyr);
  if (cfg->nprop < 1) return fail(ctx, HD_EINVAL, "hd_solve: nprop=%d < 1", cfg->nprop);
  if (cfg->nmom < 0) return fail(ctx, HD_EINVAL, "hd_solve: nmom=%d < 0", cfg->nmom);
  if (cfg->flags & ~(HD_FLAG_LAMBER | HD_FLAG_PLANCK | HD_FLAG_ONLYFL))
    return fail(ctx, HD_EINVAL, "hd_solve: unsupported flags 0x%x", cfg->flags);
  if (in->nwave < 0 || in->ncol < 0)
    return fail(ctx, HD_EINVAL, "hd_solve: negative nwave/ncol");
  if ((long)in->nwave * in->ncol > 0 && (!in->prop || !flux))
    return fail(ctx, HD_EINVAL, "hd_solve: prop and flux are required");
  if ((cfg->flags & HD_FLAG_PLANCK) && (!in->temf || !in->wave_lower || !in->wave_upper))
    return fail(ctx, HD_EINVAL, "hd_solve: planck needs temf, wave_lower, wave_upper");
  if ((long)in->nwave * in->ncol > (long)0x7fffffff)
    return fail(ctx, HD_EINVAL, "hd_solve: nwave*ncol exceeds 2^31");
  return HD_OK;
}

}  // namespace

namespace hd {
int set_global_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  std::lock_guard<std::mutex> lk(g_err_mu);
  g_err = buf;
  return code;
}
}  // namespace hd

extern "C" {

int hd_version(void) { return HDISORT_VERSION; }

// A copy per calling thread: valid until this thread's next hd_last_error call,
// whatever other threads do to the context meanwhile.
const char* hd_last_error(const hd_context* ctx_) {
  static thread_local std::string copy;
  if (ctx_) {
    hd_context* ctx = const_cast<hd_context*>(ctx_);
    std::lock_guard<std::mutex> lk(ctx->err_mu);
    copy = ctx->err;
  } else {
    std::lock_guard<std::mutex> lk(g_err_mu);
    copy = g_err;
  }
  return copy.c_str();
}

int hd_context_create(hd_context** out, int device) {
  if (!out) return fail(nullptr, HD_EINVAL, "hd_context_create: null out");
  *out = nullptr;
  DeviceGuard guard;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    (void)hipGetLastError();
    return fail(nullptr, HD_EHIP, "hd_context_create: no HIP device available");
  }
  if (device < 0 || device >= ndev)
    return fail(nullptr, HD_EINVAL, "hd_context_create: device %d out of range (%d)", device,
                ndev);
  hd_context* ctx = new hd_context();
  if (const char* e = hd::ab_env("HD_JACOBI_WARM")) ctx->warm = std::atoi(e) != 0;
  if (const char* e = hd::ab_env("HD_SWEEP_QUAD")) ctx->quad = std::atoi(e) < 0 ? -1 : std::atoi(e) != 0;
  if (const char* e = hd::ab_env("HD_BAND_CMAJ")) ctx->band_cmaj = std::atoi(e) != 0;
#if HD_AB_VARIANTS
  if (const char* e = hd::ab_env("HD_TEAM_SWEEP_LEAN")) ctx->lean = std::atoi(e) != 0;
  if (const char* e = hd::ab_env("HD_SWEEP_LEAN8")) ctx->lean8 = std::atoi(e) != 0;
  if (const char* e = hd::ab_env("HD_COLUMN")) ctx->column = std::atoi(e) != 0;
#endif
  ctx->device = device;
  auto init = [ctx]() -> int {
    HD_HIP(ctx, hipSetDevice(ctx->device));
    HD_HIP(ctx, hipMalloc(&ctx->anyerr, sizeof(int)));
    HD_HIP(ctx, hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
    HD_HIP(ctx, hipStreamCreateWithFlags(&ctx->lay, hipStreamNonBlocking));
    HD_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
    HD_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_done, hipEventDisableTiming));
    HD_HIP(ctx, hipMalloc(&ctx->sink, 4096 * sizeof(double)));
    for (int b = 0; b < 2; ++b) {
      HD_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_layer[b], hipEventDisableTiming));
      HD_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_sweep[b], hipEventDisableTiming));
      HD_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_back[b], hipEventDisableTiming));
      HD_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_pro[b], hipEventDisableTiming));
    }
    return HD_OK;
  };
  const int rc = init();
  if (rc != HD_OK) {  // nothing leaks: destroy frees whatever init created
    std::string msg;
    {
      std::lock_guard<std::mutex> lk(ctx->err_mu);
      msg = ctx->err;
    }
    hd_context_destroy(ctx);
    return fail(nullptr, rc, "%s", msg.c_str());
  }
  *out = ctx;
  return HD_OK;
}

int hd_context_destroy(hd_context* ctx) {
  if (!ctx) return HD_OK;
  DeviceGuard guard;
  (void)hipSetDevice(ctx->device);
  drain(ctx);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->pflux) (void)hipFree(ctx->pflux);
  if (ctx->hstage) (void)hipFree(ctx->hstage);
  if (ctx->hstream) (void)hipStreamDestroy(ctx->hstream);
  if (ctx->hstream2) (void)hipStreamDestroy(ctx->hstream2);
  if (ctx->hstream3) (void)hipStreamDestroy(ctx->hstream3);
  for (int b = 0; b < 2; ++b) {
    if (ctx->hev_in[b]) (void)hipEventDestroy(ctx->hev_in[b]);
    if (ctx->hev_done[b]) (void)hipEventDestroy(ctx->hev_done[b]);
  }
  if (ctx->status) (void)hipFree(ctx->status);
  if (ctx->anyerr) (void)hipFree(ctx->anyerr);
  for (int b = 0; b < 2; ++b) {
    if (ctx->ev_layer[b]) (void)hipEventDestroy(ctx->ev_layer[b]);
    if (ctx->ev_sweep[b]) (void)hipEventDestroy(ctx->ev_sweep[b]);
    if (ctx->ev_back[b]) (void)hipEventDestroy(ctx->ev_back[b]);
    if (ctx->ev_pro[b]) (void)hipEventDestroy(ctx->ev_pro[b]);
  }
  if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
  if (ctx->ev_done) (void)hipEventDestroy(ctx->ev_done);
  if (ctx->sink) (void)hipFree(ctx->sink);
  if (ctx->rad_grid) (void)hipFree(ctx->rad_grid);
  if (ctx->side) (void)hipStreamDestroy(ctx->side);
  if (ctx->lay) (void)hipStreamDestroy(ctx->lay);
  for (auto& e : ctx->pool)
    if (e) (void)hipEventDestroy(e);
  delete ctx;
  return HD_OK;
}

int hd_context_set_chunk(hd_context* ctx, long max_solves) {
  if (!ctx || max_solves < 0) return fail(ctx, HD_EINVAL, "hd_context_set_chunk: bad args");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->chunk = max_solves;
  return HD_OK;
}

int hd_context_set_max_sweeps(hd_context* ctx, int max_sweeps) {
  if (!ctx || max_sweeps < 0 || max_sweeps > 64)
    return fail(ctx, HD_EINVAL, "hd_context_set_max_sweeps: bad args");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->max_sweeps = max_sweeps > 0 ? max_sweeps : 16;
  return HD_OK;
}

int hd_context_set_timing(hd_context* ctx, int enable) {
  if (!ctx) return fail(nullptr, HD_EINVAL, "hd_context_set_timing: null ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->timing = enable != 0;
  ctx->pool_used = 0;  // (re)start accumulating
  ctx->times = hd_timing{};
  return HD_OK;
}

int hd_context_get_timing(const hd_context* ctx_, hd_timing* out) {
  if (!ctx_ || !out) return fail(nullptr, HD_EINVAL, "hd_context_get_timing: null arg");
  hd_context* ctx = const_cast<hd_context*>(ctx_);
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = resolve_timing(ctx);
  if (rc) return rc;
  *out = ctx->times;
  return HD_OK;
}

int hd_context_reserve(hd_context* ctx, const hd_config* cfg, long nsolve) {
  if (!ctx || !cfg || nsolve < 0) return fail(ctx, HD_EINVAL, "hd_context_reserve: bad args");
  if (cfg->nstr < 2 || cfg->nstr % 2 || cfg->nstr / 2 > hd::kMaxNN || cfg->nlyr < 1)
    return fail(ctx, HD_EINVAL, "hd_context_reserve: bad config");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard guard;
  HD_HIP(ctx, hipSetDevice(ctx->device));
  const bool planck_r = (cfg->flags & HD_FLAG_PLANCK) != 0;
  const long chunk = ctx->chunk > 0 ? std::min(ctx->chunk, nsolve)
                                    : max_auto_chunk(nsolve, cfg->nstr / 2, cfg->nlyr, planck_r);
  const size_t per = hd::scratch_doubles_per_solve(cfg->nstr / 2, cfg->nlyr,
                                                   (cfg->flags & HD_FLAG_PLANCK) != 0);
  // room for hd_solve_band's epilogue too, at its largest (any nwave): so a
  // reserved context captures either solve without growing
  const long c1 = std::max<long>(chunk, 1);
  const int nslot_max = hd::band_slots(1);
  const size_t band_extra = std::max(4 * (size_t)c1 + (size_t)((c1 + 63) / 64) * nslot_max *
                                                          2 * (size_t)(cfg->nlyr + 1),
                                     2 * (size_t)c1 * 2 * (size_t)(cfg->nlyr + 1));
  int rc = ensure_scratch(ctx, per * c1 + band_extra);
  if (rc) return rc;
  // and hd_solve_band's row-major route (largest call that takes it: nsolve itself)
  if (band_rowmajor(ctx, cfg->nstr / 2, nsolve)) {
    rc = ensure_pflux(ctx, (size_t)nsolve * 2 * (size_t)(cfg->nlyr + 1));
    if (rc) return rc;
  }
  rc = ensure_tables(ctx);
  if (rc) return rc;
  return ensure_status(ctx, (size_t)nsolve);
}

long hd_chunk_solves(const hd_config* cfg, long nsolve) {
  if (!cfg || nsolve < 0 || cfg->nstr < 2 || cfg->nstr % 2 || cfg->nstr / 2 > hd::kMaxNN ||
      cfg->nlyr < 1)
    return -1;
  return auto_chunk(nsolve, cfg->nstr / 2, cfg->nlyr, (cfg->flags & HD_FLAG_PLANCK) != 0);
}

int hd_quadrature(int nstr, double* mu, double* w) {
  if (nstr < 2 || nstr % 2 || !mu || !w)
    return fail(nullptr, HD_EINVAL, "hd_quadrature: bad args");
  gauss01(nstr / 2, mu, w);
  return HD_OK;
}

}  // extern "C"

namespace {

// hd_solve's enqueue body: everything it launches ends on `stream` (the side
// and lay streams fork from it and join back into it)
int solve_enqueue(hd_context* ctx, const hd_config* cfg, const hd_inputs* in, double* flux,
                  const hd_band* band, int*& status, hipStream_t stream) {
  int rc = HD_OK;
  const long nsolve = (long)in->nwave * in->ncol;
  const int nn = cfg->nstr / 2;
  const int nlyr = cfg->nlyr;
  const bool planck = (cfg->flags & HD_FLAG_PLANCK) != 0;
  const bool sync = status == nullptr;
  const bool reg = nn <= hd::kMaxRegNN;
  const size_t nlev2 = 2 * (size_t)(nlyr + 1);

  long chunk = ctx->chunk > 0 ? std::min(ctx->chunk, nsolve) : auto_chunk(nsolve, nn, nlyr, planck);
  const size_t ne1 = hd::layer_record_doubles(nn);
  const size_t ne2 = hd::bsub_record_doubles(nn);
  const size_t per = hd::scratch_doubles_per_solve(nn, nlyr, planck);
  // fused band epilogue: register path -- column-major chunks, the surface
  // fluxes of two chunks in flight [2][2][chunk] and one chunk's run partials
  // [wave][nslot][lev][2]; team path -- one chunk's fluxes when the caller
  // keeps none
  const int nslot = band ? hd::band_slots(in->nwave) : 0;
  size_t band_extra = 0;
  if (band && reg) band_extra = 4 * (size_t)chunk + (size_t)((chunk + 63) / 64) * nslot * nlev2;
  // team path without caller fluxes: two chunk flux buffers (the band reduce of chunk
  // k runs on the side stream beside sweep k+1)
  if (band && !reg && !flux) band_extra = 2 * (size_t)chunk * nlev2;
  rc = ensure_scratch(ctx, per * chunk + band_extra);
  if (rc) return rc;
  rc = ensure_tables(ctx);
  if (rc) return rc;
  if (sync) {
    rc = ensure_status(ctx, (size_t)nsolve);
    if (rc) return rc;
    status = ctx->status;
  }
  HD_HIP(ctx, hipMemsetAsync(status, 0, sizeof(int) * nsolve, stream));
  HD_HIP(ctx, hipMemsetAsync(ctx->anyerr, 0, sizeof(int), stream));
  const int nm = std::max(0, std::min(cfg->nmom, cfg->nprop - 2));
  const int cmaj = band && reg ? 1 : 0;

  // a register-path call of one chunk has nothing to overlap: it runs wholly on
  // the caller's stream (prologue, layer kernel, sweep, tail back-substitution),
  // without the fork/join of the three-stream pipeline below (C1/C3 latency)
  // nstr 16 by the column kernel: every chunk wholly on the caller's stream
  const bool col = reg && nn == 8 && ctx->column;
  const bool single = reg && !col && nsolve <= chunk;
  // team path with several chunks: chunk k+1's prologue and layer kernel on the
  // `lay` stream beside chunk k's sweep on the caller's stream
  const bool team_pipe = !reg && nsolve > chunk;
  const bool beam = in->fbeam != nullptr;
  // Without Planck emission the layer kernels' beam sources are for a unit beam at
  // the layer top and the sweep scales them by exp(-tau_c/mu0) from its own running
  // depth, so no chunk needs the cumulative-depth prologue.  Register path: it sat
  // on the side stream behind the previous back-substitution and held each chunk's
  // layer kernel back until the sweep beside it was done.  Team path: chunk k+1's
  // prologue, launched as chunk k's sweep, waited for SIMDs the sweep's two
  // 254-register waves hold (up to 3.3 ms of a 48 ms C5 step,
  // profiles/r04/c5_timeline_last_step_v2.txt).  With Planck the sources mix beam
  // and thermal terms and the prologue stays.
  const bool beam_in_sweep = beam && !planck;
  const bool need_tauc = beam && !beam_in_sweep;
  const bool need_pro = planck || need_tauc;
  const int nb = 2;  // buffers of the per-chunk regions (two chunks in flight)
  // Scratch regions, sized for the largest chunk so that no region moves between
  // chunks (inside a region the kernels interleave with the chunk's own nsc):
  //   layer ops[nb] | bsub[nb] | xsurf[nb] | planck[nb] | tauc[nb]
  // Register path (three streams): chunk k uses buffer k&1; its layer kernel
  // (stream lay) runs beside chunk k-1's sweep (the caller's stream), its
  // back-substitution (side stream) beside chunk k+1's layer kernel, and chunk
  // k+1's tauc/planck prologue (side stream) beside chunk k.
  double* layer_b[2];
  double* bsub_b[2];
  double* xsurf_b[2];
  double* planck_b[2];
  double* tauc_b[2];
  double* band_q = nullptr;  // band-epilogue scratch after the regions
  {
    double* q = ctx->scratch;
    for (int b = 0; b < nb; ++b, q += ne1 * nlyr * (size_t)chunk) layer_b[b] = q;
    for (int b = 0; b < nb; ++b, q += ne2 * nlyr * (size_t)chunk) bsub_b[b] = q;
    for (int b = 0; b < nb; ++b, q += chunk) xsurf_b[b] = q;
    for (int b = 0; b < nb; ++b) {
      planck_b[b] = planck ? q : nullptr;
      if (planck) q += (size_t)(nlyr + 3) * chunk;
    }
    for (int b = 0; b < nb; ++b, q += (size_t)nlyr * chunk) tauc_b[b] = q;
    band_q = q;
  }
  double* fsurf_b[2] = {nullptr, nullptr};
  double* part = nullptr;
  double* fchunk_b[2] = {nullptr, nullptr};
  if (band && reg) {
    fsurf_b[0] = band_q;
    fsurf_b[1] = band_q + 2 * (size_t)chunk;
    part = band_q + 4 * (size_t)chunk;
  } else if (band && !flux) {
    fchunk_b[0] = band_q;
    fchunk_b[1] = band_q + (size_t)chunk * nlev2;
  }
  auto band_args = [&](long s0, int nsc, int b) {
    hd::BandArgs ba{};
    ba.part = part;
    ba.fchunk = part ? nullptr : (flux ? flux + (size_t)s0 * nlev2 : fchunk_b[b]);
    ba.wts = band->weight;
    ba.bflux = band->bflux;
    ba.s0 = s0;
    ba.nsc = nsc;
    ba.ncol = in->ncol;
    ba.nwave = in->nwave;
    ba.nlev = nlyr + 1;
    ba.nslot = nslot;
    return ba;
  };
  auto prologue_args = [&](long s0, int nsc, int b, hd::TaucArgs& ta, hd::PlanckArgs& pa) {
    ta = hd::TaucArgs{};
    ta.prop = in->prop;
    ta.out = tauc_b[b];
    ta.s0 = s0;
    ta.nsc = nsc;
    ta.nlyr = nlyr;
    ta.nprop = cfg->nprop;
    ta.use_f = nm >= cfg->nstr;
    ta.f_slot = 1 + cfg->nstr;
    ta.cmaj = cmaj;
    ta.nwave = in->nwave;
    ta.ncol = in->ncol;
    pa = hd::PlanckArgs{};
    pa.temf = in->temf;
    pa.btemp = in->btemp;
    pa.ttemp = in->ttemp;
    pa.temis = in->temis;
    pa.wlo = in->wave_lower;
    pa.whi = in->wave_upper;
    pa.out = planck_b[b];
    pa.s0 = s0;
    pa.nsc = nsc;
    pa.ncol = in->ncol;
    pa.nlyr = nlyr;
    pa.cmaj = cmaj;
    pa.nwave = in->nwave;
  };

  if ((reg && !single && !col) || team_pipe) {
    // fork: the side stream sees everything the caller's stream did before this
    // call (the inputs) -- and, under stream capture, joins the graph here
    HD_HIP(ctx, hipEventRecord(ctx->ev_fork, stream));
    HD_HIP(ctx, hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
    HD_HIP(ctx, hipStreamWaitEvent(ctx->lay, ctx->ev_fork, 0));
  }
  long k = 0;  // chunk index
  for (long s0 = 0; s0 < nsolve; s0 += chunk, ++k) {
    const int nsc = (int)std::min(chunk, nsolve - s0);
    const int buf = (int)(k & 1);
    hd::TaucArgs ta;
    hd::PlanckArgs pa;
    prologue_args(s0, nsc, buf, ta, pa);
    if (team_pipe) {
      // buffer `buf` is free once sweep k-2 (its last reader) is done
      if (k >= 2) HD_HIP(ctx, hipStreamWaitEvent(ctx->lay, ctx->ev_sweep[buf], 0));
      hd::launch_prologue(planck ? &pa : nullptr, need_tauc ? &ta : nullptr, ctx->lay);
    } else if (!reg || single || col) {
      hd::launch_prologue(planck ? &pa : nullptr, need_tauc ? &ta : nullptr, stream);
    } else if (k == 0 && need_pro) {
      hd::launch_prologue(planck ? &pa : nullptr, need_tauc ? &ta : nullptr, ctx->side);
      HD_HIP(ctx, hipEventRecord(ctx->ev_pro[0], ctx->side));
    }
    hd::LayerArgs la{};
    la.prop = in->prop;
    la.tauc = need_tauc ? tauc_b[buf] : nullptr;  // null with a beam: unit beam at the top
    la.fbeam = in->fbeam;
    la.umu0 = in->umu0;
    la.planckv = planck_b[buf];
    la.scr = layer_b[buf];
    la.status = status;
    la.anyerr = ctx->anyerr;
    la.s0 = s0;
    la.nsc = nsc;
    la.ncol = in->ncol;
    la.nlyr = nlyr;
    la.nprop = cfg->nprop;
    la.nmom = nm;
    la.planck = planck;
    la.max_sweeps = ctx->max_sweeps;
    la.warm = ctx->warm;
    la.sink = ctx->sink;
    la.cmaj = cmaj;
    la.nwave = in->nwave;
    hd::SweepArgs sa{};
    sa.scr = layer_b[buf];
    sa.bsub = bsub_b[buf];
    sa.xsurf = xsurf_b[buf];
    sa.flux = flux;
    sa.fbeam = in->fbeam;
    sa.umu0 = in->umu0;
    sa.albedo = in->albedo;
    sa.fisot = in->fisot;
    sa.planckv = planck_b[buf];
    sa.status = status;
    sa.anyerr = ctx->anyerr;
    sa.s0 = s0;
    sa.nsc = nsc;
    sa.ncol = in->ncol;
    sa.nlyr = nlyr;
    sa.planck = planck;
    sa.sink = ctx->sink;
    sa.cmaj = cmaj;
    sa.nwave = in->nwave;
    sa.beam_scale = beam_in_sweep ? 1 : 0;
    sa.lean = ctx->lean;
    sa.quad = ctx->quad;
    sa.lean8 = ctx->lean8;
    if (band && reg) {
      sa.wts = band->weight;
      sa.part = part;
      sa.fsurf = fsurf_b[buf];
      sa.nslot = nslot;
      sa.rsteps = hd::band_steps(in->nwave);
    } else if (band && !flux) {
      sa.flux = fchunk_b[buf];
      sa.flux_local = 1;
    }
    hipEvent_t* ev = nullptr;
    if (ctx->timing) {
      if (ctx->pool_used >= 4 * 512) {
        rc = resolve_timing(ctx);
        if (rc) return rc;
      }
      while (ctx->pool.size() < ctx->pool_used + 4) {
        hipEvent_t e;
        HD_HIP(ctx, hipEventCreate(&e));
        ctx->pool.push_back(e);
      }
      ev = &ctx->pool[ctx->pool_used];
      ctx->pool_used += 4;
    }
    hipError_t e = hipSuccess;
    if (col) {
      if (ev) HD_HIP(ctx, hipEventRecord(ev[0], stream));
      e = hd::launch_column_nn(nn, la, sa, stream);
      if (ev) HD_HIP(ctx, hipEventRecord(ev[1], stream));
      if (ev) HD_HIP(ctx, hipEventRecord(ev[2], stream));
      if (ev) HD_HIP(ctx, hipEventRecord(ev[3], stream));
      if (e == hipSuccess && band) e = hd::launch_band_reduce(band_args(s0, nsc, buf), stream);
    } else if (single) {
      if (ev) HD_HIP(ctx, hipEventRecord(ev[0], stream));
      e = hd::launch_layer_nn(nn, la, stream);
      if (ev) HD_HIP(ctx, hipEventRecord(ev[1], stream));
      if (ev) HD_HIP(ctx, hipEventRecord(ev[2], stream));
      if (e == hipSuccess) e = hd::launch_sweep_nn(nn, sa, stream);
      if (ev) HD_HIP(ctx, hipEventRecord(ev[3], stream));
      if (e == hipSuccess) e = hd::launch_backsub_nn(nn, sa, stream, true);
      if (e == hipSuccess && band) e = hd::launch_band_reduce(band_args(s0, nsc, buf), stream);
    } else if (reg) {
      // layer kernel k on `lay`: its inputs (prologue k) are in, and sweep k-2,
      // the last reader of layer records[buf], is done
      if (need_pro) HD_HIP(ctx, hipStreamWaitEvent(ctx->lay, ctx->ev_pro[buf], 0));
      if (k >= 2) HD_HIP(ctx, hipStreamWaitEvent(ctx->lay, ctx->ev_sweep[buf], 0));
      if (ev) HD_HIP(ctx, hipEventRecord(ev[0], ctx->lay));
      e = hd::launch_layer_nn(nn, la, ctx->lay);
      if (ev) HD_HIP(ctx, hipEventRecord(ev[1], ctx->lay));
      HD_HIP(ctx, hipEventRecord(ctx->ev_layer[buf], ctx->lay));
      // sweep k on the caller's stream: after layer k, and after back-substitution
      // k-2, the last reader of the back-substitution records[buf]
      if (e == hipSuccess) {
        HD_HIP(ctx, hipStreamWaitEvent(stream, ctx->ev_layer[buf], 0));
        if (k >= 2) HD_HIP(ctx, hipStreamWaitEvent(stream, ctx->ev_back[buf], 0));
        if (ev) HD_HIP(ctx, hipEventRecord(ev[2], stream));
        e = hd::launch_sweep_nn(nn, sa, stream);
        if (ev) HD_HIP(ctx, hipEventRecord(ev[3], stream));
      }
    } else if (team_pipe) {
      if (ev) HD_HIP(ctx, hipEventRecord(ev[0], ctx->lay));
      e = hd::launch_team_layer_nn(nn, la, ctx->lay);
      if (ev) HD_HIP(ctx, hipEventRecord(ev[1], ctx->lay));
      HD_HIP(ctx, hipEventRecord(ctx->ev_layer[buf], ctx->lay));
      if (e == hipSuccess) {
        HD_HIP(ctx, hipStreamWaitEvent(stream, ctx->ev_layer[buf], 0));
        // the chunk flux buffer[buf] is free once band reduce k-2 (its reader) is done
        if (band && k >= 2) HD_HIP(ctx, hipStreamWaitEvent(stream, ctx->ev_back[buf], 0));
        if (ev) HD_HIP(ctx, hipEventRecord(ev[2], stream));
        e = hd::launch_team_sweep_nn(nn, sa, stream);
        if (ev) HD_HIP(ctx, hipEventRecord(ev[3], stream));
      }
      HD_HIP(ctx, hipEventRecord(ctx->ev_sweep[buf], stream));
      // the band reduce of chunk k on the side stream: on the caller's stream it sat
      // between sweep k and sweep k+1 waiting for SIMDs the co-running layer kernel
      // held (6.4 ms average per 11 us launch, profiles/r04/c5_kernel_stats_final.csv);
      // the reduces stay in chunk order (bflux accumulates chunk by chunk)
      if (e == hipSuccess && band) {
        HD_HIP(ctx, hipStreamWaitEvent(ctx->side, ctx->ev_sweep[buf], 0));
        e = hd::launch_band_reduce(band_args(s0, nsc, buf), ctx->side);
        HD_HIP(ctx, hipEventRecord(ctx->ev_back[buf], ctx->side));
      }
    } else {
      e = hd::launch_solve_chunk_team(nn, nullptr, nullptr, la, sa, stream, ev);
      if (e == hipSuccess && band) e = hd::launch_band_reduce(band_args(s0, nsc, buf), stream);
    }
    if (e != hipSuccess) return fail(ctx, HD_EHIP, "hd_solve: launch failed: %s", hipGetErrorString(e));
    if (reg && !single && !col) {
      HD_HIP(ctx, hipEventRecord(ctx->ev_sweep[buf], stream));
      // next chunk's prologue into the other buffer (free: the side stream already
      // waited for the sweep of chunk k-1, the last user of that buffer)
      const long s1 = s0 + chunk;
      if (s1 < nsolve && need_pro) {
        hd::TaucArgs ta1;
        hd::PlanckArgs pa1;
        prologue_args(s1, (int)std::min(chunk, nsolve - s1), buf ^ 1, ta1, pa1);
        hd::launch_prologue(planck ? &pa1 : nullptr, need_tauc ? &ta1 : nullptr, ctx->side);
        HD_HIP(ctx, hipEventRecord(ctx->ev_pro[buf ^ 1], ctx->side));
      }
      HD_HIP(ctx, hipStreamWaitEvent(ctx->side, ctx->ev_sweep[buf], 0));
      // The last chunk's back-substitution takes the uncapped tail kernel (nothing
      // overlaps it).  With at most three chunks every chunk's does: the capped
      // kernel then still runs beside the last layer kernel when the step could
      // end, while the tail kernel takes the SIMDs briefly and is done -- 8-GPU
      // rank shape (80 000 solves, 2 chunks) 9.47 -> 10.50 M solves/s, 4-GPU
      // (160 000, 3 chunks) 10.0 -> 10.3 M; with 5 and 10 chunks the capped kernel
      // hidden under the next layer kernel stays ahead (profiles/r02_tail_ab/)
      const bool tail = s1 >= nsolve || (nsolve + chunk - 1) / chunk <= 3;
      e = hd::launch_backsub_nn(nn, sa, ctx->side, tail);
      if (e == hipSuccess && band) e = hd::launch_band_reduce(band_args(s0, nsc, buf), ctx->side);
      if (e != hipSuccess)
        return fail(ctx, HD_EHIP, "hd_solve: back-substitution launch failed: %s",
                    hipGetErrorString(e));
      HD_HIP(ctx, hipEventRecord(ctx->ev_back[buf], ctx->side));
    }
  }
  if ((reg && !single && !col) || (team_pipe && band)) {  // every chunk's fluxes complete
    for (long b = 0; b < std::min<long>(k, 2); ++b)
      HD_HIP(ctx, hipStreamWaitEvent(stream, ctx->ev_back[b], 0));
  }
  return HD_OK;
}

// The common frame of the two solve entry points: context lock, device guard,
// ordering behind the context's previous solve, and the synchronous error
// check when the caller passed no status buffer.
template <class Enqueue>
int run_solve(hd_context* ctx, int* status, void* stream_, const char* what, Enqueue&& enqueue) {
  DeviceGuard guard;
  HD_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
  bool capturing = false;
  int rc = enter(ctx, stream, &capturing);
  if (rc) return rc;
  const bool sync = status == nullptr;
  ctx->capturing = capturing;
  rc = enqueue(status, stream);
  ctx->capturing = false;
  int any = 0;
  if (rc == HD_OK && sync) {
    const hipError_t e = hipMemcpyAsync(&any, ctx->anyerr, sizeof(int), hipMemcpyDeviceToHost, stream);
    if (e != hipSuccess) rc = fail(ctx, HD_EHIP, "%s: anyerr copy: %s", what, hipGetErrorString(e));
  }
  const int rc2 = leave(ctx, stream, capturing);  // also after a partial enqueue
  if (rc) return rc;
  if (rc2) return rc2;
  if (sync) {
    HD_HIP(ctx, hipStreamSynchronize(stream));
    if (any)
      return fail(ctx, HD_ENUMERIC,
                  "%s: at least one solve failed (bad input, eigen breakdown or non-finite "
                  "result); DisortWrapper::Run failed.", what);
  }
  return HD_OK;
}

}  // namespace

extern "C" {

int hd_solve(hd_context* ctx, const hd_config* cfg, const hd_inputs* in, double* flux,
             int* status, void* stream) {
  if (!ctx) return fail(nullptr, HD_EINVAL, "hd_solve: null context");
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = validate(ctx, cfg, in, flux);
  if (rc) return rc;
  if ((long)in->nwave * in->ncol == 0) return HD_OK;
  return run_solve(ctx, status, stream, "hd_solve", [&](int*& st, hipStream_t s) {
    return solve_enqueue(ctx, cfg, in, flux, nullptr, st, s);
  });
}

int hd_solve_band(hd_context* ctx, const hd_config* cfg, const hd_inputs* in,
                  const hd_band* band, double* flux, int* status, void* stream) {
  if (!ctx) return fail(nullptr, HD_EINVAL, "hd_solve_band: null context");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!band || !band->weight || !band->bflux)
    return fail(ctx, HD_EINVAL, "hd_solve_band: band weights and bflux are required");
  // flux is optional here: validate against a non-null stand-in
  int rc = validate(ctx, cfg, in, flux ? flux : band->bflux);
  if (rc) return rc;
  const long nsolve = (long)in->nwave * in->ncol;
  if (nsolve == 0) return HD_OK;
  if (!flux && band_rowmajor(ctx, cfg->nstr / 2, nsolve)) {
    return run_solve(ctx, status, stream, "hd_solve_band", [&](int*& st, hipStream_t s) {
      int r = ensure_pflux(ctx, (size_t)nsolve * 2 * (size_t)(cfg->nlyr + 1));
      if (r) return r;
      r = solve_enqueue(ctx, cfg, in, ctx->pflux, nullptr, st, s);
      if (r) return r;
      r = hd_band_flux(ctx->pflux, band->weight, in->nwave, in->ncol, cfg->nlyr + 1,
                       band->bflux, s);
      return r ? fail(ctx, r, "hd_solve_band: hd_band_flux launch failed") : HD_OK;
    });
  }
  return run_solve(ctx, status, stream, "hd_solve_band", [&](int*& st, hipStream_t s) {
    return solve_enqueue(ctx, cfg, in, flux, band, st, s);
  });
}

}  // extern "C"

namespace {

// hd_solve_host / hd_solve_band_host: the same solve on the caller's host arrays
// (pydisort's CPU-tensor contract).  The inputs go to a device staging area of
// the context, the solve runs on the context's own stream, the outputs come back;
// synchronous.  No CPU arithmetic: without a device the call fails like hd_solve.
int solve_host(hd_context* ctx, const hd_config* cfg, const hd_inputs* in, double* flux,
               const double* weight, double* bflux, int* status, const char* what) {
  if (!ctx) return fail(nullptr, HD_EINVAL, "%s: null context", what);
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!cfg || !in) return fail(ctx, HD_EINVAL, "%s: null config or inputs", what);
  const bool band = bflux != nullptr;
  if (band && !weight) return fail(ctx, HD_EINVAL, "%s: band weights are required", what);
  int rc = validate(ctx, cfg, in, flux ? flux : bflux);
  if (rc) return rc;
  const long nsolve = (long)in->nwave * in->ncol;
  if (nsolve == 0) return HD_OK;
  const bool planck = (cfg->flags & HD_FLAG_PLANCK) != 0;
  const int nlev = cfg->nlyr + 1;
  const size_t nlev2 = 2 * (size_t)nlev;
  const size_t ns = (size_t)nsolve;
  const size_t ncol = (size_t)in->ncol;
  // Pieces of whole waves (contiguous slices of every input): piece j+1's arrays
  // go over PCIe (copy stream) while piece j is solved (compute stream); two input
  // buffers.  ~128 k solves per piece keeps each solve near full-batch efficiency.
  const long wpp = std::max<long>(1, std::min<long>(in->nwave, (131072 + in->ncol - 1) / in->ncol));
  const int npiece = (int)((in->nwave + wpp - 1) / wpp);
  const size_t pin_prop = (size_t)wpp * ncol * cfg->nlyr * (size_t)cfg->nprop;
  const size_t pin_bc = (size_t)wpp * ncol;
  const double* bc_h[7] = {in->fbeam, in->umu0, in->albedo, in->btemp,
                           in->ttemp, in->temis, in->fisot};
  int nbc = 0;
  for (int k = 0; k < 7; ++k) nbc += bc_h[k] != nullptr;
  const size_t pin = pin_prop + nbc * pin_bc;
  const size_t n_temf = planck ? ncol * nlev : 0;
  const size_t n_wave = planck ? (size_t)in->nwave : 0;
  const size_t n_w = band ? (size_t)in->nwave + npiece : 0;  // weights, then ones
  const size_t n_flux = flux ? ns * nlev2 : 0;
  const size_t n_part = band ? (size_t)npiece * ncol * nlev2 + ncol * nlev2 : 0;
  const size_t n_stat = (ns + 1) / 2;  // int32 in double slots
  const size_t total = 2 * pin + n_temf + 2 * n_wave + n_w + n_flux + n_part + n_stat;
  DeviceGuard guard;
  HD_HIP(ctx, hipSetDevice(ctx->device));
  if (!ctx->hstream) HD_HIP(ctx, hipStreamCreateWithFlags(&ctx->hstream, hipStreamNonBlocking));
  if (!ctx->hstream2) HD_HIP(ctx, hipStreamCreateWithFlags(&ctx->hstream2, hipStreamNonBlocking));
  if (!ctx->hstream3) HD_HIP(ctx, hipStreamCreateWithFlags(&ctx->hstream3, hipStreamNonBlocking));
  for (int b = 0; b < 2; ++b) {
    if (!ctx->hev_in[b]) HD_HIP(ctx, hipEventCreateWithFlags(&ctx->hev_in[b], hipEventDisableTiming));
    if (!ctx->hev_done[b])
      HD_HIP(ctx, hipEventCreateWithFlags(&ctx->hev_done[b], hipEventDisableTiming));
  }
  if (ctx->hstage_len < total) {
    drain(ctx);
    if (ctx->hstage) (void)hipFree(ctx->hstage);
    ctx->hstage = nullptr;
    ctx->hstage_len = 0;
    if (hipMalloc(&ctx->hstage, total * sizeof(double)) != hipSuccess) {
      (void)hipGetLastError();
      return fail(ctx, HD_ENOMEM, "%s: cannot allocate %zu bytes of staging", what,
                  total * sizeof(double));
    }
    ctx->hstage_len = total;
  }
  // uploads, solves, downloads: the per-point fluxes of piece j go back on their own
  // stream while piece j+2's arrays go up (both PCIe directions at once)
  hipStream_t cs = ctx->hstream, xs = ctx->hstream2, ds = ctx->hstream3;
  // whatever happens below, nothing may still be reading or writing the
  // caller's arrays when this returns
  struct Drain {
    hipStream_t a, b, c;
    ~Drain() {
      (void)hipStreamSynchronize(a);
      (void)hipStreamSynchronize(b);
      (void)hipStreamSynchronize(c);
    }
  } drain_on_exit{cs, xs, ds};
  double* q = ctx->hstage;
  double* inbuf[2] = {q, q + pin};
  q += 2 * pin;
  double* temf_d = n_temf ? q : nullptr;
  q += n_temf;
  double* wlo_d = n_wave ? q : nullptr;
  q += n_wave;
  double* whi_d = n_wave ? q : nullptr;
  q += n_wave;
  double* w_d = band ? q : nullptr;
  q += n_w;
  double* flux_d = flux ? q : nullptr;
  q += n_flux;
  double* part_d = band ? q : nullptr;  // [piece][ncol][nlev][2], then the band sum
  q += n_part;
  int* st_d = reinterpret_cast<int*>(q);
  auto h2d = [&](double* d, const double* h, size_t n) {
    return hipMemcpyAsync(d, h, n * sizeof(double), hipMemcpyHostToDevice, cs);
  };
  if (n_temf) HD_HIP(ctx, h2d(temf_d, in->temf, n_temf));
  if (n_wave) {
    HD_HIP(ctx, h2d(wlo_d, in->wave_lower, n_wave));
    HD_HIP(ctx, h2d(whi_d, in->wave_upper, n_wave));
  }
  if (band) {
    HD_HIP(ctx, h2d(w_d, weight, (size_t)in->nwave));
    std::vector<double> ones((size_t)npiece, 1.0);
    HD_HIP(ctx, hipMemcpy(w_d + in->nwave, ones.data(), npiece * sizeof(double),
                          hipMemcpyHostToDevice));
  }
  std::vector<int> st_h(status ? 0 : ns);
  int* st_out = status ? status : st_h.data();
  auto d2h = [&](int j) -> int {  // piece j's per-point fluxes and status, after its solve
    const long w0 = (long)j * wpp, wj = std::min<long>(wpp, in->nwave - w0);
    const size_t o = (size_t)w0 * ncol, n = (size_t)wj * ncol;
    HD_HIP(ctx, hipStreamWaitEvent(ds, ctx->hev_done[j & 1], 0));
    if (flux)
      HD_HIP(ctx, hipMemcpyAsync(flux + o * nlev2, flux_d + o * nlev2, n * nlev2 * sizeof(double),
                                 hipMemcpyDeviceToHost, ds));
    HD_HIP(ctx, hipMemcpyAsync(st_out + o, st_d + o, n * sizeof(int), hipMemcpyDeviceToHost, ds));
    return HD_OK;
  };
  for (int j = 0; j < npiece; ++j) {
    const int b = j & 1;
    const long w0 = (long)j * wpp, wj = std::min<long>(wpp, in->nwave - w0);
    const size_t o = (size_t)w0 * ncol, n = (size_t)wj * ncol;
    // buffer b was last read by the solve of piece j-2
    if (j >= 2) HD_HIP(ctx, hipStreamWaitEvent(cs, ctx->hev_done[b], 0));
    hd_inputs din = *in;
    din.nwave = (int)wj;
    double* p = inbuf[b];
    const size_t nprop = n * cfg->nlyr * (size_t)cfg->nprop;
    HD_HIP(ctx, h2d(p, in->prop + o * cfg->nlyr * (size_t)cfg->nprop, nprop));
    din.prop = p;
    p += nprop;
    const double** bc_d[7] = {&din.fbeam, &din.umu0, &din.albedo, &din.btemp,
                              &din.ttemp, &din.temis, &din.fisot};
    for (int k = 0; k < 7; ++k) {
      if (!bc_h[k]) continue;
      HD_HIP(ctx, h2d(p, bc_h[k] + o, n));
      *bc_d[k] = p;
      p += n;
    }
    din.temf = temf_d;
    din.wave_lower = wlo_d ? wlo_d + w0 : nullptr;
    din.wave_upper = whi_d ? whi_d + w0 : nullptr;
    HD_HIP(ctx, hipEventRecord(ctx->hev_in[b], cs));
    HD_HIP(ctx, hipStreamWaitEvent(xs, ctx->hev_in[b], 0));
    double* fd = flux ? flux_d + o * nlev2 : nullptr;
    rc = run_solve(ctx, st_d + o, xs, what, [&](int*& st, hipStream_t ss) {
      if (!band) return solve_enqueue(ctx, cfg, &din, fd, nullptr, st, ss);
      hd_band bb{w_d + w0, part_d + (size_t)j * ncol * nlev2};
      return solve_enqueue(ctx, cfg, &din, fd, &bb, st, ss);
    });
    if (rc) return rc;
    HD_HIP(ctx, hipEventRecord(ctx->hev_done[b], xs));
    if (j >= 1 && (rc = d2h(j - 1))) return rc;
  }
  if ((rc = d2h(npiece - 1))) return rc;
  if (band) {
    // the pieces' band partials, in piece (= wave) order
    double* bsum = part_d + (size_t)npiece * ncol * nlev2;
    rc = hd_band_flux(part_d, w_d + in->nwave, npiece, (int)ncol, nlev, bsum, xs);
    if (rc) return fail(ctx, rc, "%s: band sum: %s", what, hd_last_error(nullptr));
    HD_HIP(ctx, hipEventRecord(ctx->hev_done[0], xs));
    HD_HIP(ctx, hipStreamWaitEvent(ds, ctx->hev_done[0], 0));
    HD_HIP(ctx, hipMemcpyAsync(bflux, bsum, ncol * nlev2 * sizeof(double), hipMemcpyDeviceToHost, ds));
  }
  HD_HIP(ctx, hipStreamSynchronize(cs));
  HD_HIP(ctx, hipStreamSynchronize(xs));
  HD_HIP(ctx, hipStreamSynchronize(ds));
  for (size_t i = 0; i < ns; ++i)
    if (st_out[i] & HD_STATUS_ERROR_MASK)
      return fail(ctx, HD_ENUMERIC,
                  "%s: at least one solve failed (bad input, eigen breakdown or non-finite "
                  "result); DisortWrapper::Run failed.", what);
  return HD_OK;
}

}  // namespace

extern "C" {

int hd_solve_host(hd_context* ctx, const hd_config* cfg, const hd_inputs* in, double* flux,
                  int* status) {
  if (!flux) return fail(ctx, HD_EINVAL, "hd_solve_host: null flux");
  return solve_host(ctx, cfg, in, flux, nullptr, nullptr, status, "hd_solve_host");
}

int hd_solve_band_host(hd_context* ctx, const hd_config* cfg, const hd_inputs* in,
                       const double* weight, double* bflux, double* flux, int* status) {
  if (!bflux) return fail(ctx, HD_EINVAL, "hd_solve_band_host: null bflux");
  return solve_host(ctx, cfg, in, flux, weight, bflux, status, "hd_solve_band_host");
}

}  // extern "C"

namespace {

int validate_rad(hd_context* ctx, const hd_config* cfg, const hd_inputs* in,
                 const hd_radiance* rad, double* flux, double* uu) {
  int rc = validate(ctx, cfg, in, flux);
  if (rc) return rc;
  if (!rad) return fail(ctx, HD_EINVAL, "hd_solve_radiance: null radiance config");
  const int nn = cfg->nstr / 2;
  if (nn > hd::kRadMaxNN)
    return fail(ctx, HD_EINVAL, "hd_solve_radiance: nstr=%d; the intensity path supports nstr <= %d",
                cfg->nstr, 2 * hd::kRadMaxNN);
  const bool radiances = rad->onlyfl == 0;
  const int nlyr = cfg->nlyr;
  const int ntau = rad->ntau > 0 ? rad->ntau : nlyr + 1;
  const int numu = radiances ? rad->numu : 0;
  const int nphi = radiances ? rad->nphi : 0;
  if (rad->corint != 0 && rad->corint != 1)
    return fail(ctx, HD_EINVAL,
                "hd_solve_radiance: corint=%d; 0 (none) and 1 (Nakajima-Tanaka, cdisort's "
                "old_intensity_correction) are implemented, cdisort's new correction is not",
                rad->corint);
  if (rad->ntau < 0 || (rad->ntau > 0 && !rad->utau))
    return fail(ctx, HD_EINVAL, "hd_solve_radiance: ntau=%d needs utau", rad->ntau);
  for (int i = 0; i < rad->ntau; ++i)
    if (!(rad->utau[i] >= 0.0) || (i > 0 && !(rad->utau[i] >= rad->utau[i - 1])))
      return fail(ctx, HD_EINVAL, "hd_solve_radiance: utau must be >= 0 and ascending");
  if (radiances) {
    if (numu < 1 || !rad->umu || nphi < 1 || !rad->phi || !uu)
      return fail(ctx, HD_EINVAL,
                  "hd_solve_radiance: radiances need numu >= 1, nphi >= 1, umu, phi and uu");
    for (int i = 0; i < numu; ++i)
      if (!(rad->umu[i] != 0.0) || !(std::fabs(rad->umu[i]) <= 1.0))
        return fail(ctx, HD_EINVAL, "hd_solve_radiance: umu[%d]=%g must be in [-1,0)U(0,1]", i,
                    rad->umu[i]);
  }
  return HD_OK;
}

int rad_enqueue(hd_context* ctx, const hd_config* cfg, const hd_inputs* in,
                const hd_radiance* rad, double* flux, double* uu, int*& status,
                hipStream_t stream) {
  int rc = HD_OK;
  const int nn = cfg->nstr / 2;
  const bool radiances = rad->onlyfl == 0;
  const int nlyr = cfg->nlyr;
  const int ntau = rad->ntau > 0 ? rad->ntau : nlyr + 1;
  const int numu = radiances ? rad->numu : 0;
  const int nphi = radiances ? rad->nphi : 0;
  const long nsolve = (long)in->nwave * in->ncol;
  const bool planck = (cfg->flags & HD_FLAG_PLANCK) != 0;
  const bool beam = in->fbeam != nullptr;
  const bool sync = status == nullptr;
  const int nm_mode = (radiances && beam) ? cfg->nstr : 1;
  const int nmom = std::max(0, std::min(cfg->nmom, cfg->nprop - 2));

  // the user grid is copied from host arrays and its buffer may grow: a radiance
  // solve is not capturable (a replay would reread host memory the caller may have
  // freed, and nothing may be allocated under capture)
  if (ctx->capturing)
    return fail(ctx, HD_EINVAL,
                "hd_solve_radiance: not capturable into a HIP graph (host user grid)");
  rc = ensure_rad_tables(ctx);
  if (rc) return rc;
  // user grid on the device: umu | phi | utau
  const size_t ngrid = (size_t)numu + nphi + rad->ntau;
  if (ngrid > ctx->rad_grid_len) {
    drain(ctx);
    if (ctx->rad_grid) (void)hipFree(ctx->rad_grid);
    ctx->rad_grid = nullptr;
    ctx->rad_grid_len = 0;
    HD_HIP(ctx, hipMalloc(&ctx->rad_grid, ngrid * sizeof(double)));
    ctx->rad_grid_len = ngrid;
  }
  double* d_umu = ctx->rad_grid;
  double* d_phi = d_umu + numu;
  double* d_utau = d_phi + nphi;
  if (numu) HD_HIP(ctx, hipMemcpyAsync(d_umu, rad->umu, numu * sizeof(double), hipMemcpyHostToDevice, stream));
  if (nphi) HD_HIP(ctx, hipMemcpyAsync(d_phi, rad->phi, nphi * sizeof(double), hipMemcpyHostToDevice, stream));
  if (rad->ntau)
    HD_HIP(ctx, hipMemcpyAsync(d_utau, rad->utau, rad->ntau * sizeof(double), hipMemcpyHostToDevice, stream));

  // chunk: scratch per solve = modes x (per-unit records + radiance per mode) + prologue
  const size_t per_unit = hd::rad_scratch_doubles_per_unit(nn, nlyr) + (size_t)ntau * numu;
  const size_t per_solve = (size_t)nm_mode * per_unit + (size_t)(nlyr + 1) + nlyr +
                           (planck ? (size_t)nlyr + 3 : 0);
  // 16 GB of the 288 GB: chunks of ~1e5 units keep every SIMD busy in the per-unit sweep
  const double budget = 16.0 * 1024.0 * 1024.0 * 1024.0 / 8.0;  // doubles
  long chunk = std::max<long>(1, std::min<long>(nsolve, (long)(budget / (double)per_solve)));
  chunk = std::min<long>(chunk, 0x7fffffffL / std::max(1, nm_mode));
  if (ctx->chunk > 0) chunk = std::min(chunk, ctx->chunk);
  rc = ensure_scratch(ctx, per_solve * chunk);
  if (rc) return rc;
  if (sync) {
    rc = ensure_status(ctx, (size_t)nsolve);
    if (rc) return rc;
    status = ctx->status;
  }
  HD_HIP(ctx, hipMemsetAsync(status, 0, sizeof(int) * nsolve, stream));
  HD_HIP(ctx, hipMemsetAsync(ctx->anyerr, 0, sizeof(int), stream));

  const size_t nuc = (size_t)nm_mode * chunk;  // units of the largest chunk
  double* q = ctx->scratch;
  // the intensity kernels keep the register-path layer record layout at every
  // nstr (hd::layer_record_doubles gives the team layout above nstr 16)
  double* r_sw = q;   q += (size_t)nlyr * hd::rad_layer_record_doubles(nn) * nuc;
  double* r_rd = q;   q += (size_t)nlyr * hd::rad_rec_doubles(nn) * nuc;
  double* r_bs = q;   q += (size_t)nlyr * hd::rad_bsub_doubles(nn) * nuc;
  double* r_lev = q;  q += (size_t)(nlyr + 1) * 2 * nn * nuc;
  double* r_cst = q;  q += (size_t)nlyr * 2 * nn * nuc;
  double* r_radm = q; q += (size_t)ntau * numu * nuc;
  double* r_taus = q; q += (size_t)(nlyr + 1) * chunk;
  double* r_tauc = q; q += (size_t)nlyr * chunk;
  double* r_planck = planck ? q : nullptr;

  for (long s0 = 0; s0 < nsolve; s0 += chunk) {
    const int ns = (int)std::min(chunk, nsolve - s0);
    hd::TaucArgs ta{};
    ta.prop = in->prop;
    ta.out = r_tauc;
    ta.s0 = s0;
    ta.nsc = ns;
    ta.nlyr = nlyr;
    ta.nprop = cfg->nprop;
    ta.use_f = nmom >= cfg->nstr;
    ta.f_slot = 1 + cfg->nstr;
    hd::PlanckArgs pa{};
    pa.temf = in->temf;
    pa.btemp = in->btemp;
    pa.ttemp = in->ttemp;
    pa.temis = in->temis;
    pa.wlo = in->wave_lower;
    pa.whi = in->wave_upper;
    pa.out = r_planck;
    pa.s0 = s0;
    pa.nsc = ns;
    pa.ncol = in->ncol;
    pa.nlyr = nlyr;
    hd::launch_prologue(planck ? &pa : nullptr, beam ? &ta : nullptr, stream);
    hd::RadArgs a{};
    a.prop = in->prop;
    a.fbeam = in->fbeam;
    a.umu0 = in->umu0;
    a.albedo = in->albedo;
    a.fisot = in->fisot;
    a.phi0 = rad->phi0;
    a.planckv = r_planck;
    a.tauc = beam ? r_tauc : nullptr;
    a.taus = r_taus;
    a.umu = d_umu;
    a.phi = d_phi;
    a.utau = rad->ntau > 0 ? d_utau : nullptr;
    a.rsw = r_sw;
    a.rrd = r_rd;
    a.bsub = r_bs;
    a.lev = r_lev;
    a.cst = r_cst;
    a.radm = r_radm;
    a.flux = flux;
    a.uu = uu;
    a.status = status;
    a.anyerr = ctx->anyerr;
    a.s0 = s0;
    a.ns = ns;
    a.nm = nm_mode;
    a.nu = ns * nm_mode;
    a.ncol = in->ncol;
    a.nlyr = nlyr;
    a.nprop = cfg->nprop;
    a.nmom = nmom;
    a.planck = planck;
    a.max_sweeps = ctx->max_sweeps;
    a.numu = numu;
    a.nphi = nphi;
    a.ntau = ntau;
    a.corint = rad->corint != 0;
    a.sink = ctx->sink;
    hipError_t e = hd::launch_rad_chunk(nn, a, radiances, stream);
    if (e != hipSuccess)
      return fail(ctx, HD_EHIP, "hd_solve_radiance: launch failed: %s", hipGetErrorString(e));
  }
  return HD_OK;
}

}  // namespace

extern "C" {

int hd_solve_radiance(hd_context* ctx, const hd_config* cfg, const hd_inputs* in,
                      const hd_radiance* rad, double* flux, double* uu, int* status,
                      void* stream) {
  if (!ctx) return fail(nullptr, HD_EINVAL, "hd_solve_radiance: null context");
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = validate_rad(ctx, cfg, in, rad, flux, uu);
  if (rc) return rc;
  if ((long)in->nwave * in->ncol == 0) return HD_OK;
  return run_solve(ctx, status, stream, "hd_solve_radiance", [&](int*& st, hipStream_t s) {
    return rad_enqueue(ctx, cfg, in, rad, flux, uu, st, s);
  });
}


}  // extern "C"
