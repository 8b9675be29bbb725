// C-ABI of libzmpc.so (declared in include/zmpc.h).  Host-side only: argument checks,
// device selection, buffer ownership of plans, error reporting.  No compute runs here.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "zmpc_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(ZMPC_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// Switch to the plan's device for the duration of a call, restore the caller's device.
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    if ((err = hipGetDevice(&prev)) != hipSuccess) return;
    if (prev != dev) err = hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// A launcher's verdict: an argument it rejects comes with a reason (EINVAL), a failed
// per-launch workspace allocation is hipErrorOutOfMemory (ENOMEM), anything else is HIP's.
int launch_result(hipError_t e, const std::string& why, const char* what) {
  if (e == hipSuccess) return ZMPC_OK;
  if (!why.empty()) return fail(ZMPC_EINVAL, why);
  if (e == hipErrorOutOfMemory)
    return fail(ZMPC_ENOMEM, std::string(what) + ": device workspace allocation failed");
  return hip_fail(e, (std::string(what) + " launch").c_str());
}

void free_plan(zmpc_plan* p) {
  if (!p) return;
  double* bufs[] = {p->p, p->Px, p->M,  p->L,     p->k,      p->kx,     p->kffa,
                    p->ksum, p->X, p->G,  p->v,  p->Hz,    p->scanP,  p->fft_tw, p->fft_g};
  for (double* b : bufs)
    if (b) (void)hipFree(b);
  if (p->info) (void)hipFree(p->info);
  if (p->lqtab) (void)hipFree(p->lqtab);
  if (p->lqcnt) (void)hipFree(p->lqcnt);
  delete p;
}

// per-device one-time kernel attributes and pool threshold; plan creation may run on several
// host threads at once (zmpc.h: plans are shareable across threads), so the check-and-set is
// under a lock
std::mutex g_attrs_mu;
bool attrs_done[64] = {};

}  // namespace

extern "C" {

int zmpc_abi_version(void) { return ZMPC_ABI_VERSION; }

const char* zmpc_last_error(void) { return g_err.c_str(); }

int zmpc_plan_create(int device, int32_t N, double T, double T2_2, double T3_6, double hg,
                     double Thg, double Q, double R, int32_t strict, void* stream,
                     zmpc_plan** out) {
  g_err.clear();
  if (!out) return fail(ZMPC_EINVAL, "out is NULL");
  *out = nullptr;
  if (N < 1 || N > 4096) return fail(ZMPC_EINVAL, "horizon N must be in [1, 4096]");
  if (!(T > 0) || !(Q > 0) || !(R >= 0))
    return fail(ZMPC_EINVAL, "need dt > 0, Q > 0, R >= 0");
  if (strict && N > ZMPC_STRICT_MAX_N)
    return fail(ZMPC_EINVAL, "strict horizon N must be <= " + std::to_string(ZMPC_STRICT_MAX_N));
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
  if (device < 0 || device >= ndev) return fail(ZMPC_EINVAL, "device index out of range");
  DeviceGuard g(device);
  if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
  std::unique_lock<std::mutex> attrs_lock(g_attrs_mu);
  if (device >= 64 || !attrs_done[device]) {
    if ((e = zmpc_rollout_unc_set_attrs()) != hipSuccess) return hip_fail(e, "set LDS attrs");
    if ((e = zmpc_strict_set_attrs()) != hipSuccess) return hip_fail(e, "set LDS attrs");
    if ((e = zmpc_strict_lq_set_attrs()) != hipSuccess) return hip_fail(e, "set LDS attrs");
    if ((e = zmpc_herdt_set_attrs()) != hipSuccess) return hip_fail(e, "set LDS attrs");
    // the strict solvers' per-launch workspaces come from the stream-ordered pool: keep up to
    // ZMPC_POOL_KEEP_MB (default 4096) of freed blocks in the pool across synchronisations
    // instead of returning them to the driver every time; anything above is released
    hipMemPool_t pool = nullptr;
    if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess && pool) {
      // (the only environment variable of the product library; memory retention only)
      const char* env = getenv("ZMPC_POOL_KEEP_MB");
      long long mb = 4096;
      if (env) {
        char* end = nullptr;
        const long long v = strtoll(env, &end, 10);
        if (end != env && *end == '\0' && v >= 0 && v <= (1ll << 22))
          mb = v;
        else
          fprintf(stderr, "libzmpc: ignoring ZMPC_POOL_KEEP_MB=%s (expected 0..%lld MiB)\n",
                  env, 1ll << 22);
      }
      uint64_t keep = (uint64_t)mb << 20;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
    if (device < 64) attrs_done[device] = true;
  }
  attrs_lock.unlock();

  zmpc_plan* P = new zmpc_plan();
  P->device = device;
  if ((e = hipDeviceGetAttribute(&P->cus, hipDeviceAttributeMultiprocessorCount, device)) !=
      hipSuccess) {
    delete P;
    return hip_fail(e, "hipDeviceGetAttribute");
  }
  P->N = N;
  P->Kpad = (N + 15) & ~15;
  P->strict = strict ? 1 : 0;
  P->T = T;
  P->T2_2 = T2_2;
  P->T3_6 = T3_6;
  P->hg = hg;
  P->Thg = Thg;
  P->Q = Q;
  P->R = R;
  P->lc = LipmConsts{T, T2_2, T3_6};
  const size_t nn = (size_t)N * N;
  struct {
    double** ptr;
    size_t n;
  } allocs[] = {{&P->p, (size_t)N},  {&P->Px, 3 * (size_t)N}, {&P->M, nn}, {&P->L, nn},
                {&P->k, (size_t)P->Kpad + 64}, {&P->kx, 4}, {&P->kffa, 4 * (size_t)kffa_rows(N)},
                {&P->ksum, (size_t)ksum_rows(N)},
                {&P->scanP, kScanDoubles},
                {&P->X, strict ? nn : 0}, {&P->G, strict ? nn : 0},
                {&P->v, strict ? (size_t)N : 0}, {&P->Hz, strict ? nn : 0},
                {&P->fft_tw, 2 * (size_t)kFftPT}, {&P->fft_g, 2 * (size_t)kFftGComplex}};
  for (auto& a : allocs) {
    if (a.n == 0) continue;
    if ((e = hipMalloc((void**)a.ptr, a.n * sizeof(double))) != hipSuccess) {
      free_plan(P);
      return fail(ZMPC_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
  }
  if ((e = hipMalloc((void**)&P->info, sizeof(int))) != hipSuccess) {
    free_plan(P);
    return fail(ZMPC_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  if (strict) {
    P->strict_slots = 2 * P->cus;
    if ((e = hipMalloc((void**)&P->lqtab, zmpc_strict_lq_table_doubles(N) * sizeof(double))) !=
        hipSuccess) {
      free_plan(P);
      return fail(ZMPC_ENOMEM, std::string("hipMalloc strict table: ") + hipGetErrorString(e));
    }
  }
  // work counters of the active-set solvers (strict and Herdt), every plan
  if ((e = hipMalloc((void**)&P->lqcnt, ZMPC_NCOUNTERS * sizeof(unsigned long long))) !=
      hipSuccess) {
    free_plan(P);
    return fail(ZMPC_ENOMEM, std::string("hipMalloc counters: ") + hipGetErrorString(e));
  }
  hipStream_t s = (hipStream_t)stream;
  (void)hipMemsetAsync(P->k, 0, ((size_t)P->Kpad + 64) * sizeof(double), s);
  if (P->lqcnt)
    (void)hipMemsetAsync(P->lqcnt, 0, ZMPC_NCOUNTERS * sizeof(unsigned long long), s);
  // stage timings (zmpc_plan_timings): events between the plan-build stages
  hipEvent_t ev[ZMPC_PLAN_STAGES] = {};
  bool timed = true;
  for (auto& x : ev) timed = timed && hipEventCreate(&x) == hipSuccess;
  struct EvGuard {
    hipEvent_t* ev;
    ~EvGuard() {
      for (int i = 0; i < ZMPC_PLAN_STAGES; ++i)
        if (ev[i]) (void)hipEventDestroy(ev[i]);
    }
  } evg{ev};
  if ((e = zmpc_launch_plan(P, s, timed ? ev : nullptr)) != hipSuccess) {
    free_plan(P);
    return hip_fail(e, "plan kernels");
  }
  if (P->lqtab && (e = zmpc_strict_lq_build_table(P, s)) != hipSuccess) {
    free_plan(P);
    return hip_fail(e, "strict table kernel");
  }
  if (timed) (void)hipEventRecord(ev[ZMPC_PLAN_STAGES - 1], s);
  if ((e = hipStreamSynchronize(s)) != hipSuccess) {
    free_plan(P);
    return hip_fail(e, "plan synchronize");
  }
  if (timed) {
    for (int i = 0; i + 1 < ZMPC_PLAN_STAGES; ++i)
      (void)hipEventElapsedTime(&P->stage_ms[i], ev[i], ev[i + 1]);
    (void)hipEventElapsedTime(&P->stage_ms[ZMPC_PLAN_STAGES - 1], ev[0],
                              ev[ZMPC_PLAN_STAGES - 1]);
  }
  int info = 0;
  if ((e = hipMemcpy(&info, P->info, sizeof(int), hipMemcpyDeviceToHost)) != hipSuccess) {
    free_plan(P);
    return hip_fail(e, "plan info copy");
  }
#ifdef ZMPC_DIAG
  const bool keep_failed = getenv("ZMPC_DEBUG_PLAN") != nullptr;  // diagnostics: export it
#else
  const bool keep_failed = false;
#endif
  if (info != 0 && !keep_failed) {
    free_plan(P);
    return fail(ZMPC_ESTATE, "PuᵀPu + (R/Q)I is not positive definite (pivot " +
                                 std::to_string(info) + ")");
  }
  *out = P;
  return ZMPC_OK;
}

int zmpc_plan_destroy(zmpc_plan* plan) {
  g_err.clear();
  if (!plan) return ZMPC_OK;
  DeviceGuard g(plan->device);
  (void)hipDeviceSynchronize();
  free_plan(plan);
  return ZMPC_OK;
}

int zmpc_plan_timings(const zmpc_plan* P, float* dst, int32_t count) {
  g_err.clear();
  if (!P || !dst) return fail(ZMPC_EINVAL, "NULL plan or destination");
  for (int i = 0; i < count && i < ZMPC_PLAN_STAGES; ++i) dst[i] = P->stage_ms[i];
  return ZMPC_OK;
}

int zmpc_plan_set_option(zmpc_plan* P, int32_t option, int64_t value) {
  g_err.clear();
  if (!P) return fail(ZMPC_EINVAL, "NULL plan");
  static const int64_t hi[ZMPC_NOPTIONS] = {1, 3, 1, 1, 4, 2};  // largest value of each option
  if (option < 0 || option >= ZMPC_NOPTIONS) return fail(ZMPC_EINVAL, "unknown option");
  if (value < 0 || value > hi[option])
    return fail(ZMPC_EINVAL, "option value out of range (0.." + std::to_string(hi[option]) + ")");
  if (option == ZMPC_OPT_STRICT_SOLVER && (value == 1 || value == 2) &&
      (!P->strict || P->N > 512))
    return fail(ZMPC_EINVAL, "the reduced-Cholesky strict kernels need a strict plan, N <= 512");
  if (option == ZMPC_OPT_STRICT_SOLVER && value == 4 &&
      (!P->strict || !zmpc_strict_scan_supported(P)))
    return fail(ZMPC_EINVAL, "the small-batch strict kernel needs a strict plan, N <= 960");
  if (option == ZMPC_OPT_STRICT_SOLVER && value == 3 && !zmpc_strict_lq_supported(P))
    return fail(ZMPC_EINVAL, "the LQ strict kernel needs a strict plan, N <= " +
                                  std::to_string(ZMPC_STRICT_MAX_N));
  P->opt[option] = (int)value;
  return ZMPC_OK;
}

int zmpc_plan_get_option(const zmpc_plan* P, int32_t option, int64_t* value) {
  g_err.clear();
  if (!P || !value) return fail(ZMPC_EINVAL, "NULL plan or destination");
  if (option < 0 || option >= ZMPC_NOPTIONS) return fail(ZMPC_EINVAL, "unknown option");
  *value = P->opt[option];
  return ZMPC_OK;
}

int zmpc_plan_export(const zmpc_plan* P, int32_t what, double* dst, int64_t count) {
  g_err.clear();
  if (!P || !dst) return fail(ZMPC_EINVAL, "NULL plan or destination");
  const int64_t N = P->N;
  const double* src = nullptr;
  int64_t n = 0;
  switch (what) {
    case 0: src = P->p; n = N; break;
    case 1: src = P->Px; n = 3 * N; break;
    case 2: src = P->M; n = N * N; break;
    case 3: src = P->k; n = N; break;
    case 4: src = P->kx; n = 3; break;
    case 5: src = P->G; n = P->G ? N * N : 0; break;
    case 6: src = P->L; n = N * N; break;
    case 7: src = P->Hz; n = P->Hz ? N * N : 0; break;
    default: return fail(ZMPC_EINVAL, "unknown export id");
  }
  if (!src || n == 0) return fail(ZMPC_ESTATE, "quantity not held by this plan");
  if (count < n) return fail(ZMPC_EINVAL, "destination too small");
  DeviceGuard g(P->device);
  if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return hip_fail(e, "hipDeviceSynchronize");
  e = hipMemcpy(dst, src, n * sizeof(double), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_fail(e, "hipMemcpy");
  return ZMPC_OK;
}

int zmpc_plan_counters(const zmpc_plan* P, uint64_t* dst, int32_t count, int32_t reset) {
  g_err.clear();
  if (!P || !dst) return fail(ZMPC_EINVAL, "NULL plan or destination");
  if (count < 0) return fail(ZMPC_EINVAL, "count < 0");
  if (!P->lqcnt) return fail(ZMPC_ESTATE, "plan has no solver counters");
  DeviceGuard g(P->device);
  if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return hip_fail(e, "hipDeviceSynchronize");
  unsigned long long h[ZMPC_NCOUNTERS];
  e = hipMemcpy(h, P->lqcnt, sizeof(h), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_fail(e, "hipMemcpy");
  for (int i = 0; i < count && i < ZMPC_NCOUNTERS; ++i) dst[i] = (uint64_t)h[i];
  if (reset) {
    e = hipMemset(P->lqcnt, 0, sizeof(h));
    if (e != hipSuccess) return hip_fail(e, "hipMemset");
  }
  return ZMPC_OK;
}

int zmpc_step(const zmpc_plan* P, int64_t B, const double* x, const double* zmax_win,
              const double* zmin_win, double* x_next, int32_t* status, void* stream) {
  g_err.clear();
  if (!P) return fail(ZMPC_EINVAL, "NULL plan");
  if (B < 0) return fail(ZMPC_EINVAL, "B < 0");
  if (B == 0) return ZMPC_OK;
  if (!x || !zmax_win || !zmin_win || !x_next)
    return fail(ZMPC_EINVAL, "NULL array argument");
  if (B > (int64_t)0x7fffffff * 4) return fail(ZMPC_EINVAL, "batch too large");
  DeviceGuard g(P->device);
  if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
  std::string why;
  hipError_t e = P->strict ? zmpc_launch_step_strict(P, B, x, zmax_win, zmin_win, x_next, status,
                                                     (hipStream_t)stream, &why)
                           : zmpc_launch_step_unc(P, B, x, zmax_win, zmin_win, x_next, status,
                                                  (hipStream_t)stream);
  return launch_result(e, why, "zmpc_step");
}

static int rollout_impl(const zmpc_plan* P, int64_t B, int64_t n, const double* zmax,
                        const double* zmin, int64_t bounds_stride, const double* x0,
                        const double* kick, int64_t kick_step, const int64_t* kick_steps,
                        double* hist, int32_t* status, void* stream) {
  g_err.clear();
  if (!P) return fail(ZMPC_EINVAL, "NULL plan");
  if (B < 0 || n < 1) return fail(ZMPC_EINVAL, "need B >= 0 and n >= 1");
  if (B == 0) return ZMPC_OK;
  if (!zmax || !zmin || !x0 || !hist) return fail(ZMPC_EINVAL, "NULL array argument");
  if (B > 0x7fffffff) return fail(ZMPC_EINVAL, "batch too large");
  if (n > (1 << 24)) return fail(ZMPC_EINVAL, "walk too long");
  if (bounds_stride != 0 && bounds_stride < 2 * n)
    return fail(ZMPC_EINVAL, "bounds_stride must be 0 (shared CoP) or >= 2n");
  DeviceGuard g(P->device);
  if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
  std::string why;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = P->strict ? zmpc_launch_rollout_strict(P, B, n, zmax, zmin, bounds_stride, x0,
                                                        kick, kick_step, kick_steps, hist,
                                                        status, s, &why)
                           : zmpc_launch_rollout_unc(P, B, n, zmax, zmin, bounds_stride, x0,
                                                     kick, kick_step, kick_steps, hist, status,
                                                     s, &why);
  return launch_result(e, why, "zmpc_rollout");
}

int zmpc_rollout(const zmpc_plan* P, int64_t B, int64_t n, const double* zmax,
                 const double* zmin, int64_t bounds_stride, const double* x0,
                 const double* kick, int64_t kick_step, double* hist, int32_t* status,
                 void* stream) {
  return rollout_impl(P, B, n, zmax, zmin, bounds_stride, x0, kick, kick_step, nullptr, hist,
                      status, stream);
}

int zmpc_rollout_kicks(const zmpc_plan* P, int64_t B, int64_t n, const double* zmax,
                       const double* zmin, int64_t bounds_stride, const double* x0,
                       const double* kick, const int64_t* kick_steps, double* hist,
                       int32_t* status, void* stream) {
  if (!kick_steps) {
    g_err.clear();
    return fail(ZMPC_EINVAL, "kick_steps is NULL (use zmpc_rollout for one kick step)");
  }
  return rollout_impl(P, B, n, zmax, zmin, bounds_stride, x0, kick, -1, kick_steps, hist,
                      status, stream);
}

static int herdt_check(const zmpc_plan* P, const zmpc_herdt_params* prm, int64_t B) {
  if (!P || !prm) return fail(ZMPC_EINVAL, "NULL plan or params");
  if (B < 0) return fail(ZMPC_EINVAL, "B < 0");
  for (int sd = 0; sd < 2; ++sd)
    if (prm->nfacets[sd] < 3 || prm->nfacets[sd] > ZMPC_HERDT_MAX_FACETS)
      return fail(ZMPC_EINVAL, "polytope facets must be in [3, 16]");
  if (prm->max_footsteps < 0 || prm->max_footsteps > 8)
    return fail(ZMPC_EINVAL, "max_footsteps must be in [0, 8]");
  if (prm->max_passes < 0 || prm->max_passes > 100000)
    return fail(ZMPC_EINVAL, "max_passes must be in [0, 100000] (0: default)");
  if (!(prm->alpha > 0) || !(prm->beta >= 0) || !(prm->gamma > 0))
    return fail(ZMPC_EINVAL, "need alpha > 0, beta >= 0, gamma > 0");
  return ZMPC_OK;
}

int zmpc_herdt_rollout(const zmpc_plan* P, const zmpc_herdt_params* prm, int64_t B, int64_t n,
                       const double* v_ref, int64_t v_stride, const int8_t* states,
                       int64_t s_stride, const int32_t* nb_next, int64_t nb_stride,
                       const double* x0, const double* kick, int64_t kick_step, double* hist,
                       double* foot, int32_t* status, void* stream) {
  g_err.clear();
  int rc = herdt_check(P, prm, B);
  if (rc != ZMPC_OK) return rc;
  if (n < 1) return fail(ZMPC_EINVAL, "need n >= 1");
  if (B == 0) return ZMPC_OK;
  if (!v_ref || !states || !nb_next || !x0 || !hist || !foot)
    return fail(ZMPC_EINVAL, "NULL array argument");
  if (B > 0x7fffffff || n > (1 << 24)) return fail(ZMPC_EINVAL, "batch too large");
  if ((v_stride != 0 && v_stride < 2 * n) || (s_stride != 0 && s_stride < n) ||
      (nb_stride != 0 && nb_stride < n))
    return fail(ZMPC_EINVAL, "strides must be 0 (shared) or cover a whole walk");
  DeviceGuard g(P->device);
  if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
  hipStream_t s = (hipStream_t)stream;
  if (status) {
    hipError_t e = hipMemsetAsync(status, 0, sizeof(int32_t) * B, s);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync");
  }
  std::string why;
  hipError_t e = zmpc_launch_herdt(P, prm, B, n, 0, v_ref, v_stride, states, s_stride, nb_next,
                                   nb_stride, x0, kick, kick_step, nullptr, nullptr, nullptr,
                                   hist, foot, status, s, &why);
  return launch_result(e, why, "zmpc_herdt_rollout");
}

int zmpc_herdt_step(const zmpc_plan* P, const zmpc_herdt_params* prm, int64_t B,
                    const double* x, const double* v_win, const int8_t* s_win,
                    const int8_t* current, const double* foot, const int8_t* side,
                    double* x_next, double* step, int32_t* status, void* stream) {
  g_err.clear();
  int rc = herdt_check(P, prm, B);
  if (rc != ZMPC_OK) return rc;
  if (B == 0) return ZMPC_OK;
  if (!x || !v_win || !s_win || !current || !foot || !side || !x_next || !step)
    return fail(ZMPC_EINVAL, "NULL array argument");
  if (B > 0x7fffffff) return fail(ZMPC_EINVAL, "batch too large");
  DeviceGuard g(P->device);
  if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
  std::string why;
  hipError_t e = zmpc_launch_herdt(P, prm, B, 1, 1, v_win, 2 * (int64_t)P->N, s_win, P->N,
                                   nullptr, 0, x, nullptr, -1, current, foot, side, x_next, step,
                                   status, (hipStream_t)stream, &why);
  return launch_result(e, why, "zmpc_herdt_step");
}

int zmpc_cop_generate(int device, int64_t B, const double* params, int64_t n_cap,
                      double* zmax, double* zmin, int8_t* states, int64_t* n_out,
                      void* stream) {
  g_err.clear();
  if (B < 0 || n_cap < 0) return fail(ZMPC_EINVAL, "need B >= 0 and n_cap >= 0");
  if (B == 0) return ZMPC_OK;
  if (!params) return fail(ZMPC_EINVAL, "params is NULL");
  if (n_cap > 0 && (!zmax || !zmin)) return fail(ZMPC_EINVAL, "NULL output bounds");
  if (n_cap == 0 && !n_out) return fail(ZMPC_EINVAL, "n_cap = 0 needs n_out");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
  if (device < 0 || device >= ndev) return fail(ZMPC_EINVAL, "device index out of range");
  DeviceGuard g(device);
  if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
  e = zmpc_launch_cop(B, params, n_cap, n_cap > 0 ? zmax : nullptr, n_cap > 0 ? zmin : nullptr,
                      n_cap > 0 ? states : nullptr, n_out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "zmpc_cop_generate launch");
  return ZMPC_OK;
}

}  // extern "C"
