// Internal declarations shared by the HIP translation units of libzmpc.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "zmpc.h"

// Scalar LIPM constants of zmp_controller.py:18-20 (A = [[1,T,T²/2],[0,1,T],[0,0,1]],
// B = [T³/6, T²/2, T]ᵀ), evaluated on the host as Python evaluates them.
// Rollout scan propagators per chunk width C = 1..8: (Ā^C)^(2^r), r = 0..kScanLevels-1
// (64-lane Kogge-Stone rounds use r <= 5; the 128-lane kernels' cross-wave offset uses r = 6).
constexpr int kScanLevels = 7;
constexpr int kScanStride = kScanLevels * 9;
// ... followed by the per-lane powers (Ā^C)^k, k = 0..32, [8][33][9] (the DPP scan's cross-row
// steps, rollout.hip scan_dpp)
constexpr int kScanPowOff = 8 * kScanStride;
// ... and the chunk-sum columns Ā^p B, Ā^p e1 (p = 0..7), [8][6] (rollout.hip split_walk: a
// lane's chunk end state Σ_q Ā^(C−1−q) B f_q, and the kick's Ā^(C−1−q) e1)
constexpr int kScanGOff = kScanPowOff + 8 * 33 * 9;
constexpr int kScanDoubles = kScanGOff + 8 * 6;

// Longest strict horizon of the LQ kernel (strict_lq.hip lq_variant_for: its per-wave LDS —
// slot flags, 2 bits per slot and lane since round 6, and the parked V and state — fits a CU at
// two waves per workgroup, checked there by a static_assert); unchanged since round 5.
constexpr int ZMPC_STRICT_MAX_N = 2464;

struct LipmConsts {
  double T;     // A[0,1] = A[1,2] = B[2]
  double T2_2;  // A[0,2] = B[1]
  double T3_6;  // B[0]
};

struct zmpc_plan {
  int device = 0;
  int cus = 0;      // compute units of the plan's device (grid sizing of the launches)
  int N = 0;        // horizon (nb_steps)
  int Kpad = 0;     // N rounded up to a multiple of 16, the zero-padded length of k
  int strict = 0;
  double T = 0, T2_2 = 0, T3_6 = 0, hg = 0, Thg = 0, Q = 1, R = 0;
  LipmConsts lc{};
  // device buffers
  double* p = nullptr;   // [N] Toeplitz column of Pu
  double* Px = nullptr;  // [N,3]
  double* M = nullptr;   // [N,N] PuᵀPu + (R/Q) I
  double* L = nullptr;   // [N,N] lower Cholesky factor of M
  double* k = nullptr;   // [Kpad] gain row e0ᵀ M⁻¹ Puᵀ (zero-padded)
  double* kx = nullptr;  // [3]  k·Px
  double* kffa = nullptr;  // [kffa_rows(N)][4] two-parallel fast-FIR taps of k (rollout.hip):
                           // (E_m, O_m, E_m + O_{m−1}, 0), E_m = k_{2m}, O_m = k_{2m+1}, zero past N
  double* ksum = nullptr;  // [ksum_rows(N)] suffix sums of k for the sparse-difference
                           // correlation (rollout.hip axis_correlate_sparse; layout at ksum_rows)
  double* scanP = nullptr;  // [8][kScanLevels][9] (Ā^C)^(2^r) rollout scan propagators, then
                            // [8][33][9] (Ā^C)^k (kScanPowOff)
  double* X = nullptr;   // [N,N] L⁻¹ Puᵀ (strict plans)
  double* G = nullptr;   // [N,N] Pu (R I + Q PuᵀPu)⁻¹ Puᵀ (strict plans)
  double* v = nullptr;   // [N]   first column of Pu⁻¹ (strict plans)
  double* Hz = nullptr;  // [N,N] Q I + R Pu⁻ᵀPu⁻¹ = G⁻¹ (strict plans)
  int* info = nullptr;   // [1] factorisation status
  // strict reduced-Cholesky solver (strict.hip): persistent-grid slots (its factor scratch is
  // allocated per launch, stream-ordered)
  int strict_slots = 0;
  // strict LQ solver (strict_lq.hip): free-tail Riccati table [N][16] and work counters
  double* lqtab = nullptr;
  unsigned long long* lqcnt = nullptr;  // [ZMPC_NCOUNTERS]
  // FFT correlation of long unconstrained walks (rollout.hip): twiddles e^{−2πi m/PT}
  // [PT] complex, and per transform size P = 2^p in [kFftPmin, PT] the spectrum of the
  // gain kernel g[d] = k_{d−1} (d = 1..N), DFT(g)/P, at complex offset P − kFftPmin
  double* fft_tw = nullptr;
  double* fft_g = nullptr;
  // plan-build stage durations (zmpc_plan_timings), milliseconds
  float stage_ms[ZMPC_PLAN_STAGES] = {};
  // algorithm options (zmpc_plan_set_option), defaults as include/zmpc.h
  int opt[ZMPC_NOPTIONS] = {0, 0, 0, 1, 0, 0};
};

// rows of the fast-FIR tap table: m = 0..⌈(N+1)/2⌉−1, plus zero rows for an unrolled loop
__host__ __device__ constexpr int kffa_rows(int N) { return (N + 2) / 2 + 8; }

// suffix sums S_j = Σ_{j' ≥ j} k_{j'} of the gain row: entry i = S_{i−8} for 1 ≤ i − 8 ≤ N − 1,
// zero elsewhere in [0, N + 16) (so a lane's 8-wide read at any clamped offset stays inside),
// S_0 at N + 16
__host__ __device__ constexpr int ksum_rows(int N) { return N + 18; }
__host__ __device__ constexpr int ksum_s0(int N) { return N + 16; }

constexpr int kFftPT = 8192;    // largest transform (twiddle table size)
constexpr int kFftPmin = 256;   // smallest transform with a gain spectrum
constexpr int kFftGComplex = 2 * kFftPT - kFftPmin;  // Σ_P P over P = kFftPmin..kFftPT

// kernels launchers (plan.hip); ev (may be NULL): ZMPC_PLAN_STAGES events, ev[0] recorded
// before the first stage and ev[i + 1] after stage i for stages 0..9 of include/zmpc.h
// zmpc_plan_timings (stages the plan skips record their event right after the previous one);
// the caller records ev[11] after stage 10 (the strict LQ table)
hipError_t zmpc_launch_plan(zmpc_plan* p, hipStream_t s, hipEvent_t* ev);

// batched CoP-bound producer (cop.hip): params [B][7] = distance, step_length, foot_spread,
// ssp, dsp, standing, dt; n_cap = 0 counts only (n_out)
hipError_t zmpc_launch_cop(int64_t B, const double* params, int64_t n_cap, double* zmax,
                           double* zmin, int8_t* states, int64_t* n_out, hipStream_t s);

// unconstrained rollout / step (rollout.hip)
hipError_t zmpc_launch_rollout_unc(const zmpc_plan* p, int64_t B, int64_t n, const double* zmax,
                                   const double* zmin, int64_t bstride, const double* x0,
                                   const double* kick, int64_t kick_step,
                                   const int64_t* kick_steps, double* hist, int32_t* status,
                                   hipStream_t s, std::string* why);
hipError_t zmpc_launch_step_unc(const zmpc_plan* p, int64_t B, const double* x,
                                const double* zmax_win, const double* zmin_win, double* x_next,
                                int32_t* status, hipStream_t s);

// strict box-QP rollout / step (strict.hip)
hipError_t zmpc_launch_rollout_strict(const zmpc_plan* p, int64_t B, int64_t n,
                                      const double* zmax, const double* zmin, int64_t bstride,
                                      const double* x0,
                                      const double* kick, int64_t kick_step,
                                      const int64_t* kick_steps, double* hist,
                                      int32_t* status, hipStream_t s, std::string* why);
hipError_t zmpc_launch_step_strict(const zmpc_plan* p, int64_t B, const double* x,
                                   const double* zmax_win, const double* zmin_win,
                                   double* x_next, int32_t* status, hipStream_t s,
                                   std::string* why);

// strict box-QP in LQ form, one instance per lane (strict_lq.hip); the default strict path
hipError_t zmpc_launch_rollout_strict_lq(const zmpc_plan* p, int64_t B, int64_t n,
                                         const double* zmax, const double* zmin,
                                         int64_t bstride, const double* x0, const double* kick,
                                         int64_t kick_step, const int64_t* kick_steps,
                                         double* hist, int32_t* status, hipStream_t s,
                                         std::string* why);
hipError_t zmpc_launch_step_strict_lq(const zmpc_plan* p, int64_t B, const double* x,
                                      const double* zmax_win, const double* zmin_win,
                                      double* x_next, int32_t* status, hipStream_t s,
                                      std::string* why);
bool zmpc_strict_lq_supported(const zmpc_plan* p);
hipError_t zmpc_strict_lq_set_attrs();
size_t zmpc_strict_lq_table_doubles(int N);
hipError_t zmpc_strict_lq_build_table(zmpc_plan* p, hipStream_t s);

// strict box-QP for small batches, one instance per wave, parallel in time (strict_scan.hip)
hipError_t zmpc_launch_rollout_strict_scan(const zmpc_plan* p, int64_t B, int64_t n,
                                           const double* zmax, const double* zmin,
                                           int64_t bstride, const double* x0, const double* kick,
                                           int64_t kick_step, const int64_t* kick_steps,
                                           double* hist, int32_t* status, hipStream_t s,
                                           std::string* why);
hipError_t zmpc_launch_step_strict_scan(const zmpc_plan* p, int64_t B, const double* x,
                                        const double* zmax_win, const double* zmin_win,
                                        double* x_next, int32_t* status, hipStream_t s,
                                        std::string* why);
bool zmpc_strict_scan_supported(const zmpc_plan* p);

// walk order for the lane-per-instance kernels (order.hip): perm[B] = the walks sorted by
// (kick step, kick), so that a wave's lanes take similar disturbances; ws of
// zmpc_kick_order_bytes(B) bytes (device, stream-ordered)
size_t zmpc_kick_order_bytes(int64_t B);
hipError_t zmpc_kick_order(const double* kick, const int64_t* kick_steps, int64_t kick_step,
                           int64_t B, int32_t* perm, void* ws, hipStream_t s);

// Herdt joint footstep QP (herdt.hip); support states as cop_generator.State
constexpr int ZMPC_STANDING = 0, ZMPC_DOUBLE_SUPPORT = 1, ZMPC_SINGLE_SUPPORT = 2;
hipError_t zmpc_launch_herdt(const zmpc_plan* p, const zmpc_herdt_params* prm, int64_t B,
                             int64_t n, int window_mode, const double* vref, int64_t vs,
                             const int8_t* st, int64_t ss, const int32_t* nb, int64_t ns,
                             const double* x0, const double* kick, int64_t kick_step,
                             const int8_t* cur0, const double* fc0, const int8_t* side0,
                             double* hist, double* foot, int32_t* status, hipStream_t s,
                             std::string* why);
hipError_t zmpc_herdt_set_attrs();

hipError_t zmpc_rollout_unc_set_attrs();
hipError_t zmpc_strict_set_attrs();

// Dynamic LDS the rollout kernel needs for (N, n); 0 if it does not fit a CU.
size_t zmpc_rollout_unc_lds_bytes(int Kpad, int64_t n);
