/*
 * zmpc.h — C-ABI of the MI355X batched Wieber LIPM-ZMP MPC solver (libzmpc.so).
 *
 * This is the drop-in boundary for the reference hot path
 *   src/mpc_bipedal/controllers/zmp_controller.py  (ZMPController, reference @ 2025-12-26)
 * Every entry point names the reference code it replaces.  The Python host layer
 * (mpc_bipedal/_native.py, ctypes) binds exactly these symbols; see INTEGRATION.md.
 *
 * Conventions
 *  - All array pointers are DEVICE pointers (e.g. torch tensor .data_ptr()), contiguous,
 *    IEEE fp64 unless stated.  Nothing is copied to or from the host by the solve calls.
 *  - Calls are asynchronous on `stream` (a hipStream_t; NULL = the null stream).
 *  - Return 0 on success, a negative ZMPC_E* code on failure; zmpc_last_error() returns a
 *    thread-local message for the last failure on the calling thread.  No C++ exception
 *    crosses the ABI.
 *  - A plan is immutable after creation (and after its zmpc_plan_set_option calls, which
 *    belong before it is shared) and may be shared across threads and streams of its device.
 *  - The library reads no environment variable that changes a result: algorithm choices are
 *    explicit plan options (zmpc_plan_set_option); diagnostic ablations exist only in the
 *    separate diagnostics build (make diag → libzmpc_diag.so, -DZMPC_DIAG).
 *  - status[b] (int32, may be NULL) receives ZMPC_OK, or a per-instance failure flag
 *    (ZMPC_ST_*).  The reference raises RuntimeError("QP solver did not find a solution")
 *    for a failed strict solve (zmp_controller.py:193-194); the host layer does the same
 *    when any status is non-zero.
 */
#ifndef ZMPC_H
#define ZMPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZMPC_ABI_VERSION 7

/* return codes */
#define ZMPC_OK 0
#define ZMPC_EINVAL (-1)   /* bad argument (size, pointer, range) */
#define ZMPC_EHIP (-2)     /* HIP runtime error (message has hipGetErrorString) */
#define ZMPC_ENOMEM (-3)   /* device allocation failed */
#define ZMPC_ESTATE (-4)   /* plan does not support the request (e.g. strict workspace) */

/* per-instance status flags (bitwise OR) */
#define ZMPC_ST_MAXITER 1  /* strict active-set iteration cap reached */
#define ZMPC_ST_NONFINITE 2 /* a non-finite value was produced */
#define ZMPC_ST_FACTOR 4   /* reduced KKT matrix not positive definite (Herdt: also a
                              window with more footsteps than params.max_footsteps, flagged
                              on every walk of its 32-walk wave) */
#define ZMPC_ST_INFEASIBLE 8 /* Herdt: the swing polytope has no usable facet and the
                                unconstrained footstep lies outside it (degenerate or
                                unbounded half-spaces); since ABI 5 */

typedef struct zmpc_plan zmpc_plan;

/*
 * Build the batch-invariant solver plan on `device` (stream-ordered on `stream`, then
 * synchronised): the Toeplitz column p of Pu and Px (zmp_controller.py:162-171, built on
 * the device from the host-evaluated constants so they match the reference bit for bit),
 * M = PuᵀPu + (R/Q)·I (FP64 MFMA when N >= 64, zmp_controller.py:198), its Cholesky
 * factor, the gain row k = e0ᵀ M⁻¹ Puᵀ and kx = k·Px (the only part of
 * -inv(M) Puᵀ (Px x - z_ref) the reference uses, X[0], zmp_controller.py:198-199) and,
 * when strict != 0, the z-space inverse Hessian G = Pu (R·I + Q·PuᵀPu)⁻¹ Puᵀ of the
 * strict QP (zmp_controller.py:173-195).
 * Replaces the per-call matrix build in ZMPController.predict_wieber_axis
 * (zmp_controller.py:162-171) and the inverse at :198.
 *   T, T2_2 = T²/2, T3_6 = T³/6, hg = h/g, Thg = T·h/g: as Python evaluates them
 *   (mpc_bipedal/models/lipm_model.py:plan_constants).
 */
int zmpc_plan_create(int device, int32_t N, double T, double T2_2, double T3_6, double hg,
                     double Thg, double Q, double R, int32_t strict, void* stream,
                     zmpc_plan** out);

/* Release a plan (synchronises its device). */
int zmpc_plan_destroy(zmpc_plan* plan);

/* Plan quantities copied to HOST memory for inspection/tests.
 * what: 0 = p (N), 1 = Px (N*3, row-major), 2 = M (N*N), 3 = gain k (N), 4 = kx (3),
 *       5 = G (N*N, strict plans only), 6 = Cholesky factor L of M (N*N, lower),
 *       7 = Hz = Q·I + R·Pu⁻ᵀPu⁻¹ = G⁻¹ (N*N, strict plans only).
 * count = number of doubles dst can hold; must be >= the quantity's size. */
int zmpc_plan_export(const zmpc_plan* plan, int32_t what, double* dst_host, int64_t count);

/*
 * Work counters of a plan's active-set solvers, summed over its launches since creation or the
 * last reset (diagnostics for the roofline accounting; the reference has no equivalent).
 * Copied to HOST memory after synchronising the plan's device.  Strict box-QP solver
 * (zmpc_step / zmpc_rollout on a strict plan):
 *   [0] wave passes   (active-set passes of a 64-instance wave, lockstep)
 *   [1] instance passes (active-set iterations summed over instances and timesteps)
 *   [2] instance-slots through the working-set Riccati step (the rest of the
 *       [1] x N instance-slots took the free-tail step)
 *   [3] launches
 * Herdt joint footstep QP (zmpc_herdt_rollout / zmpc_herdt_step, any plan; since ABI 4):
 *   [4] wave passes, [5] instance passes (one instance = one walk axis),
 *   [6] sum over instance passes of the window's footstep count m, [7] the same of m^2
 * Maxima (since ABI 6): [8] the most active-set passes any one strict solve took,
 *   [9] the same for the Herdt solver (passes of the solve's lane pair)
 * count = number of uint64 dst can hold (at most ZMPC_NCOUNTERS are written); reset != 0
 * zeroes the counters after the copy.  Since ABI 3 ([0..3]); [4..7] since ABI 4; [8..9]
 * since ABI 6.
 */
#define ZMPC_NCOUNTERS 10
int zmpc_plan_counters(const zmpc_plan* plan, uint64_t* dst_host, int32_t count, int32_t reset);

/*
 * Durations in milliseconds of the plan-build stages of zmpc_plan_create (HIP events recorded
 * on the creation stream between the stages; the reference rebuilds the same quantities in
 * every predict_wieber_axis call, zmp_controller.py:162-171,198).  Since ABI 5.
 *   [0] p, Px                        [1] M = PuᵀPu + (R/Q)·I (FP64 MFMA Gram at N >= 64)
 *   [2] Cholesky M = L·Lᵀ (blocked)  [3] gain row k, kx (two triangular solves)
 *   [4] rollout scan propagators     [5] FFT correlation tables
 *   [6] strict: X = L⁻¹·Puᵀ          [7] strict: G = XᵀX / Q (FP64 MFMA Gram)
 *   [8] strict: v = Pu⁻¹·e0          [9] strict: Hz = Q·I + R·VᵀV (FP64 MFMA Gram)
 *   [10] strict: LQ free-tail table  [11] total
 * Stages a plan does not run read 0.  count = floats dst can hold (at most ZMPC_PLAN_STAGES
 * are written).
 */
#define ZMPC_PLAN_STAGES 12
int zmpc_plan_timings(const zmpc_plan* plan, float* dst_host, int32_t count);

/*
 * Algorithm selection on a plan (since ABI 7).  Every option chooses between forms that compute
 * the same solution — bitwise for ZMPC_OPT_KICK_ORDER, to rounding for the others (the tests hold
 * each pair to <= 1e-11 on O(1) states); zmpc_plan_create sets the defaults (value 0 unless
 * stated).  For cross-checks and A/B timing; the reference has no counterpart.
 *   ZMPC_OPT_CORRELATION    unconstrained rollouts: 0 = auto (the sparse-difference correlation
 *                           for walks whose z_ref changes at most 40 (64 for walks of more than
 *                           513 samples) times per axis), 1 = the dense forms only
 *   ZMPC_OPT_LONG_WALK      unconstrained walks of more than 513 samples: 0 = auto,
 *                           1 = direct correlation, 2 = FFT correlation (where the transform
 *                           fits the workgroup), 3 = the chunked one-wave kernel
 *   ZMPC_OPT_ROLLOUT_KERNEL unconstrained walks of at most 513 samples: 0 = auto, 1 = the
 *                           one-wave-per-walk kernel (the cross-check of the split kernels)
 *   ZMPC_OPT_KICK_ORDER     strict rollouts: 1 = walks mapped to lanes in (kick step, kick)
 *                           order (default), 0 = input order
 *   ZMPC_OPT_STRICT_SOLVER  strict plans: 0 = auto (small batches — up to 16384 (walk, axis)
 *                           instances — the parallel-in-time one-instance-per-wavefront kernel,
 *                           larger ones the LQ lane-per-instance kernel), 1 = the reduced-
 *                           Cholesky tile kernel (16 instances per workgroup; cross-check),
 *                           2 = the reduced-Cholesky one-instance-per-wavefront kernel
 *                           (cross-check), 3 = the LQ kernel, 4 = the parallel-in-time kernel
 *                           (1 and 2: horizons up to 512; 4: up to 960)
 *   ZMPC_OPT_STRICT_BOUNDS  strict rollouts on the LQ kernel: 0 = auto (run-length bounds;
 *                           rows for a shared CoP before round 5), 1 = the bounds staged one row
 *                           per sample, 2 = run-length bounds (one entry per run of equal
 *                           bounds); bitwise the same results
 * Returns ZMPC_EINVAL for an unknown option or value.
 */
#define ZMPC_OPT_CORRELATION 0
#define ZMPC_OPT_LONG_WALK 1
#define ZMPC_OPT_ROLLOUT_KERNEL 2
#define ZMPC_OPT_KICK_ORDER 3
#define ZMPC_OPT_STRICT_SOLVER 4
#define ZMPC_OPT_STRICT_BOUNDS 5
#define ZMPC_NOPTIONS 6
int zmpc_plan_set_option(zmpc_plan* plan, int32_t option, int64_t value);
int zmpc_plan_get_option(const zmpc_plan* plan, int32_t option, int64_t* value);

/*
 * Batched ZMPController.predict_wieber_axis (zmp_controller.py:149-201):
 * B independent one-axis QP solves, one per instance b:
 *   x[b] (3) state, zmax_win[b], zmin_win[b] (N) the preview window
 *   → x_next[b] (3) = A x + B·u0, u0 = first jerk of the QP solution
 *     (unconstrained: :196-198; strict box-QP: :173-195).
 */
int zmpc_step(const zmpc_plan* plan, int64_t B, const double* x, const double* zmax_win,
              const double* zmin_win, double* x_next, int32_t* status, void* stream);

/*
 * Batched Wieber rollout: ZMPController.generate_com_trajectory_wieber
 * (zmp_controller.py:59-108) and generate_state_trajectory_wieber (:110-147) for B walks.
 *   zmax, zmin : [B, n, 2]   CoP bounds per walk (x, y); the window at step i is rows
 *                            i+1 .. i+N, padded with the last row (:81-88)
 *   bounds_stride            doubles between consecutive walks' bound arrays: 2n for a
 *                            dense [B,n,2] batch, 0 when every walk shares one CoP
 *                            (e.g. a disturbance sweep over one footstep plan)
 *   x0         : [B, 2, 3]   initial (x-axis, y-axis) states
 *   kick       : [B] or NULL velocity impulse dt·F_ext/m subtracted from the y state
 *                            produced at step kick_step (:90,105-106); NULL = no force
 *   hist       : [B, n, 2, 3] output state history, hist[:,0] = x0
 * n >= 1.  The CoM trajectory of the reference is hist[:, :, :, 0].
 */
int zmpc_rollout(const zmpc_plan* plan, int64_t B, int64_t n, const double* zmax,
                 const double* zmin, int64_t bounds_stride, const double* x0,
                 const double* kick, int64_t kick_step, double* hist, int32_t* status,
                 void* stream);

/*
 * zmpc_rollout with a kick step per walk (ragged batches: the reference applies the force at
 * step n_b//2 of each walk, zmp_controller.py:90).  kick_steps: [B] int64 device array; a
 * step outside [0, n-1) means no kick for that walk.  Since ABI 2.
 */
int zmpc_rollout_kicks(const zmpc_plan* plan, int64_t B, int64_t n, const double* zmax,
                       const double* zmin, int64_t bounds_stride, const double* x0,
                       const double* kick, const int64_t* kick_steps, double* hist,
                       int32_t* status, void* stream);

/*
 * Batched CoP-bound producer: CoPGenerator.generate_cop_trajectory
 * (generators/cop_generator.py:34-115) over the footstep plan of
 * generators/footstep_generator.py:19-49, one walk per set of parameters.
 *   params : [B, 7] device doubles = distance, step_length, foot_spread, ssp_duration,
 *            dsp_duration, standing_duration, dt (the reference's float clock t += dt is
 *            reproduced exactly, so the sample counts match)
 *   n_cap = 0: count only — n_out[b] = samples of walk b (int64 device array)
 *   n_cap > 0: zmax, zmin [B, n_cap, 2] (rows past n_b repeat the walk's last row, the
 *            rollout's own window padding), states [B, n_cap] int8 (0 STANDING,
 *            1 DOUBLE_SUPPORT, 2 SINGLE_SUPPORT, -1 padding) or NULL, n_out or NULL.
 * Since ABI 2.
 */
int zmpc_cop_generate(int device, int64_t B, const double* params, int64_t n_cap,
                      double* zmax, double* zmin, int8_t* states, int64_t* n_out,
                      void* stream);

/*
 * Herdt joint footstep QP (config.method == "herdt"), since ABI 4.
 * The plan supplies N (horizon) and the LIPM constants (dt, h, g); its strict flag is unused.
 * Support states are int8: 0 STANDING, 1 DOUBLE_SUPPORT, 2 SINGLE_SUPPORT (cop_generator.py:11-15).
 */
#define ZMPC_HERDT_MAX_FACETS 16
typedef struct zmpc_herdt_params {
  double alpha, beta, gamma;         /* cost weights (config.py:42-45) */
  double foot_length, foot_width;    /* ZMP box around the foot centre: ±½·dim (:666, :680) */
  double foot_spread;                /* initial y foot position, standing hull (:457, :726-731) */
  int32_t nfacets[2];                /* facets of the left / right swing polytope */
  double facets[2][ZMPC_HERDT_MAX_FACETS][3]; /* (a_x, a_y, b): a·(f − f_current) <= b, the
                                        reference's _polytope_halfspace (:828-865) */
  int32_t max_footsteps;             /* most footsteps (support segments after the current
                                        one) inside any horizon window of the batch, <= 8 */
  int32_t max_passes;                /* active-set pass cap per joint QP (0: the default 64).
                                        A solve that reaches it keeps its last iterate (as OSQP
                                        returns its iterate at its own iteration limit) and sets
                                        ZMPC_ST_MAXITER.  A solve whose swing polytope is
                                        infeasible — the analogue of OSQP returning no solution
                                        — takes the reference's failure fallback
                                        (zmp_controller.py:796-802: zero jerk on both axes, the
                                        first footstep at the air foot's centre; the current
                                        foot for zmpc_herdt_step) and sets ZMPC_ST_INFEASIBLE */
} zmpc_herdt_params;

/*
 * Batched ZMPController.generate_com_trajectory_herdt (zmp_controller.py:435-531) over
 * predict_herdt_joint (:533-826) for B walks of n samples (exact QP solution; the reference's
 * cvxpy/OSQP result differs by up to OSQP's tolerances).
 *   v_ref [B, n, 2] reference velocities (v_stride doubles between walks, 0 = shared)
 *   states [B, n] int8 (s_stride bytes between walks, 0 = shared)
 *   nb_next [B, n] int32: find_nb_steps(padded states)[i][0] (:470), the divisor of the
 *            air-foot interpolation (:497-500) (nb_stride elements between walks, 0 = shared)
 *   x0 [B, 2, 3] initial (x, y) states; kick [B] or NULL: y-velocity impulse dt·F_ext/m
 *            subtracted at step kick_step (:525-526)
 *   hist [B, n, 2, 3] state history; foot [B, n, 2] foot positions (foot_hist, :529-530)
 */
int zmpc_herdt_rollout(const zmpc_plan* plan, const zmpc_herdt_params* params, int64_t B,
                       int64_t n, const double* v_ref, int64_t v_stride, const int8_t* states,
                       int64_t s_stride, const int32_t* nb_next, int64_t nb_stride,
                       const double* x0, const double* kick, int64_t kick_step, double* hist,
                       double* foot, int32_t* status, void* stream);

/*
 * Batched predict_herdt_joint (zmp_controller.py:533-826), one QP per instance, cold start:
 *   x [B, 2, 3] (x, y) states; v_win [B, N, 2] window of v_ref; s_win [B, N] window states;
 *   current [B] int8 current support state; foot [B, 2] current foot (x_fc, y_fc);
 *   side [B] int8 (0 left, 1 right)
 *   → x_next [B, 2, 3]; step [B, 2] first planned footstep (NaN when the window holds none,
 *     the reference's None).
 */
int zmpc_herdt_step(const zmpc_plan* plan, const zmpc_herdt_params* params, int64_t B,
                    const double* x, const double* v_win, const int8_t* s_win,
                    const int8_t* current, const double* foot, const int8_t* side,
                    double* x_next, double* step, int32_t* status, void* stream);

/* Message describing the last failure on the calling thread ("" if none). */
const char* zmpc_last_error(void);

/* ZMPC_ABI_VERSION of the loaded library. */
int zmpc_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* ZMPC_H */
