// Strict (ZMP box-constrained) Wieber QP, one instance per lane, solved in LQ form.
//
// Reference, per axis and timestep (zmp_controller.py:173-195, cvxpy→OSQP there):
//   min_J ½Q‖Px x + Pu J − z_ref‖² + ½R‖J‖²   s.t.  z_min ≤ Px x + Pu J ≤ z_max,  u0 = J[0]
// Pu[k,j] = C A^(k−j) B and Px[k] = C A^(k+1) (zmp_controller.py:162-171), so the predicted ZMP
// is the output of the LIPM itself: with x_0 = x and x_{k+1} = A x_k + B u_k,
//   z_k = C x_{k+1} = c1ᵀ x_k + p0 u_k,     c1 = (CA)ᵀ = [1, T, T²/2 − h/g],  p0 = CB = p(0).
// The QP is a linear-quadratic tracking problem over the horizon with one output bound per
// step.  For a working set (slot k active at t_k = z_max or z_min) the equality-constrained
// problem is solved exactly by a backward Riccati recursion: a free step minimises over u_k,
// an active step has u_k = (t_k − c1ᵀx_k)/p0 forced (p0 ≠ 0).  One unified update covers both
// (u = −K x − kff; K = Qux/Quu or c1/p0):
//   P ← Qxx − Qux_i K_j + K_i D_j,   s ← −qx + K qu − kff D,   D = Quu K − Qux (0 when free)
// with Qxx = Q c1c1ᵀ + AᵀPA, Qux = Q p0 c1 + BᵀPA, Quu = Q p0² + R + BᵀPB, qu = −Q p0 r − Bᵀs,
// qx = −Q r c1 − Aᵀs for the value function V(x) = ½xᵀPx − sᵀx.  The forward pass rolls the
// trajectory out and recovers, from λ_{k+1} = ∇V_{k+1}(x_{k+1}) = P x_{k+1} − s, the bound
// multipliers ν_k = −(R u_k + Bᵀλ_{k+1})/p0 − Q (t_k − r_k) of the active slots (the same ν
// as the z-space KKT  H δ − W + ν = 0 of strict.hip: ≥ 0 at upper, ≤ 0 at lower bounds).
// The working set comes from the same primal-dual active-set iteration as strict.hip —
// warm-started with the previous timestep's set shifted one slot, release wrong-signed
// multipliers, add violated free slots, stop when the set repeats — so the iterates and the
// solution are the same, at O(N) per pass instead of a reduced Cholesky.
//
// Mapping: a lane owns one instance (one walk, one axis) for the whole rollout; a wave holds
// 64 walks of one axis.  The bounds come in [axis][t][walk] (a staging transpose), so a wave's
// load of one window slot is 1 KiB contiguous ((z_max, z_min) pairs, 16 B per lane).  Per pass:
//   sweep A  backward Riccati over the horizon in segments of S steps, checkpointing (P, s)
//            at segment boundaries to a per-lane global slab (coalesced [.., 9, 64]);
//   sweep B  per segment from the front: reload its checkpoint, recompute its S Riccati
//            steps into registers (K, kff, bounds, flags), roll forward through it, check
//            primal/dual feasibility, update the slot flags (LDS, [N][64] bytes).
// Everything a pass touches besides the bounds and the checkpoints lives in registers.
//
// Free structure.  The quadratic part P of the value function (with the gain K and 1/Quu)
// depends on the working set only, never on the bounds.  Behind the last active slot of every
// lane of a wave (the free tail) they are the plan's table (zmpc_strict_lq_build_table, the
// same arithmetic), so a tail slot costs the linear recursion of s twice and the forward step
// (≈70 FLOP instead of ≈280), with no flag loads and no costate.  In sweep A, a segment before
// the tail in which no lane has an active slot runs the free form of the step (no per-lane
// selects, no D).
// The x axis of a walk is free almost everywhere; the y axis keeps active slots through most
// of the horizon while the robot steps (scripts/strict_active_stats.py).
#include <cstdio>
#include <cstring>
#include <cstdlib>

#include "zmpc_internal.h"

#pragma clang fp contract(off)  // every fused multiply-add below is an explicit fma()

namespace {

constexpr int LQ_MAXIT = 64;  // active-set pass cap (as strict.hip)
constexpr int TAB = 16;       // doubles per slot of the free-tail table: [0..2] K, [3] 1/Quu,
                              // [4..9] P after the slot (V_k: slots k..N−1 free), padding

struct LqArgs {
  int N, NS;             // horizon, segments ⌈N/S⌉
  int toff;              // window slot k reads time i + toff + k (1 rollout, 0 step)
  int window_mode;
  int drift;             // max timesteps a lane may run ahead of its wave's slowest lane
  int warm_free_term;    // warm start: slot N−2 (the previous solve's terminal slot) starts free
  int64_t n;             // samples per walk (rollout; 1 in window mode)
  int64_t nsteps;        // timesteps (n − 1, or 1)
  int64_t B;             // walks (rollout) or instances (step)
  // staged bounds, tiled [axis][group of 64 walks][row][64] of (z_max, z_min) pairs: row t of a
  // window slot holds the group's 64 pairs for time t, one 16-byte load per lane (rows past
  // n − 1 repeat the last sample — the window padding of zmp_controller.py:81-88 — so no
  // clamping in the kernel)
  int64_t rows;          // rows per (axis, group)
  int64_t groups;        // groups per axis in the staging (1 for a shared CoP)
  int shared;            // 1: every walk reads group 0 (bounds_stride = 0)
  const double2* hl;
  const double* x0;      // rollout [B,2,3], step [B,3]
  const double* kick;    // [B] or null
  int64_t kick_step;
  const int64_t* kick_steps;
  const int32_t* perm;   // walk of lane position b0 + lane (order.hip), or null (identity)
  double* out;           // rollout hist [B,n,2,3], step x_next [B,3]
  int32_t* status;
  double* ck;            // checkpoints [waves][NS][9][64]
  unsigned long long* cnt;  // plan work counters (zmpc_plan_counters), may be null
  // LIPM / QP constants.  The passes run in scaled coordinates ξ = [x0, T x1, T² x2],
  // v = T³ u, objective divided by Q: Â = [[1,1,½],[0,1,1],[0,0,1]], B̂ = [⅙, ½, 1],
  // z = ĉᵀξ + π v with ĉ = [1, 1, γ], γ = ½ − (h/g)/T², π = ⅙ − (h/g)/T² (= p(0)/T³),
  // cost ½(z − r)² + ½ρ v², ρ = R/(Q T⁶).  Few distinct constants, most of them inline.
  double T, T2, T3;      // reference-form state advance (zmp_controller.py:18-20,199)
  double Tsq, Tcu;       // T², T³ (coordinate scaling)
  double gam, pi, ipi;   // γ, π, 1/π
  double rho, quu0;      // ρ, π² + ρ
  double gipi, gam2, pig;  // γ/π, γ², πγ
  double tolnu;          // multiplier tolerance in the scaled objective (1e-13 / Q)
  int dbg;               // ZMPC_DEBUG_LQ (A/B diagnostics only): bit 0 = every wave reads the
                         // staged bounds of group 0 (window traffic from cache; results wrong),
                         // bits 1 / 2 = x / y waves exit at once
};

struct Ric {  // value function V(x) = ½xᵀPx − sᵀx
  double p00, p01, p02, p11, p12, p22, s0, s1, s2;
};

template <int S>
struct SegIn {  // a segment's window slots: bounds and working-set flags
  double hi[S], lo[S];
  int f[S];
};

template <int S>
struct SegOut {  // a segment's feedback (u = −K x − kff) and forward outputs, per step
  double K0[S], K1[S], K2[S], kf[S];
  double w[S];  // forward: z_k − r_k at free slots, u_k at active slots
  int nf[S];    // forward: the free slots' primal verdict (0 stays free, 1/2 violated)
};

constexpr double kH = 0.5, kS6 = 1.0 / 6.0;

// One backward Riccati step in scaled coordinates (see header and LqArgs), per-lane slot flag
// f.  Inputs: V_{k+1} in v, bounds.  Outputs the step's feedback v_k = −K ξ_k − kff.
template <bool LEAN>
__device__ __forceinline__ void ric_step(const LqArgs& a, Ric& v, double hi, double lo, int f,
                                         double& K0, double& K1, double& K2, double& kf) {
  // P B̂, B̂ᵀs, B̂ᵀPB̂
  const double pb0 = fma(kS6, v.p00, fma(kH, v.p01, v.p02));
  const double pb1 = fma(kS6, v.p01, fma(kH, v.p11, v.p12));
  const double pb2 = fma(kS6, v.p02, fma(kH, v.p12, v.p22));
  const double sb = fma(kS6, v.s0, fma(kH, v.s1, v.s2));
  const double bpb = fma(kS6, pb0, fma(kH, pb1, pb2));
  // P Â (columns 1, 2) and ÂᵀPÂ
  const double m01 = v.p00 + v.p01, m02 = fma(kH, v.p00, v.p01 + v.p02);
  const double m11 = v.p01 + v.p11, m12 = fma(kH, v.p01, v.p11 + v.p12);
  const double m22 = fma(kH, v.p02, v.p12 + v.p22);
  const double S11 = m01 + m11, S12 = m02 + m12, S22 = fma(kH, m02, m12 + m22);
  // Qux = π ĉ + (PB̂)ᵀÂ, Quu, qu, −qx = r ĉ + Âᵀs
  const double ux0 = a.pi + pb0;
  const double ux1 = a.pi + (pb0 + pb1);
  const double ux2 = a.pig + fma(kH, pb0, pb1 + pb2);
  const double Quu = a.quu0 + bpb;
  const double r = (hi + lo) / 2;  // z_ref (zmp_controller.py:184)
  const double qu = -fma(a.pi, r, sb);
  const double nqx0 = r + v.s0;
  const double nqx1 = r + (v.s0 + v.s1);
  const double nqx2 = fma(a.gam, r, fma(kH, v.s0, v.s1 + v.s2));
  const bool act = f != 0;
  // 1/Quu: hardware reciprocal + two Newton steps (Quu ≥ ρ + π² > 0, no special cases)
  double iq = __builtin_amdgcn_rcp(Quu);
  iq = fma(iq, fma(-Quu, iq, 1.0), iq);
  iq = fma(iq, fma(-Quu, iq, 1.0), iq);
  double P00, P01, P02, P11, P12, P22;
  if constexpr (LEAN) {
    // Few per-lane selects (each a pair of v_cndmask_b32): the free part (iqa) and the active
    // part (ka, kfa, zero at free slots) of the law, K = Qux·iqa + ka and kff = qu·iqa + kfa —
    // exactly ux·iq / qu·iq at a free slot and ĉ/π / −t/π at an active one.  D = Quu K − Qux is
    // formed unconditionally (rounding noise at free slots) and enters only through ka and kfa,
    // which vanish there: the same values as the per-field selects, up to the sign of a zero.
    const double iqa = act ? 0.0 : iq;
    const double ka01 = act ? a.ipi : 0.0;
    const double ka2 = act ? a.gipi : 0.0;
    const double tz = (f == 1) ? hi : ((f == 2) ? lo : 0.0);
    const double kfa = -tz * a.ipi;
    K0 = fma(ux0, iqa, ka01);
    K1 = fma(ux1, iqa, ka01);
    K2 = fma(ux2, iqa, ka2);
    kf = fma(qu, iqa, kfa);
    const double D0 = fma(Quu, K0, -ux0);
    const double D1 = fma(Quu, K1, -ux1);
    const double D2 = fma(Quu, K2, -ux2);
    // P = ĉĉᵀ + ÂᵀPÂ − Qux Kᵀ + K Dᵀ   (ĉĉᵀ = [[1,1,γ],[1,1,γ],[γ,γ,γ²]])
    P00 = fma(ka01, D0, fma(-ux0, K0, 1.0 + v.p00));
    P01 = fma(ka01, D1, fma(-ux0, K1, 1.0 + m01));
    P02 = fma(ka01, D2, fma(-ux0, K2, a.gam + m02));
    P11 = fma(ka01, D1, fma(-ux1, K1, 1.0 + S11));
    P12 = fma(ka01, D2, fma(-ux1, K2, a.gam + S12));
    P22 = fma(ka2, D2, fma(-ux2, K2, a.gam2 + S22));
    v.s0 = fma(-kfa, D0, fma(K0, qu, nqx0));
    v.s1 = fma(-kfa, D1, fma(K1, qu, nqx1));
    v.s2 = fma(-kfa, D2, fma(K2, qu, nqx2));
  } else {
    // per-field selects (sweep B: the lean form above needs more registers there)
    const double t = (f == 1) ? hi : lo;
    K0 = act ? a.ipi : ux0 * iq;
    K1 = act ? a.ipi : ux1 * iq;
    K2 = act ? a.gipi : ux2 * iq;
    kf = act ? -t * a.ipi : qu * iq;
    const double D0 = act ? fma(Quu, K0, -ux0) : 0.0;
    const double D1 = act ? fma(Quu, K1, -ux1) : 0.0;
    const double D2 = act ? fma(Quu, K2, -ux2) : 0.0;
    P00 = fma(K0, D0, fma(-ux0, K0, 1.0 + v.p00));
    P01 = fma(K0, D1, fma(-ux0, K1, 1.0 + m01));
    P02 = fma(K0, D2, fma(-ux0, K2, a.gam + m02));
    P11 = fma(K1, D1, fma(-ux1, K1, 1.0 + S11));
    P12 = fma(K1, D2, fma(-ux1, K2, a.gam + S12));
    P22 = fma(K2, D2, fma(-ux2, K2, a.gam2 + S22));
    v.s0 = fma(-kf, D0, fma(K0, qu, nqx0));
    v.s1 = fma(-kf, D1, fma(K1, qu, nqx1));
    v.s2 = fma(-kf, D2, fma(K2, qu, nqx2));
  }
  v.p00 = P00;
  v.p01 = P01;
  v.p02 = P02;
  v.p11 = P11;
  v.p12 = P12;
  v.p22 = P22;
}

// The same step for a free slot (ric_step with f = 0 and D = 0 folded: identical values up to
// the sign of a zero).  Also returns 1/Quu (the free-tail table).
__device__ __forceinline__ void ric_free(const LqArgs& a, Ric& v, double r, double& K0,
                                         double& K1, double& K2, double& kf, double& iqo) {
  const double pb0 = fma(kS6, v.p00, fma(kH, v.p01, v.p02));
  const double pb1 = fma(kS6, v.p01, fma(kH, v.p11, v.p12));
  const double pb2 = fma(kS6, v.p02, fma(kH, v.p12, v.p22));
  const double sb = fma(kS6, v.s0, fma(kH, v.s1, v.s2));
  const double bpb = fma(kS6, pb0, fma(kH, pb1, pb2));
  const double m01 = v.p00 + v.p01, m02 = fma(kH, v.p00, v.p01 + v.p02);
  const double m11 = v.p01 + v.p11, m12 = fma(kH, v.p01, v.p11 + v.p12);
  const double m22 = fma(kH, v.p02, v.p12 + v.p22);
  const double S11 = m01 + m11, S12 = m02 + m12, S22 = fma(kH, m02, m12 + m22);
  const double ux0 = a.pi + pb0;
  const double ux1 = a.pi + (pb0 + pb1);
  const double ux2 = a.pig + fma(kH, pb0, pb1 + pb2);
  const double Quu = a.quu0 + bpb;
  const double qu = -fma(a.pi, r, sb);
  const double nqx0 = r + v.s0;
  const double nqx1 = r + (v.s0 + v.s1);
  const double nqx2 = fma(a.gam, r, fma(kH, v.s0, v.s1 + v.s2));
  double iq = __builtin_amdgcn_rcp(Quu);
  iq = fma(iq, fma(-Quu, iq, 1.0), iq);
  iq = fma(iq, fma(-Quu, iq, 1.0), iq);
  K0 = ux0 * iq;
  K1 = ux1 * iq;
  K2 = ux2 * iq;
  kf = qu * iq;
  iqo = iq;
  const double P00 = fma(-ux0, K0, 1.0 + v.p00);
  const double P01 = fma(-ux0, K1, 1.0 + m01);
  const double P02 = fma(-ux0, K2, a.gam + m02);
  const double P11 = fma(-ux1, K1, 1.0 + S11);
  const double P12 = fma(-ux1, K2, a.gam + S12);
  const double P22 = fma(-ux2, K2, a.gam2 + S22);
  v.s0 = fma(K0, qu, nqx0);
  v.s1 = fma(K1, qu, nqx1);
  v.s2 = fma(K2, qu, nqx2);
  v.p00 = P00;
  v.p01 = P01;
  v.p02 = P02;
  v.p11 = P11;
  v.p12 = P12;
  v.p22 = P22;
}

// A free-tail step: P, K and 1/Quu come from the table, only s moves (ric_free's s update).
__device__ __forceinline__ void ric_tail(const LqArgs& a, Ric& v, double r, double K0, double K1,
                                         double K2, double iq, double& kf) {
  const double sb = fma(kS6, v.s0, fma(kH, v.s1, v.s2));
  const double qu = -fma(a.pi, r, sb);
  const double nqx0 = r + v.s0;
  const double nqx1 = r + (v.s0 + v.s1);
  const double nqx2 = fma(a.gam, r, fma(kH, v.s0, v.s1 + v.s2));
  kf = qu * iq;
  v.s0 = fma(K0, qu, nqx0);
  v.s1 = fma(K1, qu, nqx1);
  v.s2 = fma(K2, qu, nqx2);
}

struct Lane {
  const double2* hl;  // wave's staged (z_max, z_min) rows (uniform)
  int lane;
};

// Per-lane working-set flags of the wave's N slots in LDS (0 free, 1 at z_max, 2 at z_min):
// one byte per slot ([slot][64]), or, in the prefetching kernel (PK), two slots per byte
// ([slot/2][64], low nibble = even slot) so that the segment buffers fit beside them.
template <bool PK>
struct Flags {
  unsigned char* p;
  __device__ __forceinline__ int get(int k, int lane) const {
    if constexpr (PK)
      return (p[(k >> 1) * 64 + lane] >> ((k & 1) << 2)) & 0xF;
    else
      return p[k * 64 + lane];
  }
  __device__ __forceinline__ void set(int k, int lane, int v) const {
    if constexpr (PK) {
      unsigned char* b = p + (k >> 1) * 64 + lane;
      const int sh = (k & 1) << 2;
      *b = (unsigned char)((*b & ~(0xF << sh)) | (v << sh));
    } else {
      p[k * 64 + lane] = (unsigned char)v;
    }
  }
};

// Segment prefetch through LDS (PK): the next segment's staged bound rows (S × 1 KiB) and
// checkpoint (9 × 512 B, copied as five 1-KiB pieces) go global → LDS with LDS-DMA
// (global_load_lds_dwordx4: lane-linear, no VGPR destination) while the current segment
// computes; at 256 VGPRs (two waves per SIMD) nothing else hides the load latency, and a
// register prefetch spills.
template <int S>
__device__ __forceinline__ void glds_rows(const LqArgs& a, int j, const Lane& L, int64_t i,
                                          double2* rbuf) {
  const int64_t row0 = i + a.toff + (int64_t)j * S;
  const double2* hp = L.hl + row0 * 64 + L.lane;
#pragma unroll
  for (int q = 0; q < S; ++q)
    __builtin_amdgcn_global_load_lds((const void*)(hp + q * 64), (void*)(rbuf + q * 64), 16, 0,
                                     0);
}

// Pieces [c0, c1) of segment j's checkpoint in the paired layout (ck_store<PK>): piece c is the
// [64] (double2) array of component pairs c — (p00, p01), (p02, p11), (p12, p22), (s0, s1),
// (s2, –) — so each lane copies only its own 16 bytes (lanes outside the pass, masked off, then
// miss nothing another lane needs).
__device__ __forceinline__ void glds_ck(const double* ck, int j, int lane, double2* cbuf,
                                        int c0, int c1) {
  const double2* src = reinterpret_cast<const double2*>(ck + (size_t)j * 10 * 64) + lane;
  for (int c = c0; c < c1; ++c)
    __builtin_amdgcn_global_load_lds((const void*)(src + c * 64), (void*)(cbuf + c * 64), 16, 0,
                                     0);
}

// s_waitcnt vmcnt(0) / lgkmcnt(0) (gfx9 encoding: vmcnt [3:0]+[15:14], expcnt [6:4],
// lgkmcnt [11:8])
__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }

// Issue the loads of segment j's slots (bounds, and the flags when FLAGS).  Slots past N read
// padded rows (loaded, never used) so the loads carry no guards.
template <int S, bool FLAGS, class FL>
__device__ __forceinline__ void seg_load(const LqArgs& a, int j, const Lane& L, int64_t i,
                                         const FL& fl, SegIn<S>& in) {
  // segment's first row (the lane's own timestep); its S rows are 1 KiB apart: one address,
  // immediate offsets
  const int64_t row0 = i + a.toff + (int64_t)j * S;
  const double2* hp = L.hl + row0 * 64;
#pragma unroll
  for (int q = 0; q < S; ++q) {
    const double2 v = hp[q * 64 + L.lane];
    in.hi[q] = v.x;
    in.lo[q] = v.y;
    if (FLAGS) in.f[q] = fl.get(j * S + q, L.lane);
  }
}

// The same from the segment prefetched into LDS (rbuf: [S][64] pairs).
template <int S, bool FLAGS, class FL>
__device__ __forceinline__ void seg_load_lds(int j, const Lane& L, const double2* rbuf,
                                             const FL& fl, SegIn<S>& in) {
#pragma unroll
  for (int q = 0; q < S; ++q) {
    const double2 v = rbuf[q * 64 + L.lane];
    in.hi[q] = v.x;
    in.lo[q] = v.y;
    if (FLAGS) in.f[q] = fl.get(j * S + q, L.lane);
  }
}

// No lane taking part has an active slot in the segment (wave-uniform).
template <int S>
__device__ __forceinline__ bool seg_free(const SegIn<S>& in) {
  int any = 0;
#pragma unroll
  for (int q = 0; q < S; ++q) any |= in.f[q];
  return !__any(any != 0);
}

// Riccati steps of segment j (slots jS + S−1 down to jS).  KEEP: feedback kept in g (sweep
// B) or dropped (sweep A).  FULL: every slot of the segment is < N (straight-line code).
// FREE: no lane has an active slot here.
template <int S, bool FULL, bool KEEP, bool FREE>
__device__ __forceinline__ void seg_riccati(const LqArgs& a, int j, Ric& v, const SegIn<S>& in,
                                            SegOut<S>& g) {
#pragma unroll
  for (int q = S - 1; q >= 0; --q) {
    const int k = j * S + q;
    if (FULL || k < a.N) {
      double K0, K1, K2, kf;
      if (FREE) {
        double iq;
        ric_free(a, v, (in.hi[q] + in.lo[q]) / 2, K0, K1, K2, kf, iq);
      } else {
        ric_step<!KEEP>(a, v, in.hi[q], in.lo[q], in.f[q], K0, K1, K2, kf);
      }
      if (KEEP) {
        g.K0[q] = K0;
        g.K1[q] = K1;
        g.K2[q] = K2;
        g.kf[q] = kf;
      }
    }
    // keep each step's work inside the step: hoisting the load-dependent parts of all S
    // steps ahead of the recursion buys nothing (the chain is serial) and costs registers
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Free-tail steps of segment j: the s recursion with the table's K and 1/Quu (kff kept in g
// when KEEP).
template <int S, bool FULL, bool KEEP>
__device__ __forceinline__ void seg_tail(const LqArgs& a, const double* __restrict__ tab, int j,
                                         Ric& v, const SegIn<S>& in, SegOut<S>& g) {
#pragma unroll
  for (int q = S - 1; q >= 0; --q) {
    const int k = j * S + q;
    if (FULL || k < a.N) {
      const double* t = tab + (size_t)k * TAB;
      double kf;
      ric_tail(a, v, (in.hi[q] + in.lo[q]) / 2, t[0], t[1], t[2], t[3], kf);
      if (KEEP) g.kf[q] = kf;
    }
  }
}

// Forward through segment j: roll the trajectory out (x advances to the segment's end),
// primal check of the free slots, and the per-step input of the costate sweep.
template <int S, bool FULL>
__device__ __forceinline__ void seg_forward(const LqArgs& a, int j, const SegIn<S>& in,
                                            SegOut<S>& g, double* x, double& u0) {
  const double tol = 1e-13;  // as strict.hip (tolz)
#pragma unroll
  for (int q = 0; q < S; ++q) {
    const int k = j * S + q;
    if (FULL || k < a.N) {
      const double u = -fma(g.K0[q], x[0], fma(g.K1[q], x[1], g.K2[q] * x[2])) - g.kf[q];
      if (k == 0) u0 = u;
      const double z = fma(a.pi, u, fma(a.gam, x[2], x[0] + x[1]));
      const double y0 = fma(kS6, u, fma(kH, x[2], x[0] + x[1]));
      const double y1 = fma(kH, u, x[1] + x[2]);
      const double y2 = x[2] + u;
      x[0] = y0;
      x[1] = y1;
      x[2] = y2;
      const double hi = in.hi[q], lo = in.lo[q];
      const double r = (hi + lo) / 2;
      g.w[q] = (in.f[q] == 0) ? z - r : u;
      g.nf[q] = (z > hi + tol) ? 1 : ((z < lo - tol) ? 2 : 0);
    }
  }
}

// Forward through a free-tail segment (table K, kff from seg_tail): primal check and the new
// flags (every slot here is free for every lane taking part, so no costate is needed).
template <int S, bool FULL, class FL>
__device__ __forceinline__ void seg_forward_tail(const LqArgs& a, const double* __restrict__ tab,
                                                 int j, const SegIn<S>& in, const SegOut<S>& g,
                                                 double* x, double& u0, bool& changed, int& kl,
                                                 const FL& fl, int lane) {
  const double tol = 1e-13;
#pragma unroll
  for (int q = 0; q < S; ++q) {
    const int k = j * S + q;
    if (FULL || k < a.N) {
      const double* t = tab + (size_t)k * TAB;
      const double u = -fma(t[0], x[0], fma(t[1], x[1], t[2] * x[2])) - g.kf[q];
      if (k == 0) u0 = u;
      const double z = fma(a.pi, u, fma(a.gam, x[2], x[0] + x[1]));
      const double y0 = fma(kS6, u, fma(kH, x[2], x[0] + x[1]));
      const double y1 = fma(kH, u, x[1] + x[2]);
      const double y2 = x[2] + u;
      x[0] = y0;
      x[1] = y1;
      x[2] = y2;
      const int nf = (z > in.hi[q] + tol) ? 1 : ((z < in.lo[q] - tol) ? 2 : 0);
      fl.set(k, lane, nf);
      changed |= nf != 0;
      kl = nf ? k : kl;
    }
  }
}

// Costate sweep back through segment j from λ at its end (λ_k = ∇V_k(x_k) = c1 e_k + Aᵀλ_{k+1},
// e_k = Q (z_k − r_k) + ν_k): the bound multipliers ν_k of the active slots, dual check, the
// slot's new flag; kl = the last slot active in the new set.
template <int S, bool FULL, class FL>
__device__ __forceinline__ void seg_costate(const LqArgs& a, int j, const SegIn<S>& in,
                                            const SegOut<S>& g, double* lam, bool& changed,
                                            int& kl, const FL& fl, int lane) {
#pragma unroll
  for (int q = S - 1; q >= 0; --q) {
    const int k = j * S + q;
    if (FULL || k < a.N) {
      const int f = in.f[q];
      const double hi = in.hi[q], lo = in.lo[q];
      const double bl = fma(kS6, lam[0], fma(kH, lam[1], lam[2]));  // B̂ᵀλ_{k+1}
      // active: π e + ρ v + B̂ᵀλ_{k+1} = 0 (stationarity in v_k)
      const double e = (f == 0) ? g.w[q] : -fma(a.rho, g.w[q], bl) * a.ipi;
      {
        const double r = (hi + lo) / 2;
        const double t = (f == 1) ? hi : lo;
        const double nu = e - (t - r);  // ν / Q (meaningful at active slots only)
        const bool rel = (f == 1 && nu < -a.tolnu) || (f == 2 && nu > a.tolnu);
        // the slot's new flag, written unconditionally (branch-free)
        const int nf = (f == 0) ? g.nf[q] : (rel ? 0 : f);
        fl.set(k, lane, nf);
        changed |= nf != f;
        kl = (nf != 0 && k > kl) ? k : kl;
      }
      const double l0 = lam[0], l1 = lam[1], l2 = lam[2];
      lam[0] = e + l0;
      lam[1] = e + (l0 + l1);
      lam[2] = fma(a.gam, e, fma(kH, l0, l1 + l2));
    }
  }
}

// Sweep B through one working-set segment: Riccati from its checkpoint, forward, costate.
template <int S, bool FULL, class FL>
__device__ __forceinline__ void seg_sweep_b(const LqArgs& a, int j, Ric& v, const SegIn<S>& in,
                                            SegOut<S>& g, double* xs, double& u0, bool& changed,
                                            int& kl, const FL& fl, int lane) {
  const Ric ve = v;  // V at the segment's end
  seg_riccati<S, FULL, true, false>(a, j, v, in, g);
  seg_forward<S, FULL>(a, j, in, g, xs, u0);
  double lam[3];
  lam[0] = fma(ve.p00, xs[0], fma(ve.p01, xs[1], ve.p02 * xs[2])) - ve.s0;
  lam[1] = fma(ve.p01, xs[0], fma(ve.p11, xs[1], ve.p12 * xs[2])) - ve.s1;
  lam[2] = fma(ve.p02, xs[0], fma(ve.p12, xs[1], ve.p22 * xs[2])) - ve.s2;
  seg_costate<S, FULL>(a, j, in, g, lam, changed, kl, fl, lane);
}

// Checkpoints are written once and read once per pass.  With per-walk bounds (whose rows are
// re-read every timestep and do not fit the caches) they go non-temporal (NT), so they do not
// push those rows out; with a shared CoP the bounds are cache-resident anyway and the
// checkpoints are better off cached (config 3: 98.8 → 92.2 ms NT; config 4: 142 → 158 ms NT).
template <bool NT>
struct CkIO {
  __device__ __forceinline__ void st(double* p, double v) const {
    if constexpr (NT)
      __builtin_nontemporal_store(v, p);
    else
      *p = v;
  }
  __device__ __forceinline__ double ld(const double* p) const {
    if constexpr (NT)
      return __builtin_nontemporal_load(p);
    else
      return *p;
  }
  __device__ __forceinline__ void st2(double2* p, double x, double y) const {
    typedef double v2d __attribute__((ext_vector_type(2)));
    const v2d t = {x, y};
    if constexpr (NT)
      __builtin_nontemporal_store(t, reinterpret_cast<v2d*>(p));
    else
      *reinterpret_cast<v2d*>(p) = t;
  }
};

// Doubles of one segment's checkpoint per 64 lanes: [9][64], or paired [5][64] double2 (PK).
template <bool PK>
constexpr int ck_stride() { return PK ? 10 * 64 : 9 * 64; }

template <bool PK, bool NT>
__device__ __forceinline__ void ck_store(const CkIO<NT>& io, double* ck, int j, const Ric& v,
                                         int lane) {
  if constexpr (PK) {
    double2* p = reinterpret_cast<double2*>(ck + (size_t)j * ck_stride<PK>()) + lane;
    io.st2(p + 0, v.p00, v.p01);
    io.st2(p + 64, v.p02, v.p11);
    io.st2(p + 128, v.p12, v.p22);
    io.st2(p + 192, v.s0, v.s1);
    io.st2(p + 256, v.s2, 0.0);
    return;
  }
  double* p = ck + (size_t)j * ck_stride<PK>() + lane;
  io.st(p + 0, v.p00);
  io.st(p + 64, v.p01);
  io.st(p + 128, v.p02);
  io.st(p + 192, v.p11);
  io.st(p + 256, v.p12);
  io.st(p + 320, v.p22);
  io.st(p + 384, v.s0);
  io.st(p + 448, v.s1);
  io.st(p + 512, v.s2);
}

template <bool PK, bool NT>
__device__ __forceinline__ void ck_store_s(const CkIO<NT>& io, double* ck, int j, const Ric& v,
                                           int lane) {
  if constexpr (PK) {
    double2* p = reinterpret_cast<double2*>(ck + (size_t)j * ck_stride<PK>()) + lane;
    io.st2(p + 192, v.s0, v.s1);
    io.st2(p + 256, v.s2, 0.0);
    return;
  }
  double* p = ck + (size_t)j * ck_stride<PK>() + lane;
  io.st(p + 384, v.s0);
  io.st(p + 448, v.s1);
  io.st(p + 512, v.s2);
}

template <bool NT>
__device__ __forceinline__ void ck_load(const CkIO<NT>& io, const double* ck, int j, Ric& v,
                                        int lane) {
  const double* p = ck + (size_t)j * 9 * 64 + lane;
  v.p00 = io.ld(p + 0);
  v.p01 = io.ld(p + 64);
  v.p02 = io.ld(p + 128);
  v.p11 = io.ld(p + 192);
  v.p12 = io.ld(p + 256);
  v.p22 = io.ld(p + 320);
  v.s0 = io.ld(p + 384);
  v.s1 = io.ld(p + 448);
  v.s2 = io.ld(p + 512);
}

template <bool NT>
__device__ __forceinline__ void ck_load_s(const CkIO<NT>& io, const double* ck, int j, Ric& v,
                                          int lane) {
  const double* p = ck + (size_t)j * 9 * 64 + lane;
  v.s0 = io.ld(p + 384);
  v.s1 = io.ld(p + 448);
  v.s2 = io.ld(p + 512);
}

// G waves per workgroup.  G = 8: waves 0..3 take the x axis and 4..7 the y axis of the same
// four 64-walk groups, so each SIMD (waves w and w + 4 under the round-robin placement) holds
// one wave of each axis — the y axis carries nearly all of the active-set work, and an
// axis-pure SIMD would idle once its x waves are done.  G = 4 (A/B): axis = wave parity.
// PK: segments prefetched through LDS (glds_rows / glds_ck), flags nibble-packed.
template <int S, int W, int G, bool NT = false, bool PK = false>
__global__ void __launch_bounds__(64 * G, W)
    zmpc_strict_lq_kernel(LqArgs a, const double* __restrict__ tab) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lq_smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * G + wave;
  const int N = a.N;
  // slot flags [NS·S][64] bytes, or [NS·S/2][64] packed (rows past N stay 0: the last
  // segment's loads are unguarded)
  const int fbytes = PK ? a.NS * S / 2 : a.NS * S;
  const Flags<PK> fl{lq_smem + (size_t)wave * fbytes * 64};
  double2* rbuf = nullptr;  // PK: next segment's bound rows [S][64]
  double2* cbuf = nullptr;  // PK: next segment's checkpoint, five 1-KiB pieces
  if constexpr (PK) {
    unsigned char* base = lq_smem + (size_t)G * fbytes * 64;
    rbuf = reinterpret_cast<double2*>(base) + (size_t)wave * (S + 5) * 64;
    cbuf = rbuf + S * 64;
  }
  double* ck = a.ck + (size_t)gw * a.NS * ck_stride<PK>();
  const CkIO<NT> io{};
  int axis;
  int64_t b0;
  if (a.window_mode) {
    axis = 0;
    b0 = gw * 64;
  } else if (G == 8) {
    axis = wave >> 2;
    b0 = ((int64_t)blockIdx.x * 4 + (wave & 3)) * 64;
  } else {
    axis = (int)(gw & 1);
    b0 = (gw >> 1) * 64;
  }
  // diagnostics: dbg bit 1 / bit 2 = the x / y waves of a rollout exit at once (the other
  // axis then has its SIMDs alone; A/B timing only, results of that axis unwritten)
  if (!a.window_mode && (((a.dbg & 2) && axis == 0) || ((a.dbg & 4) && axis == 1))) return;
  // lane position b0 + lane runs walk b (the kick order of order.hip, or the identity); the
  // staged bounds follow the positions, everything per walk (x0, kick, history, status) b
  const bool valid = b0 + lane < a.B;
  const int64_t b = (valid && a.perm) ? (int64_t)a.perm[b0 + lane] : b0 + lane;
  Lane L;
  L.lane = lane;
  {
    const int64_t g = (a.shared || (a.dbg & 1)) ? 0 : (b0 >> 6);
    const int64_t off = ((int64_t)axis * a.groups + g) * a.rows * 64;
    L.hl = a.hl + off;
  }
  const int jfull = N / S;  // segments [0, jfull) are full
  for (int k = 0; k < fbytes; ++k) fl.p[k * 64 + lane] = 0;

  double x[3] = {0.0, 0.0, 0.0};
  if (valid) {
    const double* xp = a.window_mode ? a.x0 + b * 3 : a.x0 + (b * 2 + axis) * 3;
    x[0] = xp[0];
    x[1] = xp[1];
    x[2] = xp[2];
    if (!a.window_mode) {
      double* h = a.out + ((b * a.n) * 2 + axis) * 3;  // hist[b, 0, axis, :] = x0
      h[0] = x[0];
      h[1] = x[1];
      h[2] = x[2];
    }
  }
  int fq = 0;
  unsigned long long n_wave_pass = 0, n_lane_pass = 0, n_ws_slots = 0;
  const int64_t kstep =
      (!a.window_mode && axis == 1 && a.kick != nullptr && valid)
          ? (a.kick_steps ? a.kick_steps[b] : a.kick_step)
          : -1;
  const double kv = (kstep >= 0) ? a.kick[b] : 0.0;

  // Each lane walks its own timestep i: a pass runs for every lane still inside its rollout
  // and at most `drift` timesteps ahead of the wave's slowest lane (so a slot's bound loads
  // stay within a few 512-byte rows); a lane whose working set repeated advances (state,
  // history, shifted warm start) while the others keep iterating.
  int64_t i = 0;
  bool active = valid && a.nsteps > 0;
  int it = 0;
  unsigned itmax = 0;  // most passes of one of this lane's solves (counter [8])
  int klast = -1;  // last active slot of this lane's working set (−1: none)
  while (__any(active)) {
    ++n_wave_pass;
    int imin = active ? (int)i : 0x7fffffff;
    for (int o = 32; o > 0; o >>= 1) imin = min(imin, __shfl_xor(imin, o));
    const bool part = active && i <= (int64_t)imin + a.drift;
    // segments [jt, NS) hold no active slot of any lane taking part: the free tail
    int kw = part ? klast : -1;
    for (int o = 32; o > 0; o >>= 1) kw = max(kw, __shfl_xor(kw, o));
    const int jt = __builtin_amdgcn_readfirstlane(kw < 0 ? 0 : kw / S + 1);
    if (part) {
      ++n_lane_pass;
      n_ws_slots += (unsigned)min(jt * S, N);
      double u0 = 0.0;
      bool changed = false;
      int kl = -1;
      {
        Ric v{0, 0, 0, 0, 0, 0, 0, 0, 0};
        SegIn<S> cur;
        SegOut<S> g;
        if constexpr (PK) glds_rows<S>(a, a.NS - 1, L, i, rbuf);
        // sweep A, free tail: the s recursion, checkpoints of s
#pragma unroll 1
        for (int j = a.NS - 1; j >= jt; --j) {
          if constexpr (PK) {
            wait_vm0();
            seg_load_lds<S, false>(j, L, rbuf, fl, cur);
            wait_lgkm0();
            if (j > 0) glds_rows<S>(a, j - 1, L, i, rbuf);
          } else {
            seg_load<S, false>(a, j, L, i, fl, cur);
          }
          ck_store_s<PK>(io, ck, j, v, lane);
          if (j < jfull)
            seg_tail<S, true, false>(a, tab, j, v, cur, g);
          else
            seg_tail<S, false, false>(a, tab, j, v, cur, g);
        }
        if (jt < a.NS) {  // V at the tail's first slot: P from the table
          const double* t = tab + (size_t)jt * S * TAB;
          v.p00 = t[4];
          v.p01 = t[5];
          v.p02 = t[6];
          v.p11 = t[7];
          v.p12 = t[8];
          v.p22 = t[9];
        }
        // sweep A, working-set segments: full Riccati, checkpoints of (P, s)
#pragma unroll 1
        for (int j = jt - 1; j >= 0; --j) {
          if constexpr (PK) {
            wait_vm0();
            seg_load_lds<S, true>(j, L, rbuf, fl, cur);
            wait_lgkm0();
            if (j > 0) glds_rows<S>(a, j - 1, L, i, rbuf);
          } else {
            seg_load<S, true>(a, j, L, i, fl, cur);
          }
          ck_store<PK>(io, ck, j, v, lane);
          const bool fr = seg_free(cur);
          if (j < jfull) {
            if (fr)
              seg_riccati<S, true, false, true>(a, j, v, cur, g);
            else
              seg_riccati<S, true, false, false>(a, j, v, cur, g);
          } else {
            if (fr)
              seg_riccati<S, false, false, true>(a, j, v, cur, g);
            else
              seg_riccati<S, false, false, false>(a, j, v, cur, g);
          }
        }
        // sweep B: per segment from the front — recompute its steps from the checkpoint,
        // forward, then (working-set segments) the costate back through it
        double xs[3] = {x[0], a.T * x[1], a.Tsq * x[2]};  // ξ
        if constexpr (PK) {
          wait_vm0();  // sweep A's checkpoint stores have landed before they are read back
          glds_rows<S>(a, 0, L, i, rbuf);
          if (jt > 0)
            glds_ck(ck, 0, lane, cbuf, 0, 5);
          else
            glds_ck(ck, 0, lane, cbuf, 3, 5);
        }
#pragma unroll 1
        for (int j = 0; j < jt; ++j) {
          if constexpr (PK) {
            wait_vm0();
            seg_load_lds<S, true>(j, L, rbuf, fl, cur);
            const double2* cb = cbuf + lane;
            const double2 c0 = cb[0], c1 = cb[64], c2 = cb[128], c3 = cb[192], c4 = cb[256];
            v.p00 = c0.x;
            v.p01 = c0.y;
            v.p02 = c1.x;
            v.p11 = c1.y;
            v.p12 = c2.x;
            v.p22 = c2.y;
            v.s0 = c3.x;
            v.s1 = c3.y;
            v.s2 = c4.x;
            wait_lgkm0();
            if (j + 1 < a.NS) {
              glds_rows<S>(a, j + 1, L, i, rbuf);
              if (j + 1 < jt)
                glds_ck(ck, j + 1, lane, cbuf, 0, 5);
              else
                glds_ck(ck, j + 1, lane, cbuf, 3, 5);
            }
          } else {
            seg_load<S, true>(a, j, L, i, fl, cur);
            ck_load(io, ck, j, v, lane);
          }
          // (a free form here, as in sweep A, costs more registers than it saves)
          if (j < jfull)
            seg_sweep_b<S, true>(a, j, v, cur, g, xs, u0, changed, kl, fl, lane);
          else
            seg_sweep_b<S, false>(a, j, v, cur, g, xs, u0, changed, kl, fl, lane);
        }
#pragma unroll 1
        for (int j = jt; j < a.NS; ++j) {
          if constexpr (PK) {
            wait_vm0();
            seg_load_lds<S, false>(j, L, rbuf, fl, cur);
            const double2* cb = cbuf + lane;
            const double2 c3 = cb[192], c4 = cb[256];
            v.s0 = c3.x;
            v.s1 = c3.y;
            v.s2 = c4.x;
            wait_lgkm0();
            if (j + 1 < a.NS) {
              glds_rows<S>(a, j + 1, L, i, rbuf);
              glds_ck(ck, j + 1, lane, cbuf, 3, 5);
            }
          } else {
            seg_load<S, false>(a, j, L, i, fl, cur);
            ck_load_s(io, ck, j, v, lane);
          }
          if (j < jfull) {
            seg_tail<S, true, true>(a, tab, j, v, cur, g);
            seg_forward_tail<S, true>(a, tab, j, cur, g, xs, u0, changed, kl, fl, lane);
          } else {
            seg_tail<S, false, true>(a, tab, j, v, cur, g);
            seg_forward_tail<S, false>(a, tab, j, cur, g, xs, u0, changed, kl, fl, lane);
          }
        }
      }
      ++it;
      if (changed && it >= LQ_MAXIT) {
        fq |= ZMPC_ST_MAXITER;
        changed = false;
      }
      if (!changed) {
        itmax = max(itmax, (unsigned)it);
        // converged: advance in the reference form x⁺ = A x + B u0 (zmp_controller.py:199)
        u0 = u0 / a.Tcu;  // v0 = T³ u0
        double xn[3];
        xn[0] = x[0] + a.T * x[1] + a.T2 * x[2] + a.T3 * u0;
        xn[1] = x[1] + a.T * x[2] + a.T2 * u0;
        xn[2] = x[2] + a.T * u0;
        if (i == kstep) xn[1] -= kv;  // force kick (zmp_controller.py:90,105-106)
        if (!(isfinite(xn[0]) && isfinite(xn[1]) && isfinite(xn[2]))) fq |= ZMPC_ST_NONFINITE;
        x[0] = xn[0];
        x[1] = xn[1];
        x[2] = xn[2];
        double* h = a.window_mode ? a.out + b * 3 : a.out + ((b * a.n + i + 1) * 2 + axis) * 3;
        h[0] = xn[0];
        h[1] = xn[1];
        h[2] = xn[2];
        ++i;
        it = 0;
        if (i < a.nsteps) {
          // warm start: the converged set shifted one slot towards the present (slot N−1
          // kept), this lane's column only
          if constexpr (PK) {
            // nibble pairs: new byte q = (slot 2q+1, slot 2q+2) of the old set
            const int nb = (N - 1) >> 1;  // bytes fully below slot N−1
#pragma unroll 4
            for (int q = 0; q < nb; ++q) {
              unsigned char* p0 = fl.p + q * 64 + lane;
              *p0 = (unsigned char)((*p0 >> 4) | ((p0[64] & 0xF) << 4));
            }
            if ((N - 1) & 1) {  // slot N−2 (low nibble of byte nb) takes slot N−1
              unsigned char* p0 = fl.p + nb * 64 + lane;
              *p0 = (unsigned char)((*p0 & 0xF0) | (*p0 >> 4));
            }
          } else {
#pragma unroll 8
            for (int k = 0; k < N - 1; ++k) fl.p[k * 64 + lane] = fl.p[(k + 1) * 64 + lane];
          }
          // the previous solve's terminal slot is no longer terminal: it starts free (its end
          // effect pinned it more often than the next solve keeps it; a CPU simulation of this
          // iteration on the default walk's y axis at F_ext 0/400/800 N: 1.387 → 1.310 passes
          // per solve).  Slot N−1 keeps the copy.  The converged set, hence the solution, is
          // the same; only the passes to reach it change.
          if (a.warm_free_term && N >= 2) fl.set(N - 2, lane, 0);
          klast = (kl >= N - 1) ? N - 1 : max(kl - 1, -1);
        } else {
          active = false;
        }
      } else {
        klast = kl;
      }
    }
  }
  if (valid && a.status != nullptr) {
    if (a.window_mode)
      a.status[b] = fq;
    else if (fq != 0)
      atomicOr(&a.status[b], fq);
  }
  if (a.cnt) {
    for (int o = 32; o > 0; o >>= 1) {
      n_lane_pass += __shfl_xor(n_lane_pass, o);
      n_ws_slots += __shfl_xor(n_ws_slots, o);
      itmax = max(itmax, (unsigned)__shfl_xor((int)itmax, o));
    }
    if (lane == 0) {
      atomicAdd(a.cnt + 0, n_wave_pass);
      atomicAdd(a.cnt + 1, n_lane_pass);
      atomicAdd(a.cnt + 2, n_ws_slots);
      if (gw == 0) atomicAdd(a.cnt + 3, 1ull);
      atomicMax(a.cnt + 8, (unsigned long long)itmax);
    }
  }
}

// The free-tail table of a plan: the Riccati recursion with every slot free, from V_N = 0
// (ric_free, the arithmetic of the kernel's free steps; the bounds do not enter P, K, 1/Quu).
__global__ void zmpc_strict_lq_table_kernel(LqArgs a, double* tab) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Ric v{0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = a.N - 1; k >= 0; --k) {
    double K0, K1, K2, kf, iq;
    ric_free(a, v, 0.0, K0, K1, K2, kf, iq);
    double* t = tab + (size_t)k * TAB;
    t[0] = K0;
    t[1] = K1;
    t[2] = K2;
    t[3] = iq;
    t[4] = v.p00;
    t[5] = v.p01;
    t[6] = v.p02;
    t[7] = v.p11;
    t[8] = v.p12;
    t[9] = v.p22;
    for (int c = 10; c < TAB; ++c) t[c] = 0.0;
  }
}

// Stage bounds into the kernel's tiled layout: source elements (b, t, axis) at
// b·sb + min(t, nsrc − 1)·st + axis·sa of z_max and z_min → dst[((axis·G + b/64)·rows + t)·64
// + b%64] = (z_max, z_min) for t < rows.  64 walks × 16 rows per workgroup through LDS;
// consecutive threads read consecutive source elements for the walk-contiguous [B, n, 2]
// layout and write consecutive destination pairs.
struct StageArgs {
  const double* hi;
  const double* lo;
  int64_t sb, st, sa, nsrc;
  int64_t B, G, rows;
  int naxes;
  const int32_t* perm;  // destination position p takes walk perm[p] (null: p)
  double2* dst;
};

__global__ void __launch_bounds__(256) zmpc_bounds_stage_kernel(StageArgs s) {
  __shared__ double2 tile[2][16][65];
  const int64_t t0 = (int64_t)blockIdx.x * 16;
  const int64_t b0 = (int64_t)blockIdx.y * 64;
  const int per_walk = 16 * s.naxes;
  for (int idx = threadIdx.x; idx < 64 * per_walk; idx += 256) {
    const int w = idx / per_walk, rem = idx - w * per_walk;
    const int tt = rem / s.naxes, ax = rem - tt * s.naxes;
    int64_t b = b0 + w;
    int64_t t = t0 + tt;
    if (t > s.nsrc - 1) t = s.nsrc - 1;  // window padding (zmp_controller.py:81-88)
    double2 v = make_double2(0.0, 0.0);
    if (b < s.B) {
      if (s.perm) b = s.perm[b];
      const int64_t e = b * s.sb + t * s.st + ax * s.sa;
      v = make_double2(s.hi[e], s.lo[e]);
    }
    tile[ax][tt][w] = v;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 64 * per_walk; idx += 256) {
    const int l = idx & 63, r = idx >> 6;
    const int ax = r / 16, tt = r - ax * 16;
    const int64_t t = t0 + tt;
    if (t < s.rows)
      s.dst[((ax * s.G + (b0 >> 6)) * s.rows + t) * 64 + l] = tile[ax][tt][l];
  }
}

hipError_t stage(const double* hi, const double* lo, int64_t sb, int64_t st, int64_t sa,
                 int64_t nsrc, int64_t B, int64_t rows, int naxes, double2* dst, hipStream_t s,
                 const int32_t* perm = nullptr) {
  StageArgs g{hi, lo, sb, st, sa, nsrc, B, (B + 63) / 64, rows, naxes, perm, dst};
  const dim3 grid((unsigned)((rows + 15) / 16), (unsigned)g.G);
  hipLaunchKernelGGL(zmpc_bounds_stage_kernel, grid, dim3(256), 0, s, g);
  return hipGetLastError();
}

// Kernel variant: Riccati steps per segment S × waves per SIMD W × waves per workgroup G, and
// PK = segment prefetch through LDS (ZMPC_STRICT_LQ="SxWxG" or "SxWxGp", A/B only; default
// below).
struct LqVariant {
  int S, W, G;
  bool pk;
  void (*kernel)(LqArgs, const double*);     // checkpoints cached (shared CoP, window mode)
  void (*kernel_nt)(LqArgs, const double*);  // checkpoints non-temporal (per-walk bounds)
};

#define ZMPC_LQV(S, W, G, PK)                                                             \
  {S, W, G, PK, zmpc_strict_lq_kernel<S, W, G, false, PK>,                                 \
   zmpc_strict_lq_kernel<S, W, G, true, PK>}
const LqVariant kLqVariants[] = {
    ZMPC_LQV(8, 2, 8, false),  // default
    ZMPC_LQV(8, 2, 4, false),  // N up to 640 (slot flags of 4 waves in LDS)
    ZMPC_LQV(8, 2, 2, false),  // N up to 1280
    ZMPC_LQV(8, 2, 1, false),  // N up to 2560
    ZMPC_LQV(8, 2, 8, true),   // segment prefetch through LDS
    ZMPC_LQV(8, 2, 4, true),
    ZMPC_LQV(6, 2, 8, false),
    ZMPC_LQV(8, 1, 8, false),
    ZMPC_LQV(4, 3, 4, false),  // A/B: 3 waves per SIMD (≤ 168 VGPRs), 4-wave workgroups
};
#undef ZMPC_LQV
constexpr size_t kLdsCap = 160 * 1024;

// LDS of one workgroup: the G waves' slot flags (+ PK: their segment buffers).
size_t lq_lds_bytes(const LqVariant& v, int N) {
  const size_t rows = (size_t)(N + v.S - 1) / v.S * v.S;
  const size_t per_wave = v.pk ? rows / 2 * 64 + (size_t)(v.S + 5) * 64 * 16 : rows * 64;
  return (size_t)v.G * per_wave;
}

LqVariant lq_variant() {
  static LqVariant v = [] {
    LqVariant d = kLqVariants[0];
    const char* e = getenv("ZMPC_STRICT_LQ");
    if (e) {
      int s = 0, w = 0, g = 8;  // "SxW", "SxWxG" or "SxWxGp"
      const int got = sscanf(e, "%dx%dx%d", &s, &w, &g);
      const bool pk = strchr(e, 'p') != nullptr;
      if (got >= 2)
        for (const LqVariant& c : kLqVariants)
          if (c.S == s && c.W == w && c.G == g && c.pk == pk) d = c;
    }
    return d;
  }();
  return v;
}

// The configured variant, or — when its LDS (G waves' slot flags, + PK buffers) does not fit a
// CU — the same S, W (and PK, then without it) with the largest G that fits (N ≤ 2560 at G = 1).
LqVariant lq_variant_for(int N) {
  const LqVariant v = lq_variant();
  if (lq_lds_bytes(v, N) <= kLdsCap) return v;
  for (bool pk : {v.pk, false})
    for (int g = v.G; g >= 1; g /= 2)
      for (const LqVariant& c : kLqVariants)
        if (c.S == v.S && c.W == v.W && c.G == g && c.pk == pk && lq_lds_bytes(c, N) <= kLdsCap)
          return c;
  return LqVariant{v.S, v.W, 0, false, nullptr, nullptr};
}

void fill_consts(const zmpc_plan* p, LqArgs& a) {
  const int S = lq_variant().S;
  a.N = p->N;
  a.NS = (p->N + S - 1) / S;
  a.T = p->T;
  a.T2 = p->T2_2;
  a.T3 = p->T3_6;
  a.Tsq = p->T * p->T;
  a.Tcu = a.Tsq * p->T;
  const double hgt = p->hg / a.Tsq;
  a.gam = 0.5 - hgt;
  a.pi = 1.0 / 6.0 - hgt;  // p(0)/T³ (zmp_controller.py:171, i = j)
  a.ipi = 1.0 / a.pi;
  a.rho = p->R / (p->Q * a.Tcu * a.Tcu);
  a.quu0 = a.pi * a.pi + a.rho;
  a.gipi = a.gam / a.pi;
  a.gam2 = a.gam * a.gam;
  a.pig = a.pi * a.gam;
  a.tolnu = 1e-13 / p->Q;
  static const int drift = [] {
    // A/B only; round 3 (profiles/r3u/): 0 → 104.5 ms, 1 → 94.8, 2 → 92.5, 3 → 91.1,
    // 4 → 90.9, 8 → 92.7 at config 3 (config 4: 2 → 143.1, 4 → 140.8 ms)
    const char* e = getenv("ZMPC_STRICT_LQ_DRIFT");
    return e ? atoi(e) : 4;
  }();
  a.drift = drift;
  static const int warm = [] {
    // warm start of the shifted slot N−2 (the old terminal slot): 1 = free (default), 0 = kept
    // as the shift leaves it (A/B)
    const char* e = getenv("ZMPC_STRICT_WARM");
    return e ? atoi(e) : 1;
  }();
  a.warm_free_term = warm;
  a.cnt = p->lqcnt;
  static const int dbg = [] {
    const char* e = getenv("ZMPC_DEBUG_LQ");
    return e ? atoi(e) : 0;
  }();
  a.dbg = dbg;
}

hipError_t launch_lq(const zmpc_plan* p, LqArgs& a, int64_t waves, hipStream_t s) {
  static const bool dbg_on = getenv("ZMPC_DEBUG_STRICT") != nullptr;  // diagnostics only
  const LqVariant var = lq_variant_for(p->N);
  const int64_t blocks = (waves + var.G - 1) / var.G;
  const size_t lds = lq_lds_bytes(var, p->N);
  // rollouts over per-walk bounds: non-temporal checkpoints (see CkIO)
  static const int nt_env = [] {  // A/B only: 0 / 1 force cached / non-temporal checkpoints
    const char* e = getenv("ZMPC_STRICT_NT");
    return e ? atoi(e) : -1;
  }();
  const bool nt = nt_env >= 0 ? nt_env == 1 : (!a.window_mode && !a.shared);
  hipLaunchKernelGGL(nt ? var.kernel_nt : var.kernel, dim3((unsigned)blocks), dim3(64 * var.G),
                     lds, s, a, (const double*)p->lqtab);
  hipError_t e = hipGetLastError();
  if (dbg_on && a.cnt && e == hipSuccess) {
    unsigned long long h[4];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h, a.cnt, sizeof(h), hipMemcpyDeviceToHost);
    fprintf(stderr,
            "[zmpc strict-lq dbg] waves=%lld cumulative: launches=%llu wave_passes=%llu "
            "lane_passes=%llu ws_slots=%llu\n",
            (long long)waves, h[3], h[0], h[1], h[2]);
  }
  return e;
}

}  // namespace

hipError_t zmpc_strict_lq_set_attrs() {
  hipError_t e = hipSuccess;
  for (const LqVariant& c : kLqVariants)
    for (auto k : {c.kernel, c.kernel_nt})
      if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
  return e;
}

bool zmpc_strict_lq_supported(const zmpc_plan* p) {
  return p->N >= 1 && p->N <= ZMPC_STRICT_MAX_N && p->lqtab != nullptr &&
         lq_variant_for(p->N).kernel != nullptr;
}

size_t zmpc_strict_lq_table_doubles(int N) { return (size_t)N * TAB; }

hipError_t zmpc_strict_lq_build_table(zmpc_plan* p, hipStream_t s) {
  LqArgs a{};
  fill_consts(p, a);
  hipLaunchKernelGGL(zmpc_strict_lq_table_kernel, dim3(1), dim3(64), 0, s, a, p->lqtab);
  return hipGetLastError();
}

hipError_t zmpc_launch_rollout_strict_lq(const zmpc_plan* p, int64_t B, int64_t n,
                                         const double* zmax, const double* zmin,
                                         int64_t bstride, const double* x0, const double* kick,
                                         int64_t kick_step, const int64_t* kick_steps,
                                         double* hist, int32_t* status, hipStream_t s,
                                         std::string* why) {
  LqArgs a{};
  fill_consts(p, a);
  a.window_mode = 0;
  a.toff = 1;
  a.n = n;
  a.nsteps = n - 1;
  a.B = B;
  a.x0 = x0;
  a.kick = kick;
  a.kick_step = kick_step;
  a.kick_steps = kick_steps;
  a.out = hist;
  a.status = status;
  hipError_t e = hipSuccess;
  if (status && (e = hipMemsetAsync(status, 0, sizeof(int32_t) * B, s)) != hipSuccess) return e;
  const int64_t waves = 2 * ((B + 63) / 64);
  // workspace: checkpoints + the staged bounds (rows past n − 1: the padded windows)
  a.shared = bstride == 0 ? 1 : 0;
  const int64_t Bst = a.shared ? 64 : B;  // a shared CoP is staged once, 64 identical lanes
  a.groups = (Bst + 63) / 64;
  a.rows = n + (int64_t)a.NS * lq_variant().S;  // the last segment reads up to NS·S − 1 ahead
  const int64_t G = lq_variant_for(p->N).G;  // checkpoints for every wave of the launched blocks
  const size_t ck_doubles = (size_t)((waves + G - 1) / G * G) * a.NS * 10 * 64;  // ≥ either layout
  const size_t st_doubles = (size_t)2 * a.groups * a.rows * 64 * 2;  // 2 axes, (hi, lo)
  // kick order (order.hip): walks with per-walk kicks sorted by (kick step, kick) onto lanes,
  // when there is more than one wave of them (ZMPC_STRICT_ORDER=0 keeps the input order; A/B)
  static const bool order_on = [] {
    const char* e = getenv("ZMPC_STRICT_ORDER");
    return !(e && atoi(e) == 0);
  }();
  const bool ordered = order_on && kick != nullptr && B > 64;
  const size_t perm_doubles = ordered ? ((size_t)B * 4 + 7) / 8 : 0;
  const size_t ord_doubles = ordered ? (zmpc_kick_order_bytes(B) + 7) / 8 : 0;
  double* ws = nullptr;
  if (hipMallocAsync((void**)&ws,
                     (ck_doubles + st_doubles + perm_doubles + ord_doubles) * sizeof(double),
                     s) != hipSuccess) {
    (void)hipGetLastError();
    return hipErrorOutOfMemory;  // ZMPC_ENOMEM at the C-ABI
  }
  a.ck = ws;
  double2* hl = reinterpret_cast<double2*>(ws + ck_doubles);
  a.perm = nullptr;
  if (ordered) {
    int32_t* perm = reinterpret_cast<int32_t*>(ws + ck_doubles + st_doubles);
    e = zmpc_kick_order(kick, kick_steps, kick_step, B, perm,
                        ws + ck_doubles + st_doubles + perm_doubles, s);
    a.perm = perm;
  }
  if (e == hipSuccess)
    e = stage(zmax, zmin, bstride, 2, 1, n, Bst, a.rows, 2, hl, s, a.shared ? nullptr : a.perm);
  a.hl = hl;
  if (e == hipSuccess) e = launch_lq(p, a, waves, s);
  hipError_t ef = hipFreeAsync(ws, s);
  return e != hipSuccess ? e : ef;
}

hipError_t zmpc_launch_step_strict_lq(const zmpc_plan* p, int64_t B, const double* x,
                                      const double* zmax_win, const double* zmin_win,
                                      double* x_next, int32_t* status, hipStream_t s,
                                      std::string* why) {
  LqArgs a{};
  fill_consts(p, a);
  a.window_mode = 1;
  a.toff = 0;
  a.n = p->N;
  a.nsteps = 1;
  a.B = B;
  a.x0 = x;
  a.kick = nullptr;
  a.kick_step = -1;
  a.out = x_next;
  a.status = status;
  a.shared = 0;
  a.groups = (B + 63) / 64;
  a.rows = (int64_t)a.NS * lq_variant().S;
  const int64_t waves = (B + 63) / 64;
  const int64_t G = lq_variant_for(p->N).G;  // checkpoints for every wave of the launched blocks
  const size_t ck_doubles = (size_t)((waves + G - 1) / G * G) * a.NS * 10 * 64;  // ≥ either layout
  const size_t st_doubles = (size_t)a.groups * a.rows * 64 * 2;  // (hi, lo)
  double* ws = nullptr;
  if (hipMallocAsync((void**)&ws, (ck_doubles + st_doubles) * sizeof(double), s) != hipSuccess) {
    (void)hipGetLastError();
    return hipErrorOutOfMemory;  // ZMPC_ENOMEM at the C-ABI
  }
  hipError_t e = hipSuccess;
  a.ck = ws;
  double2* hl = reinterpret_cast<double2*>(ws + ck_doubles);
  e = stage(zmax_win, zmin_win, p->N, 1, 0, p->N, B, a.rows, 1, hl, s);
  a.hl = hl;
  if (e == hipSuccess) e = launch_lq(p, a, waves, s);
  hipError_t ef = hipFreeAsync(ws, s);
  return e != hipSuccess ? e : ef;
}
