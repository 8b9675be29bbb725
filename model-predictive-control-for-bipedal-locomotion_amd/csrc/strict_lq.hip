// Strict (ZMP box-constrained) Wieber QP, one instance per lane, solved in LQ form.
//
// Reference, per axis and timestep (zmp_controller.py:173-195, cvxpy→OSQP there):
//   min_J ½Q‖Px x + Pu J − z_ref‖² + ½R‖J‖²   s.t.  z_min ≤ Px x + Pu J ≤ z_max,  u0 = J[0]
// Pu[k,j] = C A^(k−j) B and Px[k] = C A^(k+1) (zmp_controller.py:162-171), so the predicted ZMP
// is the output of the LIPM itself.  The QP is a linear-quadratic tracking problem over the
// horizon with one output bound per slot.  For a working set (slot k pinned at t_k = z_max or
// z_min) the equality-constrained problem is solved exactly by a backward Riccati recursion: a
// free slot minimises over its input, a pinned slot's input is forced so that z_k = t_k.  The
// forward pass rolls the trajectory out (primal check of the free slots) and a costate sweep
// gives the pinned slots' bound multipliers (dual check).  The working set comes from the
// primal-dual active-set iteration — warm-started with the previous timestep's converged set
// shifted one slot, wrong-signed multipliers released, violated free slots added, stop when the
// set repeats — at O(N) per pass.
//
// Coordinates.  ξ = [x0, T x1, T² x2], v = T³ u, objective divided by Q, and then
//   η = [ξ0 − ξ2/6, ξ1 − ξ2/2, ξ2]:   η⁺ = Ā η + e2 v,   Ā = [[1,1,1],[0,1,1],[0,0,1]],
//   z = c̄ᵀη + π v,  c̄ = [1, 1, γ'],  γ' = 7/6 − (h/g)/T²,  π = 1/6 − (h/g)/T² (= p(0)/T³),
// stage cost ½(z − r)² + ½ρv², ρ = R/(Q T⁶).  The Riccati step takes the slot's ZMP z itself
// as the input (v = (z − c̄ᵀη)/π, strict_eta.h): a pinned slot is then z = t exactly (K = 0,
// kff = −t), and the value-function update has no cancellation at any weight (round 5: the
// v-input form lost three digits at R/Q = 1e-9).  Value function V(η) = ½ηᵀPη − sᵀη; a slot's
// law z = −K η − kff:
//   free:    K = Qux/Quu, kff = qu/Quu;  pinned at t: K = 0, kff = −t
//   P ← Qxx − Qux Kᵀ,  s ← Fᵀs + Qux kff,  F = Ā − e2 c̄ᵀ/π,
//   Qux = FᵀPe2/π − ε c̄,  Quu = 1 + ε + P22/π²,  qu = −(r + s2/π),  Qxx = ε c̄c̄ᵀ + FᵀPF,
// ε = ρ/π²; F's last two columns are equal and ĀᵀPĀ-style prefix sums give FᵀPF: ≈48 FP64
// operations for the branch-free working-set step (57 in the v-input form).
// oracle/strict_lq_cpu.c restates the same algorithm in C (the checker and the optimized CPU
// baseline).
//
// Mapping: a lane owns one instance (one walk, one axis) for the whole rollout; a wave holds
// 64 walks of one axis.  The bounds come in [axis][t][walk] (a staging transpose), so a wave's
// load of one window slot is 1 KiB contiguous ((z_ref, half-width) pairs, 16 B per lane).  Per pass:
//   sweep A  backward Riccati over the horizon in segments of S steps, checkpointing (P, s)
//            at segment boundaries to a per-lane global slab (coalesced [.., 9, 64]);
//   sweep B  per segment from the front: reload its checkpoint, recompute its S Riccati
//            steps into registers (K, kff, bounds, flags), roll forward through it, check
//            primal/dual feasibility, update the slot flags (LDS, [N][64] bytes).
//
// Free structure.  P (with K and 1/Quu) depends on the working set only, never on the bounds.
// Behind the last pinned slot of every lane of a wave (the free tail) they are the plan's table
// (zmpc_strict_lq_table_kernel, the same arithmetic), so a tail slot costs the s recursion twice
// and the forward step, with no flag loads and no costate.  In sweep A, a segment before the
// tail in which no lane has a pinned slot runs the free form of the step.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <type_traits>

#include "strict_eta.h"
#include "zmpc_internal.h"

#pragma clang fp contract(off)  // every fused multiply-add below is an explicit fma()

namespace {

using namespace zmpc_eta;

// active-set pass cap (as strict.hip).  64 was too few: at (Q, R, h) = (0.1, 1e-3, 0.5) and
// N = 400 the reference's exact answer takes 150 primal-dual passes from a cold start and 212
// after an 800 N kick (strict_weights_long_ref.npz); the cap only bounds a cycling iteration
constexpr int LQ_MAXIT = 1024;
#ifdef ZMPC_DIAG
constexpr bool kLqProf = true;  // per-phase clocks (ZMPC_LQ_PROF), diagnostics build only
#else
constexpr bool kLqProf = false;
#endif
#ifndef ZMPC_LQ_DRIFT  // (A/B builds only: make ab)
#define ZMPC_LQ_DRIFT 4
#endif

// Riccati steps per checkpoint segment.  Fixed at 8: a segment's working-set flags are one
// 16-bit LDS word (Flags: [slot / 8][64], 2 bits per slot), which the segment loads, the
// new-flag writes and the warm-start shift all take whole (rounds 1-3 measured S = 6/10/12/16:
// slower or spilling).
constexpr int LQ_S = 8;
constexpr int LQ_DRIFT = ZMPC_LQ_DRIFT;  // timesteps a lane may run ahead of its wave's slowest lane
                              // (round 3, profiles/r3u/, r3drift/: 0/1/2/4/8 → 104.5/94.8/92.5/
                              // 90.9/92.7 ms at config 3 — the bound rows stay a few rows apart)
constexpr int kLdsCk = 2;  // at most this many LDS checkpoints per wave (LqArgs::nlck)
constexpr int TAB = 16;       // doubles per slot of the free-tail table: [0..2] K, [3] 1/Quu,
                              // [4..9] P after the slot (V_k: slots k..N−1 free), [10..12] Qux,
                              // padding

struct LqArgs {
  int N, NS;             // horizon, segments ⌈N/S⌉
  int nlck;              // working-set checkpoints kept in LDS per wave (0..kLdsCk): those of
                         // segments jt − 1 .. jt − nlck, sweep A's first and sweep B's last
  int toff;              // window slot k reads time i + toff + k (1 rollout, 0 step)
  int window_mode;
  int64_t n;             // samples per walk (rollout; 1 in window mode)
  int64_t nsteps;        // timesteps (n − 1, or 1)
  int64_t B;             // walks (rollout) or instances (step)
  // staged bounds, tiled [axis][group of 64 walks][row][64] of (z_ref, half-width) pairs: row t of a
  // window slot holds the group's 64 pairs for time t, one 16-byte load per lane (rows past
  // n − 1 repeat the last sample — the window padding of zmp_controller.py:81-88 — so no
  // clamping in the kernel)
  int64_t rows;          // rows per (axis, group)
  int64_t groups;        // groups per axis in the staging (1 for a shared CoP)
  int shared;            // 1: every walk reads group 0 (bounds_stride = 0)
  const double2* hl;
  // run-length bounds (RUNS kernels): per (axis, group) [run][64] (z_ref, half-width) pairs and
  // [run][64] start times (two INT_MAX sentinels after a lane's last run: the last run extends
  // over the window padding of zmp_controller.py:81-88); rstride elements per (axis, group)
  const double2* rs;
  const int* rt;
  int64_t rstride;
  const double* x0;      // rollout [B,2,3], step [B,3]
  const double* kick;    // [B] or null
  int64_t kick_step;
  const int64_t* kick_steps;
  const int32_t* perm;   // walk of lane position b0 + lane (order.hip), or null (identity)
  double* out;           // rollout hist [B,n,2,3], step x_next [B,3]
  int32_t* status;
  double* ck;            // checkpoints [waves][NS][9][64]
  unsigned long long* cnt;  // plan work counters (zmpc_plan_counters), may be null
  double T, T2, T3;      // reference-form state advance (zmp_controller.py:18-20,199)
  double Tsq, Tcu;       // T², T³ (coordinate scaling)
  // z-form step constants (strict_eta.h fill_eta): π, 1/π, 1/π², γ', ρ, ε = ρ/π², εγ', εγ'²,
  // 1 + ε, ρ/π, and the multiplier tolerance (metres, 1e-13)
  double pi, ipi, ipi2, gp, rho, eps, epsg, epsg2, quz0, epi, tolnu;
  // task queue (rollouts with more waves than the chip holds): the grid is the resident
  // blocks; each wave runs its own task first (gw), then takes the next from *queue:
  // queue index q → the remaining blocks' y waves first (the heavier axis), then their x
  // waves.  null: one task per wave (gw).
  int* queue;
  int64_t qblock0;       // first block not in the grid
  int64_t nblocks;       // blocks of the whole launch (G waves each)
  unsigned long long* prof;  // diagnostics build only (ZMPC_LQ_PROF): clocks per phase and axis
  int skip_axis;         // diagnostics build only (ZMPC_LQ_SKIP): 1 / 2 = the x / y tasks end at once
};

// Slot q's flag in a segment's word: its 2-bit field, sign-extended.
__device__ __forceinline__ int flag_at(unsigned w, int q) {
  return (int)(w << (30 - 2 * q)) >> 30;
}

// The 2-bit field of flag value v (−1, 0, +1) at slot q.
__device__ __forceinline__ unsigned flag_bits(int v, int q) { return (unsigned)(v & 3) << (2 * q); }

template <int S>
struct SegIn {  // a segment's window slots: z_ref, half-width of the box, working-set flags
  static_assert(S == 8, "a segment's flags are one 16-bit word of Flags");
  double r[S], h[S];
  unsigned fw;  // the flags, a 2-bit two's-complement field per slot (slot q: bits 2q, 2q + 1):
                // 0 free, +1 at z_max = r + h, −1 at z_min = r − h
  __device__ __forceinline__ int f(int q) const { return flag_at(fw, q); }
};

template <int S>
struct SegOut {  // a segment's feedback (v = −K η − kff) and forward outputs, per step
  double K0[S], K1[S], K2[S], kf[S];
  double w[S];             // forward: v_k (= T³u_k)
  unsigned fw;             // the segment's new flag word (S = 8): the forward's verdicts on the
                           // free slots, the costate's on the pinned ones; one LDS write
};

// A free-tail step: P, K, Qux and 1/Quu come from the table, only s moves (strict_eta.h's
// s ← Fᵀs + Qux kff with kff = −(r + s2/π)/Quu).
__device__ __forceinline__ void ric_tail(const LqArgs& a, Ric& v, double r, double u0, double u1,
                                         double u2, double iq, double& kf) {
  kf = -fma(a.ipi, v.s2, r) * iq;
  const double as2 = a.ipi * v.s2;
  const double f0 = v.s0 - as2, f1 = (v.s0 + v.s1) - as2;
  v.s0 = fma(u0, kf, f0);
  v.s1 = fma(u1, kf, f1);
  v.s2 = fma(u2, kf, f1);
}

struct Lane {
  const double2* hl;  // wave's staged (z_ref, half-width) rows (uniform)
  const double2* rs;  // RUNS: wave's run table (uniform)
  const int* rt;
  int lane;  // the wave lane (slot flags in LDS)
  int col;   // the lane's column in the staged tables (its walk position mod 64)
};

// RUNS: a lane's cursor on its walk's run list while a sweep moves through the window: the
// current run's (z_ref, half-width), the neighbouring run the sweep reaches next and both
// boundaries, so a crossing needs no load it must wait for (the refill of the neighbour lands
// with the segment's checkpoint loads).  The CoP producer's bounds are one box per support
// phase (cop_generator.py:34-115): ≈16 runs per 420-sample walk, so a sweep crosses a handful
// of boundaries instead of loading one row per slot.
struct RunCursor {
  int ci;      // current run
  int e1, e2;  // forward: starts of runs ci+1, ci+2; backward: starts of runs ci, ci−1
  double r, h, nr, nh;
  // the neighbour as last loaded: a crossing loads the new run's neighbour here, and the next
  // segment takes it into (nr, nh, e2) — one segment after the load was issued
  double pnr, pnh;
  int pe2;
};

__device__ __forceinline__ RunCursor run_fwd(const Lane& L, int ci) {
  RunCursor c;
  c.ci = ci;
  const double2 v = L.rs[ci * 64 + L.col], w = L.rs[(ci + 1) * 64 + L.col];
  c.r = v.x;
  c.h = v.y;
  c.nr = w.x;
  c.nh = w.y;
  c.e1 = L.rt[(ci + 1) * 64 + L.col];
  c.e2 = L.rt[(ci + 2) * 64 + L.col];
  c.pnr = c.nr;
  c.pnh = c.nh;
  c.pe2 = c.e2;
  return c;
}

__device__ __forceinline__ RunCursor run_bwd(const Lane& L, int ci) {
  RunCursor c;
  c.ci = ci;
  const int pi = max(ci - 1, 0);
  const double2 v = L.rs[ci * 64 + L.col], w = L.rs[pi * 64 + L.col];
  c.r = v.x;
  c.h = v.y;
  c.nr = w.x;
  c.nh = w.y;
  c.e1 = L.rt[ci * 64 + L.col];
  c.e2 = L.rt[pi * 64 + L.col];
  c.pnr = c.nr;
  c.pnh = c.nh;
  c.pe2 = c.e2;
  return c;
}

// Fill a segment's bounds from the runs (times t0 .. t0 + S − 1; backward sweeps descending).
// Most segments lie inside one run for every lane of the wave: one test per segment.  Where a
// lane crosses once, the wave walks the slots taking the neighbour already in registers; the
// crossing lanes load their new run's neighbour into (pnr, pnh, pe2), which nothing reads before
// the next segment, so the load lands while this segment computes.  (A refill into the cursor
// itself was read again within the segment: the compiler waited for it at the branch's join —
// the full latency at every crossing, and in sweep A behind the segment's checkpoint stores.)  A
// segment in which some lane crosses twice (a run shorter than S slots) takes the per-slot walk
// with synchronous refills.
template <int S, bool FWD>
__device__ __forceinline__ void seg_runs(const Lane& L, int t0, RunCursor& c, double* r,
                                         double* h) {
  c.nr = c.pnr;
  c.nh = c.pnh;
  c.e2 = c.pe2;
  const bool cross = FWD ? (t0 + S - 1 >= c.e1) : (t0 < c.e1);
  if (!__any(cross)) {
#pragma unroll
    for (int q = 0; q < S; ++q) {
      r[q] = c.r;
      h[q] = c.h;
    }
    return;
  }
  const bool twice = FWD ? (t0 + S - 1 >= c.e2) : (t0 < c.e2);
  if (__any(twice)) {
    if constexpr (FWD) {
#pragma unroll
      for (int q = 0; q < S; ++q) {
        if (t0 + q >= c.e1) {  // into run ci+1 (runs are ≥ 1 slot: one crossing per slot)
          ++c.ci;
          c.r = c.nr;
          c.h = c.nh;
          c.e1 = c.e2;
          const double2 w = L.rs[(c.ci + 1) * 64 + L.col];
          c.nr = w.x;
          c.nh = w.y;
          c.e2 = L.rt[(c.ci + 2) * 64 + L.col];
        }
        r[q] = c.r;
        h[q] = c.h;
      }
    } else {
#pragma unroll
      for (int q = S - 1; q >= 0; --q) {
        if (t0 + q < c.e1) {  // into run ci−1
          --c.ci;
          c.r = c.nr;
          c.h = c.nh;
          c.e1 = c.e2;
          const int pi = max(c.ci - 1, 0);
          const double2 w = L.rs[pi * 64 + L.col];
          c.nr = w.x;
          c.nh = w.y;
          c.e2 = L.rt[pi * 64 + L.col];
        }
        r[q] = c.r;
        h[q] = c.h;
      }
    }
    c.pnr = c.nr;
    c.pnh = c.nh;
    c.pe2 = c.e2;
    return;
  }
  bool crossed = false;
  if constexpr (FWD) {
#pragma unroll
    for (int q = 0; q < S; ++q) {
      if (t0 + q >= c.e1) {
        ++c.ci;
        c.r = c.nr;
        c.h = c.nh;
        c.e1 = c.e2;
        crossed = true;
      }
      r[q] = c.r;
      h[q] = c.h;
    }
    if (crossed) {
      const double2 w = L.rs[(c.ci + 1) * 64 + L.col];
      c.pnr = w.x;
      c.pnh = w.y;
      c.pe2 = L.rt[(c.ci + 2) * 64 + L.col];
    }
  } else {
#pragma unroll
    for (int q = S - 1; q >= 0; --q) {
      if (t0 + q < c.e1) {
        --c.ci;
        c.r = c.nr;
        c.h = c.nh;
        c.e1 = c.e2;
        crossed = true;
      }
      r[q] = c.r;
      h[q] = c.h;
    }
    if (crossed) {
      const int pi = max(c.ci - 1, 0);
      const double2 w = L.rs[pi * 64 + L.col];
      c.pnr = w.x;
      c.pnh = w.y;
      c.pe2 = L.rt[pi * 64 + L.col];
    }
  }
}

// Per-lane working-set flags of the wave's N slots in LDS (0 free, +1 at z_max, −1 at z_min):
// two bits per slot; a lane's 8-slot segment is one 16-bit word (one ds_read_u16 per segment,
// held packed in a register), two segments one 32-bit bank word of the lane, [slot / 16][64
// lanes] (so that no two lanes share a bank word).  Every access is a 16-bit one: 32-bit accesses
// to the same words through another pointer type are not ordered with these by the compiler
// (type-based aliasing) — a first version that shifted 32 bits at a time computed the same
// solutions in more passes.
// Round 6: 2 bits instead of a byte per slot — 128 instead of 512 bytes per segment and wave, so
// that 8-wave workgroups fit horizons up to 896 (224 with bytes) and the freed LDS holds
// checkpoints.
struct Flags {
  unsigned short* p;
  __device__ __forceinline__ static int idx(int c, int lane) {
    return ((c >> 1) * 64 + lane) * 2 + (c & 1);
  }
  __device__ __forceinline__ int get(int k, int lane) const { return flag_at(word(k >> 3, lane), k & 7); }
  __device__ __forceinline__ void set(int k, int lane, int v) const {
    const int c = k >> 3, q = k & 7;
    set_word(c, lane, (word(c, lane) & ~(3u << (2 * q))) | flag_bits(v, q));
  }
  // the 8 flags of slots 8c .. 8c + 7
  __device__ __forceinline__ unsigned word(int c, int lane) const { return p[idx(c, lane)]; }
  __device__ __forceinline__ void set_word(int c, int lane, unsigned w) const {
    p[idx(c, lane)] = (unsigned short)w;
  }
};

// 32-bit flag words of a wave (two segments each)
__host__ __device__ constexpr int flag_dwords(int NS) { return (NS + 1) / 2; }

// A value function parked in the wave's LDS slot ([9][64] doubles).
__device__ __forceinline__ void park(double* vp, const Ric& v, int lane) {
  double* q = vp + lane;
  q[0] = v.p00;
  q[64] = v.p01;
  q[128] = v.p02;
  q[192] = v.p11;
  q[256] = v.p12;
  q[320] = v.p22;
  q[384] = v.s0;
  q[448] = v.s1;
  q[512] = v.s2;
}

__device__ __forceinline__ void unpark(const double* vp, Ric& v, int lane) {
  const double* q = vp + lane;
  v.p00 = q[0];
  v.p01 = q[64];
  v.p02 = q[128];
  v.p11 = q[192];
  v.p12 = q[256];
  v.p22 = q[320];
  v.s0 = q[384];
  v.s1 = q[448];
  v.s2 = q[512];
}

// A segment's flags as one word (segment j is flag word j).
template <int S>
__device__ __forceinline__ unsigned seg_flags(const Flags& fl, int j, int lane) {
  return fl.word(j, lane);
}

// Issue the loads of segment j's slots (bounds, and the flags when FLAGS).  Slots past N read
// padded rows (loaded, never used) so the loads carry no guards.
template <int S, bool FLAGS>
__device__ __forceinline__ void seg_load(const LqArgs& a, int j, const Lane& L, int64_t i,
                                         const Flags& fl, SegIn<S>& in) {
  // segment's first row (the lane's own timestep); its S rows are 1 KiB apart: one address,
  // immediate offsets
  const int64_t row0 = i + a.toff + (int64_t)j * S;
  const double2* hp = L.hl + row0 * 64;
#pragma unroll
  for (int q = 0; q < S; ++q) {
    const double2 v = hp[q * 64 + L.col];
    in.r[q] = v.x;
    in.h[q] = v.y;
  }
  if (FLAGS) in.fw = seg_flags<S>(fl, j, L.lane);
}

// The same from the run lists (RUNS): bounds from the lane's cursor, flags from LDS.
template <int S, bool FLAGS, bool FWD>
__device__ __forceinline__ void seg_load_runs(const LqArgs& a, int j, const Lane& L, int64_t i,
                                              RunCursor& c, const Flags& fl, SegIn<S>& in) {
  seg_runs<S, FWD>(L, (int)(i + a.toff) + j * S, c, in.r, in.h);
  if (FLAGS) in.fw = seg_flags<S>(fl, j, L.lane);
}

// No lane taking part has a pinned slot in the segment (wave-uniform).
template <int S>
__device__ __forceinline__ bool seg_free(const SegIn<S>& in) {
  return !__any(in.fw != 0);
}

// Riccati steps of segment j (slots jS + S−1 down to jS).  KEEP: feedback kept in g (sweep
// B) or dropped (sweep A).  FULL: every slot of the segment is < N (straight-line code).
// FREE: no lane has a pinned slot here.
template <int S, bool FULL, bool KEEP, bool FREE>
__device__ __forceinline__ void seg_riccati(const LqArgs& a, int j, Ric& v, const SegIn<S>& in,
                                            SegOut<S>& g) {
#pragma unroll
  for (int q = S - 1; q >= 0; --q) {
    const int k = j * S + q;
    if (FULL || k < a.N) {
      double K0, K1, K2, kf;
      if (FREE) {
        double iq, u0, u1, u2;
        ric_free(a, v, in.r[q], K0, K1, K2, kf, iq, u0, u1, u2);
      } else {
        ric_step(a, v, in.r[q], in.h[q], in.f(q), K0, K1, K2, kf);
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
      ric_tail(a, v, in.r[q], t[10], t[11], t[12], t[3], kf);
      if (KEEP) g.kf[q] = kf;
    }
  }
}

// Forward through segment j: roll the trajectory out (η advances to the segment's end), primal
// check of the free slots — their new flags go to LDS here (predicated stores; the pinned
// slots' come from the costate) — and the per-step input of the costate sweep.
template <int S, bool FULL>
__device__ __forceinline__ void seg_forward(const LqArgs& a, int j, const SegIn<S>& in,
                                            SegOut<S>& g, double* x, double& u0, bool& changed,
                                            int& kl, const Flags& fl, int lane) {
  const double tol = 1e-13;  // as strict.hip (tolz)
  g.fw = in.fw;  // (a free slot's byte is 0 until its verdict)
#pragma unroll
  for (int q = 0; q < S; ++q) {
    const int k = j * S + q;
    if (FULL || k < a.N) {
      double u, z;
      fwd_step(a, g.K0[q], g.K1[q], g.K2[q], g.kf[q], x, u, z);
      if (k == 0) u0 = u;
      const double d = z - in.r[q], ht = in.h[q] + tol;
      g.w[q] = u;
      const int nf = (d > ht) ? 1 : ((d < -ht) ? -1 : 0);
      if (in.f(q) == 0) {
        g.fw |= flag_bits(nf, q);
        changed |= nf != 0;
        kl = nf ? k : kl;  // (slots ascend)
      }
    }
  }
}

// Forward through a free-tail segment (table K, kff from seg_tail): primal check and the new
// flags (every slot here is free for every lane taking part, so no costate is needed).
template <int S, bool FULL>
__device__ __forceinline__ void seg_forward_tail(const LqArgs& a, const double* __restrict__ tab,
                                                 int j, const SegIn<S>& in, const SegOut<S>& g,
                                                 double* x, double& u0, bool& changed, int& kl,
                                                 const Flags& fl, int lane) {
  const double tol = 1e-13;
  unsigned fw = 0;  // (every slot of a tail segment is free for the lanes taking part)
#pragma unroll
  for (int q = 0; q < S; ++q) {
    const int k = j * S + q;
    if (FULL || k < a.N) {
      const double* t = tab + (size_t)k * TAB;
      double u, z;
      fwd_step(a, t[0], t[1], t[2], g.kf[q], x, u, z);
      if (k == 0) u0 = u;
      const double d = z - in.r[q], ht = in.h[q] + tol;
      const int nf = (d > ht) ? 1 : ((d < -ht) ? -1 : 0);
      fw |= flag_bits(nf, q);
      changed |= nf != 0;
      kl = nf ? k : kl;
    }
  }
  fl.set_word(j, lane, fw);  // (slots past N stay 0)
}

// Costate sweep back through segment j from λ at its end (λ_k = ∇V_k(η_k) = Fᵀλ_{k+1} − επ v_k c̄,
// strict_eta.h): the bound multipliers ν_k of the pinned slots, dual check, the pinned slots'
// new flags (the free slots' were set by the forward); kl = the last slot pinned in the new set.
template <int S, bool FULL>
__device__ __forceinline__ void seg_costate(const LqArgs& a, int j, const SegIn<S>& in,
                                            SegOut<S>& g, double* lam, bool& changed,
                                            int& kl, const Flags& fl, int lane) {
  unsigned& fw = g.fw;  // (written to LDS by the caller)
#pragma unroll
  for (int q = S - 1; q >= 0; --q) {
    const int k = j * S + q;
    if (FULL || k < a.N) {
      const int f = in.f(q);
      {
        const double sg = (double)f;
        const double nu = pinned_nu(a, sg, in.h[q], g.w[q], lam);  // ν / Q (pinned slots only)
        // wrong-signed multiplier (ν < 0 at z_max, ν > 0 at z_min): σν < −tol
        const bool rel = sg * nu < -a.tolnu;
        if (f != 0) {
          fw &= rel ? ~(3u << (2 * q)) : ~0u;
          changed |= rel;
          kl = (!rel && k > kl) ? k : kl;
        }
      }
      costate_step(a, g.w[q], lam);
    }
  }
}

// Sweep B through one working-set segment: Riccati from its checkpoint (in v), forward,
// costate.  v is dead once the Riccati has run: `next` loads the next segment's checkpoint into
// it there, so that the load is in flight under this segment's forward and costate.  (lap: the
// diagnostics build's phase clock)
// RECOMP = false: the feedback is already in g and V at the segment's end parked (segment 0,
// from sweep A).
template <int S, bool FULL, bool RECOMP, class Next, class Lap>
__device__ __forceinline__ void seg_sweep_b(const LqArgs& a, int j, Ric& v, const SegIn<S>& in,
                                            SegOut<S>& g, double* xs, double& u0, bool& changed,
                                            int& kl, const Flags& fl, int lane, double* vpark,
                                            Next& next, Lap& lap, bool fr) {
  if constexpr (RECOMP) {
    // V at the segment's end, parked in LDS until the costate needs it (its registers hold the
    // next checkpoint meanwhile)
    park(vpark, v, lane);
    seg_riccati<S, FULL, true, false>(a, j, v, in, g);
    next(v);
  }
  lap(4);
  seg_forward<S, FULL>(a, j, in, g, xs, u0, changed, kl, fl, lane);
  lap(5);
  // (a segment no lane taking part pins needs no costate: it only prices pinned slots, and
  // the next segment's λ comes from its own parked V)
  if (!fr) {
    double lam[3];
    {
      const double* q = vpark + lane;
      lam[0] = fma(q[0], xs[0], fma(q[64], xs[1], q[128] * xs[2])) - q[384];
      lam[1] = fma(q[64], xs[0], fma(q[192], xs[1], q[256] * xs[2])) - q[448];
      lam[2] = fma(q[128], xs[0], fma(q[256], xs[1], q[320] * xs[2])) - q[512];
    }
    seg_costate<S, FULL>(a, j, in, g, lam, changed, kl, fl, lane);
  }
  fl.set_word(j, lane, g.fw);
  lap(6);
}

// Checkpoints are written once and read once per pass.  With per-walk bounds (whose rows are
// re-read every timestep and do not fit the caches) they go non-temporal (NT), so they do not
// push those rows out; with a shared CoP the bounds are cache-resident anyway and the
// checkpoints are better off cached (config 3: 84.4 → 82.5 ms NT; config 4: 112.6 → 102.4 ms
// cached, profiles/r3nt/).
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
};

constexpr int kCkStride = 9 * 64;  // doubles of one segment's checkpoint per 64 lanes

template <bool NT>
__device__ __forceinline__ void ck_store(const CkIO<NT>& io, double* ck, int j, const Ric& v,
                                         int lane) {
  double* p = ck + (size_t)j * kCkStride + lane;
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

template <bool NT>
__device__ __forceinline__ void ck_store_s(const CkIO<NT>& io, double* ck, int j, const Ric& v,
                                           int lane) {
  double* p = ck + (size_t)j * kCkStride + lane;
  io.st(p + 384, v.s0);
  io.st(p + 448, v.s1);
  io.st(p + 512, v.s2);
}

template <bool NT>
__device__ __forceinline__ void ck_load(const CkIO<NT>& io, const double* ck, int j, Ric& v,
                                        int lane) {
  const double* p = ck + (size_t)j * kCkStride + lane;
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
  const double* p = ck + (size_t)j * kCkStride + lane;
  v.s0 = io.ld(p + 384);
  v.s1 = io.ld(p + 448);
  v.s2 = io.ld(p + 512);
}

// G waves per workgroup.  G = 8: waves 0..3 take the x axis and 4..7 the y axis of the same
// four 64-walk groups, so each SIMD (waves w and w + 4 under the round-robin placement) holds
// one wave of each axis — the y axis carries nearly all of the active-set work, and an
// axis-pure SIMD would idle once its x waves are done (config 3: 117 → 98 ms, round 1).  Longer
// horizons (slot flags of G waves beyond LDS) run G = 4 (x/y = wave parity) or 2.  (Round 4:
// waves of 32 walks × both axes, so that every SIMD keeps two y-carrying waves to the end, are
// slower — config 3 87.0 vs 64.9 ms: the x lanes then run the working-set form up to the wave's
// last pinned slot, 0.76 of the pass-slots instead of 0.48, profiles/r4/r4l_*.)
// QUEUE: a grid of the resident blocks whose waves loop over tasks (a.queue); without it each
// wave runs its one task.  The task is a lambda called once or in the loop: written inline in
// the loop, the loop's live ranges cost the sweeps ≈75 more spilled registers (config 4 76.2
// ms, config 3 65.7); as a lambda the queue form spills 37–60 and runs config 4 in 72.3 ms,
// at +1 % for config 3 (profiles/r4/r4z/, r4aa/).
template <int S, int G, bool NT, bool RUNS, bool QUEUE>
__global__ void __launch_bounds__(64 * G, 2)
    zmpc_strict_lq_kernel(LqArgs a, const double* __restrict__ tab) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lq_smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * G + wave;
  const int N = a.N;
  // slot flags [⌈NS/2⌉][64] 32-bit words (slots past N stay 0: the last segment's loads are
  // unguarded)
  const int NSd = flag_dwords(a.NS);
  const Flags fl{reinterpret_cast<unsigned short*>(lq_smem) + (size_t)wave * NSd * 128};
  // after the G waves' flags: each wave's parked V at the end of its current sweep-B segment
  // ([9][64] doubles; 16-byte aligned: a wave's flags are ⌈NS/2⌉·256 bytes)
  double* vpark = reinterpret_cast<double*>(lq_smem + (size_t)G * NSd * 256) +
                  wave * (12 + 9 * a.nlck) * 64;
  // and behind it the lane's state x (the reference form), [3][64]: read at a pass's start and
  // at its end only, so it need not hold registers through the sweeps
  double* xpark = vpark + 9 * 64;
  // and behind that the wave's LDS checkpoints ([nlck][9][64] doubles): working-set segments
  // jt − 1 .. jt − nlck, written first in sweep A and read last in sweep B, so their global
  // copies were the ones the caches had lost by then (round 6: config 3's checkpoints were
  // nearly all of its 129 GB per launch)
  double* ckl = xpark + 3 * 64;
  double* ck = a.ck + (size_t)gw * a.NS * kCkStride;
  const CkIO<NT> io{};
  // work counters, wave-uniform 64-bit sums (scalar registers): wave passes, lane passes (the
  // lanes taking part) and their working-set slots
  unsigned long long n_wave_pass = 0, n_lane_pass = 0, n_ws_slots = 0;
#ifdef ZMPC_DIAG
  unsigned long long n_sb_ws = 0, n_sb_free = 0;
#endif
  unsigned itmax = 0;  // most passes of one of this lane's solves (counter [8])
  // one task: the rollout of one 64-walk group on one axis (this wave's lanes)
  auto run_task = [&](const int64_t task) {
  // (the task's block and wave: the kernel's own without a queue)
  const int64_t tblk = QUEUE ? task / G : (int64_t)blockIdx.x;
  const int twave = QUEUE ? (int)(task % G) : wave;
  int axis;
  int64_t pos;  // the lane's walk position (order.hip's kick order, or the walk itself)
  if (a.window_mode) {
    axis = 0;
    pos = task * 64 + lane;
  } else if (G == 8) {
    axis = twave >> 2;
    pos = (tblk * 4 + (twave & 3)) * 64 + lane;
  } else {
    axis = (int)(task & 1);
    pos = (task >> 1) * 64 + lane;
  }
  // lane position pos runs walk b (the kick order of order.hip, or the identity); the staged
  // bounds follow the positions (table (axis, pos / 64), column pos % 64), everything per walk
  // (x0, kick, history, status) b
  const bool valid = pos < a.B;
#ifdef ZMPC_DIAG
  if (a.skip_axis == axis + 1) return;  // (diagnostics: what one axis's tasks cost)
#endif
  // one resident round (no queue): the y waves carry nearly all the working-set work and set
  // the kernel's time, so they issue first when their SIMD's x wave competes (wave priority;
  // the x waves take the slack) — config 3 50.0 → 45.5 ms.  With the queue the same priority
  // cost config 4 62.7 → 65.0 ms (its later rounds mix y and x tasks), profiles/r5aj/.
  if constexpr (!QUEUE) {
    if (axis == 1)
      __builtin_amdgcn_s_setprio(2);
    else
      __builtin_amdgcn_s_setprio(0);
  }
  const int64_t b = (valid && a.perm) ? (int64_t)a.perm[pos] : pos;
  Lane L;
  L.lane = lane;
  L.col = RUNS ? lane : (int)(pos & 63);  // (pos = 64·group + lane; per form, as allocates best)
  {
    // the wave's (axis, group) tables; the run tables' base wave-uniform (SGPRs), the lane's
    // column added per access
    const int64_t g = a.shared ? 0 : (pos >> 6);
    if constexpr (RUNS) {
      const int64_t off = ((int64_t)axis * a.groups + g) * a.rstride;
      const int lo = __builtin_amdgcn_readfirstlane((int)(off & 0xffffffff));
      const int hi = __builtin_amdgcn_readfirstlane((int)(off >> 32));
      const int64_t uoff = ((int64_t)hi << 32) | (uint32_t)lo;
      L.rs = a.rs + uoff;
      L.rt = a.rt + uoff;
    } else {
      L.hl = a.hl + ((int64_t)axis * a.groups + g) * a.rows * 64;
    }
  }
  // RUNS: the run holding the window's last slot of the last segment (sweep A starts there)
  // and the one holding its first slot (sweep B), advanced as the lane's timestep moves
  int ra = 0, rb = 0;
  if (RUNS && valid) {  // (positions past B may lie past the staged groups: never read)
    const int tA = (int)a.toff + a.NS * S - 1, tB = (int)a.toff;
    while (L.rt[(ra + 1) * 64 + L.col] <= tA) ++ra;
    while (L.rt[(rb + 1) * 64 + L.col] <= tB) ++rb;
  }
  const int jfull = N / S;  // segments [0, jfull) are full
  for (int c = 0; c < 2 * NSd; ++c) fl.set_word(c, lane, 0u);

  {
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
    xpark[lane] = x[0];
    xpark[64 + lane] = x[1];
    xpark[128 + lane] = x[2];
  }
  int fq = 0;
  const int kstep =
      (!a.window_mode && axis == 1 && a.kick != nullptr && valid)
          ? (int)(a.kick_steps ? a.kick_steps[b] : a.kick_step)
          : -1;

  // Each lane walks its own timestep i: a pass runs for every lane still inside its rollout
  // and at most LQ_DRIFT timesteps ahead of the wave's slowest lane (so a slot's bound loads
  // stay within a few 1-KiB rows); a lane whose working set repeated advances (state, history,
  // shifted warm start) while the others keep iterating.
  int i = 0;  // (the lane's timestep; n < 2^31)
  bool active = valid && a.nsteps > 0;
  int it = 0;
  int klast = -1;      // last pinned slot of this lane's working set (−1: none)
  // diagnostics: clocks of sweep A, sweep B's working-set and tail segments, the rest; task
  // [0] sweep A tail, [1] sweep A working set, [2] sweep B's segment set-up and checkpoint
  // wait ([9] of segment 1), [4] its Riccati recompute, [5] forward, [6] costate, [7] sweep B
  // tail, [3] the rest
  unsigned long long pc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long pt = (kLqProf && a.prof) ? clock64() : 0, ptask = pt;
  auto lap = [&](int ph) {
    if (kLqProf && a.prof) {
      const unsigned long long t = clock64();
      pc[ph] += t - pt;
      pt = t;
    }
  };
  while (__any(active)) {
    ++n_wave_pass;
    int imin = active ? (int)i : 0x7fffffff;
    for (int o = 32; o > 0; o >>= 1) imin = min(imin, __shfl_xor(imin, o));
    const bool part = active && i <= imin + LQ_DRIFT;
    // segments [jt, NS) hold no pinned slot of any lane taking part: the free tail
    int kw = part ? klast : -1;
    for (int o = 32; o > 0; o >>= 1) kw = max(kw, __shfl_xor(kw, o));
    const int jt = __builtin_amdgcn_readfirstlane(kw < 0 ? 0 : kw / S + 1);
    {
      const unsigned long long np = (unsigned long long)__popcll(__ballot(part));
      n_lane_pass += np;
      n_ws_slots += np * (unsigned long long)min(jt * S, N);
    }
    if (part) {
      lap(3);
      double u0 = 0.0;
      bool changed = false;
      int kl = -1;
      {
        Ric v{0, 0, 0, 0, 0, 0, 0, 0, 0};
        SegIn<S> cur;
        SegOut<S> g;
        RunCursor rc{};
        if constexpr (RUNS) rc = run_bwd(L, ra);
        // sweep B's first segment starts from V at the end of segment 0, which sweep A holds
        // just before its last segment: parked in LDS (not stored), so that sweep B does not
        // begin with a global load — one that would wait for every checkpoint store of sweep A
        // (vmcnt counts loads and stores together, in issue order)
        // sweep A, free tail: the s recursion, checkpoints of s
#pragma unroll 1
        for (int j = a.NS - 1; j >= jt; --j) {
          if constexpr (RUNS)
            seg_load_runs<S, false, false>(a, j, L, i, rc, fl, cur);
          else
            seg_load<S, false>(a, j, L, i, fl, cur);
          // (s at the end of the last segment is V_N's: 0, no checkpoint)
          if (j == 0)
            park(vpark, v, lane);
          else if (j < a.NS - 1)
            ck_store_s(io, ck, j, v, lane);
          if (j < jfull)
            seg_tail<S, true, false>(a, tab, j, v, cur, g);
          else
            seg_tail<S, false, false>(a, tab, j, v, cur, g);
        }
        lap(0);
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
        for (int j = jt - 1; j >= 1; --j) {
          if constexpr (RUNS)
            seg_load_runs<S, true, false>(a, j, L, i, rc, fl, cur);
          else
            seg_load<S, true>(a, j, L, i, fl, cur);
          if (j >= jt - a.nlck)
            park(ckl + (jt - 1 - j) * 9 * 64, v, lane);
          else
            ck_store(io, ck, j, v, lane);
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
        // segment 0, its feedback kept: it is sweep B's first segment, which then needs no
        // recompute (its V at the end parked for the costate)
        if (jt > 0) {
          if constexpr (RUNS)
            seg_load_runs<S, true, false>(a, 0, L, i, rc, fl, cur);
          else
            seg_load<S, true>(a, 0, L, i, fl, cur);
          park(vpark, v, lane);
          if (0 < jfull)
            seg_riccati<S, true, true, false>(a, 0, v, cur, g);
          else
            seg_riccati<S, false, true, false>(a, 0, v, cur, g);
        }
        lap(1);
        // sweep B: per segment from the front — recompute its steps from the checkpoint,
        // forward, then (working-set segments) the costate back through it
        double xs[3];  // η
        {
          const double x0 = xpark[lane], x1 = xpark[64 + lane], x2 = xpark[128 + lane];
          const double xi1 = a.T * x1, xi2 = a.Tsq * x2;  // ξ
          xs[0] = fma(-1.0 / 6.0, xi2, x0);
          xs[1] = fma(-0.5, xi2, xi1);
          xs[2] = xi2;
        }
        if constexpr (RUNS) rc = run_fwd(L, rb);
        // the next segment's checkpoint into v: full for a working-set segment, s for a tail one
        auto next = [&](Ric& w, int j) {
          if (j + 1 < jt - a.nlck)
            ck_load(io, ck, j + 1, w, lane);
          else if (j + 1 < jt)
            unpark(ckl + (jt - 2 - j) * 9 * 64, w, lane);
          else if (j + 1 < a.NS - 1)
            ck_load_s(io, ck, j + 1, w, lane);
          else if (j + 1 == a.NS - 1)
            w.s0 = w.s1 = w.s2 = 0.0;  // V_N = 0
        };
        // V at the end of segment 0 (later segments' come by `next`); with working-set segments
        // sweep A has left segment 0's feedback in g and V at its end parked: the checkpoint of
        // segment 1 can be in flight from here
        if (jt > 0)
          next(v, 0);
        else
          unpark(vpark, v, lane);
        // one working-set segment of sweep B (R: recompute its feedback from the checkpoint)
        auto seg_b = [&](int j, auto R) {
          if constexpr (RUNS)
            seg_load_runs<S, true, true>(a, j, L, i, rc, fl, cur);
          else
            seg_load<S, true>(a, j, L, i, fl, cur);
          if (kLqProf && a.prof) {  // (diagnostics: the checkpoint's arrival timed apart;
            __builtin_amdgcn_s_waitcnt(0);  // segment 1's, behind sweep A's stores, separately)
            if (j == 1)
              lap(9);
            else
              lap(2);
          }
          auto nx = [&](Ric& w) { next(w, j); };
#ifdef ZMPC_DIAG
          ++n_sb_ws;  // diagnostics: sweep-B working-set segments, and those no lane pins
          if (seg_free(cur)) ++n_sb_free;
#endif
          // (43 % of these segments have no pinned slot in any lane taking part, config 3,
          // diagnostics build: they skip the costate — config 3 51.3 → 50.0 ms, profiles/r5ae/.
          // A free Riccati form for them as well spills: 300 B in round 5, and 74.9 vs 65.0 ms
          // in round 4, profiles/r4/r4n/)
          const bool fr = seg_free(cur);
          if (j < jfull) {
            seg_sweep_b<S, true, decltype(R)::value>(a, j, v, cur, g, xs, u0, changed, kl, fl,
                                                     lane, vpark, nx, lap, fr);
          } else {
            seg_sweep_b<S, false, decltype(R)::value>(a, j, v, cur, g, xs, u0, changed, kl, fl,
                                                      lane, vpark, nx, lap, fr);
          }
        };
        if (jt > 0) seg_b(0, std::false_type{});  // (sweep A's feedback)
#pragma unroll 1
        for (int j = 1; j < jt; ++j) seg_b(j, std::true_type{});
#pragma unroll 1
        for (int j = jt; j < a.NS; ++j) {  // (v.s holds the segment's checkpoint: `next`)
          if constexpr (RUNS)
            seg_load_runs<S, false, true>(a, j, L, i, rc, fl, cur);
          else
            seg_load<S, false>(a, j, L, i, fl, cur);
          if (j < jfull) {
            seg_tail<S, true, true>(a, tab, j, v, cur, g);
            next(v, j);  // (s is dead after the segment's recursion)
            seg_forward_tail<S, true>(a, tab, j, cur, g, xs, u0, changed, kl, fl, lane);
          } else {
            seg_tail<S, false, true>(a, tab, j, v, cur, g);
            next(v, j);
            seg_forward_tail<S, false>(a, tab, j, cur, g, xs, u0, changed, kl, fl, lane);
          }
        }
        lap(7);
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
        const double x0 = xpark[lane], x1 = xpark[64 + lane], x2 = xpark[128 + lane];
        xn[0] = x0 + a.T * x1 + a.T2 * x2 + a.T3 * u0;
        xn[1] = x1 + a.T * x2 + a.T2 * u0;
        xn[2] = x2 + a.T * u0;
        if ((int)i == kstep) xn[1] -= a.kick[b];  // force kick (zmp_controller.py:90,105-106)
        if (!(isfinite(xn[0]) && isfinite(xn[1]) && isfinite(xn[2]))) fq |= ZMPC_ST_NONFINITE;
        xpark[lane] = xn[0];
        xpark[64 + lane] = xn[1];
        xpark[128 + lane] = xn[2];
        double* h = a.window_mode ? a.out + b * 3 : a.out + ((b * a.n + (int64_t)i + 1) * 2 + axis) * 3;
        h[0] = xn[0];
        h[1] = xn[1];
        h[2] = xn[2];
        ++i;
        it = 0;
        if constexpr (RUNS) {
          const int tA = (int)(i + a.toff) + a.NS * S - 1, tB = (int)(i + a.toff);
          if (L.rt[(ra + 1) * 64 + L.col] <= tA) ++ra;  // one slot per timestep: one run at most
          if (L.rt[(rb + 1) * 64 + L.col] <= tB) ++rb;
        }
        if (i < a.nsteps) {
          // warm start: the converged set shifted one slot towards the present (slot N−1
          // kept), this lane's column only
          // (flag words: each takes its upper 7 fields and the next word's first; the words past
          // the one holding the last pinned slot kl are zero and stay zero)
          {
            const int keep = fl.get(N - 1, lane);
            if (kl >= 0) {
              unsigned w = fl.word(0, lane);
              for (int c = 0; c <= (kl >> 3); ++c) {
                const unsigned nx = (c + 1 < a.NS) ? fl.word(c + 1, lane) : 0u;
                fl.set_word(c, lane, (w >> 2) | ((nx << 14) & 0xffffu));
                w = nx;
              }
            }
            fl.set(N - 1, lane, keep);
          }
          // the previous solve's terminal slot is no longer terminal: it starts free (its end
          // effect pinned it more often than the next solve keeps it; a CPU simulation of this
          // iteration on the default walk's y axis at F_ext 0/400/800 N: 1.387 → 1.310 passes
          // per solve, scripts/strict_warm_sim.py).  Slot N−1 keeps the copy.  The converged
          // set, hence the solution, is the same; only the passes to reach it change.
          if (N >= 2) fl.set(N - 2, lane, 0);
          klast = (kl >= N - 1) ? N - 1 : max(kl - 1, -1);
        } else {
          active = false;
        }
      } else {
        klast = kl;
      }
    }
  }
  if (kLqProf && a.prof) {
    lap(3);
    pc[8] = clock64() - ptask;
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < 10; ++q) atomicAdd(a.prof + axis * 11 + q, pc[q]);
      atomicAdd(a.prof + axis * 11 + 10, 1ull);
    }
  }
  if (valid && a.status != nullptr) {
    if (a.window_mode)
      a.status[b] = fq;
    else if (fq != 0)
      atomicOr(&a.status[b], fq);
  }
  };
  if constexpr (QUEUE && G == 8) {
    // the wave's own task (gw), then the queue's: one device-scope atomic per task (a task is a
    // whole rollout of 64 walks)
    int64_t task = gw;
    for (;;) {
    run_task(task);
    int q = 0;
    if (lane == 0) q = atomicAdd(a.queue, 1);
    q = __builtin_amdgcn_readfirstlane(__shfl(q, 0, 64));
    const int64_t rem = a.nblocks - a.qblock0;      // blocks not in the grid
    const int64_t half = rem * (G / 2);              // their y waves (G = 8: waves 4..7)
    if (q >= 2 * half) break;
    const int64_t qq = q < half ? q : q - half;
    const int64_t blk = a.qblock0 + qq / (G / 2);
    task = blk * G + (q < half ? G / 2 : 0) + qq % (G / 2);
    }
  } else {
    run_task(gw);  // one task per wave (the host takes the queue form for 8-wave blocks only)
  }
  if (a.cnt) {
    for (int o = 32; o > 0; o >>= 1) itmax = max(itmax, (unsigned)__shfl_xor((int)itmax, o));
    if (lane == 0) {
      atomicAdd(a.cnt + 0, n_wave_pass);
      atomicAdd(a.cnt + 1, n_lane_pass);
      atomicAdd(a.cnt + 2, n_ws_slots);
      if (gw == 0) atomicAdd(a.cnt + 3, 1ull);
#ifdef ZMPC_DIAG  // (the Herdt counter slots [6], [7], unused by a strict launch)
      atomicAdd(a.cnt + 6, n_sb_ws);
      atomicAdd(a.cnt + 7, n_sb_free);
#endif
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
    double K0, K1, K2, kf, iq, u0, u1, u2;
    ric_free(a, v, 0.0, K0, K1, K2, kf, iq, u0, u1, u2);
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
    t[10] = u0;
    t[11] = u1;
    t[12] = u2;
    for (int c = 13; c < TAB; ++c) t[c] = 0.0;
  }
}

// Stage bounds into the kernel's tiled layout: source elements (b, t, axis) at
// b·sb + min(t, nsrc − 1)·st + axis·sa of z_max and z_min → dst[((axis·G + b/64)·rows + t)·64
// + b%64] = (r, h) for t < rows, r = (z_max + z_min)/2 the reference's z_ref
// (zmp_controller.py:184) and h = (z_max − z_min)/2 (a pinned slot's target r ± h equals its
// bound to an ulp; the primal check's tolerance is 1e-13).  64 walks × 16 rows per workgroup through LDS;
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
      const double hi = s.hi[e], lo = s.lo[e];
      v = make_double2((hi + lo) / 2, (hi - lo) / 2);
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

// Run-length staging (RUNS kernels): one thread per (lane position, axis) walks its walk's n
// samples once and writes the runs of equal (z_ref, half-width) — bitwise equality — into its
// lane column of the (axis, group) table: rs[r][64], rt[r][64] = start time, then two INT_MAX
// sentinels (the last run covers the window padding).  Positions past B get one dummy run.
__global__ void __launch_bounds__(64) zmpc_runs_stage_kernel(StageArgs s, double2* rs, int* rt,
                                                             int64_t rstride) {
  const int lane = threadIdx.x;
  const int64_t grp = blockIdx.x, ax = blockIdx.y;
  const int64_t p = grp * 64 + lane;
  double2* R = rs + (ax * s.G + grp) * rstride + lane;
  int* Tt = rt + (ax * s.G + grp) * rstride + lane;
  int count = 0;
  if (p < s.B) {
    const int64_t b = s.perm ? (int64_t)s.perm[p] : p;
    double pr = 0.0, ph = 0.0;
    for (int64_t t = 0; t < s.nsrc; ++t) {
      const int64_t e = b * s.sb + t * s.st + ax * s.sa;
      const double hi = s.hi[e], lo = s.lo[e];
      const double r = (hi + lo) / 2, h = (hi - lo) / 2;  // z_ref (zmp_controller.py:184)
      if (t == 0 || r != pr || h != ph) {
        R[count * 64] = make_double2(r, h);
        Tt[count * 64] = (int)t;
        ++count;
        pr = r;
        ph = h;
      }
    }
  } else {
    R[0] = make_double2(0.0, 0.0);  // as the row staging's unused positions
    Tt[0] = 0;
    count = 1;
  }
  Tt[count * 64] = 0x7fffffff;
  Tt[(count + 1) * 64] = 0x7fffffff;
  R[count * 64] = make_double2(0.0, 0.0);  // (a forward cursor's neighbour, never used)
}

hipError_t stage_runs(const double* hi, const double* lo, int64_t sb, int64_t st, int64_t sa,
                      int64_t nsrc, int64_t B, int naxes, double2* rs, int* rt, int64_t rstride,
                      hipStream_t s, const int32_t* perm) {
  StageArgs g{hi, lo, sb, st, sa, nsrc, B, (B + 63) / 64, 0, naxes, perm, nullptr};
  hipLaunchKernelGGL(zmpc_runs_stage_kernel, dim3((unsigned)g.G, (unsigned)naxes), dim3(64), 0,
                     s, g, rs, rt, rstride);
  return hipGetLastError();
}

hipError_t stage(const double* hi, const double* lo, int64_t sb, int64_t st, int64_t sa,
                 int64_t nsrc, int64_t B, int64_t rows, int naxes, double2* dst, hipStream_t s,
                 const int32_t* perm = nullptr) {
  StageArgs g{hi, lo, sb, st, sa, nsrc, B, (B + 63) / 64, rows, naxes, perm, dst};
  const dim3 grid((unsigned)((rows + 15) / 16), (unsigned)g.G);
  hipLaunchKernelGGL(zmpc_bounds_stage_kernel, grid, dim3(256), 0, s, g);
  return hipGetLastError();
}

// Workgroup shapes: G waves per workgroup (the G waves' slot flags must fit a CU's LDS), each
// with cached or non-temporal checkpoints.
struct LqVariant {
  int G;
  void (*kernel)(LqArgs, const double*);     // checkpoints cached (shared CoP, window mode)
  void (*kernel_nt)(LqArgs, const double*);  // checkpoints non-temporal (per-walk bounds)
  void (*kernel_runs)(LqArgs, const double*);     // run-length bounds, cached checkpoints
  void (*kernel_runs_nt)(LqArgs, const double*);  // run-length bounds, non-temporal
  // the same four with the task queue (G = 8 only; null otherwise)
  void (*q_kernel)(LqArgs, const double*);
  void (*q_kernel_nt)(LqArgs, const double*);
  void (*q_kernel_runs)(LqArgs, const double*);
  void (*q_kernel_runs_nt)(LqArgs, const double*);
};

#define ZMPC_LQK(G, Q)                                                               \
  zmpc_strict_lq_kernel<LQ_S, G, false, false, Q>, zmpc_strict_lq_kernel<LQ_S, G, true, false, Q>, \
      zmpc_strict_lq_kernel<LQ_S, G, false, true, Q>, zmpc_strict_lq_kernel<LQ_S, G, true, true, Q>
#define ZMPC_LQV(G) {G, ZMPC_LQK(G, false), nullptr, nullptr, nullptr, nullptr}
// (The queue form exists for run-length bounds only: with the bounds staged one row per sample,
// ZMPC_OPT_STRICT_BOUNDS = 1, its instances spill 20 B — those launches take the one-round form.)
const LqVariant kLqVariants[] = {
    {8, ZMPC_LQK(8, false), nullptr, nullptr, zmpc_strict_lq_kernel<LQ_S, 8, false, true, true>,
     zmpc_strict_lq_kernel<LQ_S, 8, true, true, true>},  // default
    ZMPC_LQV(4),  // N up to 2176 (the default G = 8: up to 896)
    ZMPC_LQV(2),  // N up to 2464 (ZMPC_STRICT_MAX_N)
};
#undef ZMPC_LQV
#undef ZMPC_LQK
constexpr size_t kLdsCap = 160 * 1024;

// LDS of one workgroup: the G waves' slot flags (2 bits per slot and lane), parked V and state
// ([12][64] doubles each) and nlck LDS checkpoints ([9][64] doubles each).
constexpr size_t lq_lds_bytes(int G, int N, int nlck = 0) {
  const size_t segs = (size_t)(N + LQ_S - 1) / LQ_S;
  return (size_t)G * ((size_t)flag_dwords((int)segs) * 64 * 4 +
                      (12 + 9 * (size_t)nlck) * 64 * sizeof(double));
}

// LDS checkpoints per wave that fit beside a workgroup shape (config 3, N = 150: 2 at G = 8)
int lq_nlck_for(int G, int N) {
  int c = kLdsCk;
  while (c > 0 && lq_lds_bytes(G, N, c) > 160 * 1024) --c;
  return c;
}

static_assert(lq_lds_bytes(2, ZMPC_STRICT_MAX_N) <= kLdsCap, "ZMPC_STRICT_MAX_N past the LDS");

// The largest workgroup whose slot flags and parks fit a CU (N ≤ 2464 at G = 2).
const LqVariant* lq_variant_for(int N) {
  for (const LqVariant& c : kLqVariants)
    if (lq_lds_bytes(c.G, N) <= kLdsCap) return &c;
  return nullptr;
}

void fill_consts(const zmpc_plan* p, LqArgs& a) {
  a.N = p->N;
  a.NS = (p->N + LQ_S - 1) / LQ_S;
  a.T = p->T;
  a.T2 = p->T2_2;
  a.T3 = p->T3_6;
  fill_eta(a, p->T, p->hg, p->Q, p->R);
  a.cnt = p->lqcnt;
}

hipError_t launch_lq(const zmpc_plan* p, LqArgs& a, int64_t waves, hipStream_t s) {
  const LqVariant* var = lq_variant_for(p->N);
  if (!var) return hipErrorInvalidValue;
  const int64_t blocks = (waves + var->G - 1) / var->G;
  a.nlck = lq_nlck_for(var->G, p->N);
#ifdef ZMPC_DIAG
  if (const char* e = getenv("ZMPC_LQ_NLCK")) a.nlck = std::min(a.nlck, atoi(e));  // (A/B)
#endif
  const size_t lds = lq_lds_bytes(var->G, p->N, a.nlck);
  // cached checkpoints (see CkIO: with run-length bounds the window rows no longer compete
  // for the caches, and non-temporal checkpoints became the slower form — config 3 55.4 vs
  // 56.7 ms, diagnostics build, profiles/r5m/)
  bool nt = false;
#ifdef ZMPC_DIAG
  if (const char* e = getenv("ZMPC_LQ_NT")) nt = atoi(e) != 0;  // (diagnostics: A/B of the policy)
#endif
  auto k = a.rs ? (nt ? var->kernel_runs_nt : var->kernel_runs) : (nt ? var->kernel_nt : var->kernel);
  auto kq = a.rs ? (nt ? var->q_kernel_runs_nt : var->q_kernel_runs)
                 : (nt ? var->q_kernel_nt : var->q_kernel);
  // more blocks than the chip holds at once: a grid of the resident blocks and a task queue
  // (an x wave is done long before its SIMD's y wave; with one task per wave its slot idles
  // until the whole block has finished, while a queue refills it with the next y wave)
  int64_t grid = blocks;
  int* queue = a.queue;
  a.queue = nullptr;
  bool use_queue = true;
#ifdef ZMPC_DIAG
  if (getenv("ZMPC_LQ_NOQUEUE")) use_queue = false;  // (diagnostics: A/B of the queue form)
#endif
  if (use_queue && queue != nullptr && kq != nullptr && !a.window_mode) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kq, 64 * var->G, lds) !=
        hipSuccess) {
      (void)hipGetLastError();
      per_cu = 0;
    }
    const int64_t resident = (int64_t)per_cu * (p->cus > 0 ? p->cus : 0);
    if (resident > 0 && blocks > resident) {
      hipError_t e = hipMemsetAsync(queue, 0, sizeof(int), s);
      if (e != hipSuccess) return e;
      grid = resident;
      k = kq;
      a.queue = queue;
      a.qblock0 = resident;
      a.nblocks = blocks;
    }
  }
#ifdef ZMPC_DIAG
  static unsigned long long* prof = [] {  // diagnostics build: per-phase clocks to stderr
    unsigned long long* q = nullptr;
    if (getenv("ZMPC_LQ_PROF") && hipMalloc((void**)&q, 22 * sizeof(unsigned long long)) != hipSuccess)
      q = nullptr;
    return q;
  }();
  if (prof) (void)hipMemsetAsync(prof, 0, 22 * sizeof(unsigned long long), s);
  a.prof = prof;
  a.skip_axis = getenv("ZMPC_LQ_SKIP") ? atoi(getenv("ZMPC_LQ_SKIP")) : 0;
#else
  a.prof = nullptr;
#endif
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(64 * var->G), lds, s, a,
                     (const double*)p->lqtab);
  hipError_t e = hipGetLastError();
  if (a.prof && e == hipSuccess) {
    unsigned long long h[22];
    (void)hipMemcpy(h, a.prof, sizeof(h), hipMemcpyDeviceToHost);
    for (int ax = 0; ax < 2; ++ax) {
      const unsigned long long* c = h + 11 * ax;
      const double t = (double)(c[8] ? c[8] : 1), nt = (double)(c[10] ? c[10] : 1);
      fprintf(stderr,
              "lq prof axis %d: %llu tasks, %.0f clocks/task: sweep A tail %.3f, sweep A "
              "working-set %.3f; sweep B working-set: set-up + checkpoint wait %.3f (segment 1 "
              "%.3f), Riccati %.3f, forward %.3f, costate %.3f; sweep B tail %.3f; rest %.3f\n",
              ax, c[10], t / nt, c[0] / t, c[1] / t, c[2] / t, c[9] / t, c[4] / t, c[5] / t,
              c[6] / t, c[7] / t, c[3] / t);
    }
  }
  return e;
}

}  // namespace

hipError_t zmpc_strict_lq_set_attrs() {
  hipError_t e = hipSuccess;
  for (const LqVariant& c : kLqVariants)
    for (auto k : {c.kernel, c.kernel_nt, c.kernel_runs, c.kernel_runs_nt, c.q_kernel,
                   c.q_kernel_nt, c.q_kernel_runs, c.q_kernel_runs_nt})
      if (k != nullptr && e == hipSuccess)
        e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
  return e;
}

bool zmpc_strict_lq_supported(const zmpc_plan* p) {
  return p->N >= 1 && p->N <= ZMPC_STRICT_MAX_N && p->lqtab != nullptr &&
         lq_variant_for(p->N) != nullptr;
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
  a.rows = n + (int64_t)a.NS * LQ_S;  // the last segment reads up to NS·S − 1 ahead
  const LqVariant* var = lq_variant_for(p->N);
  if (!var) return hipErrorInvalidValue;
  const int64_t G = var->G;  // checkpoints for every wave of the launched blocks
  const size_t ck_doubles = (size_t)((waves + G - 1) / G * G) * a.NS * kCkStride;
  // bounds: rows (2 axes × rows × 64 (z_ref, half-width)) or runs (per (axis, group) up to
  // n + 2 runs of a pair and a start time).  ZMPC_OPT_STRICT_BOUNDS 0 (auto) = runs
  // (profiles/r4/r4e_*: config 3 71.8 → 64.3 ms with runs, L2 fetch 122 → 24 GB per launch).
  // A shared CoP's rows stay in L2, and round 4 kept rows for it (80.5 ms rows, 87.1 runs);
  // with the per-segment crossing test the runs are faster there too (config 4 64.0–64.4 vs
  // 65.5–66.1 ms, profiles/r5l/).
  const int bopt = p->opt[ZMPC_OPT_STRICT_BOUNDS];
  const bool runs = bopt != 1;
  a.rstride = (n + 2) * 64;
  const size_t st_doubles = runs ? (size_t)2 * a.groups * a.rstride * 3
                                 : (size_t)2 * a.groups * a.rows * 64 * 2;
  // kick order (order.hip): walks with per-walk kicks sorted by (kick step, kick) onto lanes,
  // when there is more than one wave of them (ZMPC_OPT_KICK_ORDER = 0 keeps the input order)
  const bool ordered = p->opt[ZMPC_OPT_KICK_ORDER] != 0 && kick != nullptr && B > 64;
  const size_t perm_doubles = ordered ? ((size_t)B * 4 + 7) / 8 : 0;
  const size_t ord_doubles = ordered ? (zmpc_kick_order_bytes(B) + 7) / 8 : 0;
  double* ws = nullptr;
  if (hipMallocAsync((void**)&ws,
                     (ck_doubles + st_doubles + perm_doubles + ord_doubles + 1) * sizeof(double),
                     s) != hipSuccess) {
    (void)hipGetLastError();
    return hipErrorOutOfMemory;  // ZMPC_ENOMEM at the C-ABI
  }
  a.ck = ws;
  a.queue = reinterpret_cast<int*>(ws + ck_doubles + st_doubles + perm_doubles + ord_doubles);
  double2* hl = reinterpret_cast<double2*>(ws + ck_doubles);
  a.perm = nullptr;
  if (ordered) {
    int32_t* perm = reinterpret_cast<int32_t*>(ws + ck_doubles + st_doubles);
    e = zmpc_kick_order(kick, kick_steps, kick_step, B, perm,
                        ws + ck_doubles + st_doubles + perm_doubles, s);
    a.perm = perm;
  }
  if (e == hipSuccess) {
    const int32_t* perm = a.shared ? nullptr : a.perm;
    if (runs) {
      a.rs = hl;
      a.rt = reinterpret_cast<int*>(hl + 2 * a.groups * a.rstride);
      e = stage_runs(zmax, zmin, bstride, 2, 1, n, Bst, 2, hl, const_cast<int*>(a.rt), a.rstride,
                     s, perm);
    } else {
      e = stage(zmax, zmin, bstride, 2, 1, n, Bst, a.rows, 2, hl, s, perm);
      a.hl = hl;
    }
  }
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
  a.rows = (int64_t)a.NS * LQ_S;
  const int64_t waves = (B + 63) / 64;
  const LqVariant* var = lq_variant_for(p->N);
  if (!var) return hipErrorInvalidValue;
  const int64_t G = var->G;  // checkpoints for every wave of the launched blocks
  const size_t ck_doubles = (size_t)((waves + G - 1) / G * G) * a.NS * kCkStride;
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
