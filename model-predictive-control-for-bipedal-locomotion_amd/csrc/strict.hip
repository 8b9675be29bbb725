// Strict (ZMP box-constrained) Wieber QP on the device (config.strict == True).
//
// Reference, per axis and timestep (zmp_controller.py:173-195, solved there by cvxpy→OSQP):
//   min_J ½Q‖Px x + Pu J − z_ref‖² + ½R‖J‖²   s.t.  z_min ≤ Px x + Pu J ≤ z_max,  u0 = J[0]
// Pu is lower-triangular Toeplitz with p(0) ≠ 0, hence invertible: in ZMP coordinates
// z = Px x + Pu J the constraints are simple bounds and the problem is a strictly convex
// box-QP, always feasible.  With c = Px x, W = Q (z_ref − c), the plan's
// G = Pu (R·I + Q·PuᵀPu)⁻¹ Puᵀ (inverse z-space Hessian) and H = G⁻¹ = Q I + R Pu⁻ᵀPu⁻¹,
// everything relative to c (δ = z − c, t = bound − c):
//   unconstrained   δ* = D = G W
//   dual side       (|A| <= |F|)  G_AA ν_A = D_A − t_A,   δ = D − G_{:,A} ν_A
//   primal side     (|A| >  |F|)  H_FF δ_F = W_F − H_FA t_A,  δ_A = t_A,  ν_A = W_A − (H δ)_A
//   KKT             ν ≥ 0 on upper-active, ν ≤ 0 on lower-active, t_lo ≤ δ ≤ t_hi on free
//   first jerk      u0 = δ_0 / p(0)
// The active set comes from a primal-dual active-set iteration warm-started with the previous
// timestep's set shifted one horizon slot (the rollout's windows slide by one).
//
// Mapping: a workgroup (4 waves) owns a tile of 16 instances (instance = walk × axis) for the
// whole rollout, persistent over tiles.  Per timestep:
//   GEMM   D[:, 16 instances] = G · W: v_mfma_f64_16x16x4_f64, G streamed from L2 (batch-
//          invariant) with the next k-group's loads in flight under the current MFMAs;
//   solve  each wave takes 4 instances: PDAS with the reduced Cholesky factor packed in LDS
//          (lane-blocked 8×8 updates, LDS-only ordering), G/H row combinations as coalesced,
//          4-row-deep pipelined loads; state advance, kick, history, next W.
#include <cstdio>
#include <cstdlib>

#include "zmpc_internal.h"

namespace {

typedef double dbl4 __attribute__((ext_vector_type(4)));

constexpr int SNB = 16;            // instances per tile (= MFMA column tile)
constexpr int SWAVES = 4;          // waves per workgroup
constexpr int SPW = SNB / SWAVES;  // instances per wave
constexpr int SMAXIT = 1024;       // PDAS iteration cap (as strict_lq.hip)

struct StrictArgs {
  int N, Np, ld;         // horizon, padded to 16, W/D leading dimension
  int pcap;              // LDS doubles for the packed reduced factor (per wave)
  int window_mode;       // 0 = rollout over [B,n,2] bounds, 1 = single step on [B,N] windows
  int64_t n;             // samples per walk (rollout)
  int64_t bstride;       // doubles between walks' bound arrays (0 = shared CoP)
  int64_t ninst;         // instances: 2B (rollout) or B (step)
  double Q, p0, hg;
  LipmConsts lc;
  const double* G;       // [N,N] inverse z-space Hessian
  const double* Hz;      // [N,N] z-space Hessian Q I + R Pu⁻ᵀPu⁻¹
  const double* zmax;
  const double* zmin;
  const double* x0;      // rollout [B,2,3], step [B,3]
  const double* kick;    // [B] or null
  int64_t kick_step;
  const int64_t* kick_steps;  // [B] per-walk kick steps, or null
  double* out;           // rollout hist [B,n,2,3], step x_next [B,3]
  int32_t* status;       // [B] or null
  double* scratch;       // per-wave factor scratch, sg_stride doubles each (gridDim*SWAVES slots)
  int64_t sg_stride;     // (N/2 + 1)²: the reduced system is min(|A|, |F|) <= N/2
  unsigned long long* dbg;  // diagnostic phase counters (ZMPC_DEBUG_STRICT), null normally
  int lds_chol;          // A/B: 1 = LDS Cholesky for every reduced size (ZMPC_STRICT_LDS_CHOL)
  int gsz;               // doubles of LDS holding G packed (0: G read from L2)
};

// Diagnostic phase timer: only when a.dbg is set (a separate, opt-in run; never in the bench).
struct PhaseClock {
  unsigned long long* dbg;
  unsigned long long t;
  __device__ explicit PhaseClock(unsigned long long* d)
      : dbg(d), t(d ? __builtin_amdgcn_s_memtime() : 0) {}
  __device__ void lap(int slot, int lane) {
    if (!dbg) return;
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    if (lane == 0) atomicAdd(dbg + slot, now - t);
    t = now;
  }
  __device__ void count(int slot, unsigned long long v, int lane) {
    if (dbg && lane == 0) atomicAdd(dbg + slot, v);
  }
};

// Orders this wave's global and LDS accesses (waits for both counters).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  __builtin_amdgcn_wave_barrier();
}
// Orders this wave's LDS accesses only: DS instructions of one wave execute in order, so a
// compiler barrier is all a cross-lane LDS hand-off inside the wave needs.
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void lipm_step(const LipmConsts& c, const double* x, double u,
                                          double* y) {
  y[0] = x[0] + c.T * x[1] + c.T2_2 * x[2] + c.T3_6 * u;
  y[1] = x[1] + c.T * x[2] + c.T2_2 * u;
  y[2] = x[2] + c.T * u;
}

// c_j = Px[j]·x with Px[j] = [1, T(j+1), T²/2 (j+1)² − h/g] evaluated as the plan (and the
// reference, zmp_controller.py:167-169) evaluates it.
__device__ __forceinline__ double px_dot(const StrictArgs& a, int j, const double* x) {
#pragma clang fp contract(off)
  const long long q = j + 1;
  const double p1 = a.lc.T * (double)q;
  const double p2 = a.lc.T2_2 * (double)(q * q) - a.hg;
  return x[0] + p1 * x[1] + p2 * x[2];
}

// Window element j of instance `inst` at timestep i (rows i+1.., padded with the last row,
// zmp_controller.py:81-88,97-98).
__device__ __forceinline__ int64_t bound_index(const StrictArgs& a, int64_t inst, int64_t i,
                                               int j) {
  if (a.window_mode) return inst * a.N + j;
  const int64_t b = inst >> 1, axis = inst & 1;
  int64_t t = i + 1 + j;
  if (t > a.n - 1) t = a.n - 1;
  return b * a.bstride + t * 2 + axis;
}

// W[j] = Q (z_ref_j − c_j); zero on the padding rows.
template <int NJ>
__device__ void build_w(const StrictArgs& a, int64_t inst, int64_t i, const double* x,
                        double* W, int lane) {
  double hi[NJ], lo[NJ];
#pragma unroll
  for (int c = 0; c < NJ; ++c) {
    const int j = lane + 64 * c;
    if (j < a.N) {
      const int64_t e = bound_index(a, inst, i, j);
      hi[c] = a.zmax[e];
      lo[c] = a.zmin[e];
    }
  }
#pragma unroll
  for (int c = 0; c < NJ; ++c) {
    const int j = lane + 64 * c;
    if (j < a.N) W[j] = a.Q * ((hi[c] + lo[c]) / 2 - px_dot(a, j, x));
  }
  for (int j = a.N + lane; j < a.Np; j += 64) W[j] = 0.0;
}

// Reduced-system factor storage: packed lower triangle in LDS (i(i+1)/2 + j) or a dense
// m×m block in the wave's global scratch when it does not fit.
template <bool PACKED>
struct Tri {
  double* S;
  int m;
  __device__ __forceinline__ double& at(int i, int j) const {
    return PACKED ? S[(i * (i + 1) >> 1) + j] : S[i * m + j];
  }
  __device__ __forceinline__ void sync() const {
    if (PACKED)
      lds_sync();
    else
      wave_sync();
  }
};

// In-place lower Cholesky of the SPD m×m matrix held in T (lower part), by one wave.  The
// trailing update walks 8×8 blocks of the lower triangle (lane = (row, col) in the block),
// so each column step costs ⌈r/8⌉(⌈r/8⌉+1)/2 wave instructions for r trailing rows.
// Returns false if a pivot is not positive.
template <bool PACKED>
__device__ bool wave_cholesky(const Tri<PACKED>& T, int lane) {
  const int m = T.m;
  const int li = lane >> 3, lj = lane & 7;
  for (int k = 0; k < m; ++k) {
    const double d = T.at(k, k);
    if (!(d > 0.0)) return false;
    const double piv = sqrt(d);
    const double inv = 1.0 / piv;
    T.sync();
    for (int i = k + 1 + lane; i < m; i += 64) T.at(i, k) *= inv;
    if (lane == 0) T.at(k, k) = piv;
    T.sync();
    const int r = m - k - 1;
    const int nb = (r + 7) >> 3;
    for (int bi = 0; bi < nb; ++bi) {
      const int i = k + 1 + 8 * bi + li;
      const double lik = (i < m) ? T.at(i, k) : 0.0;
      for (int bj = 0; bj <= bi; ++bj) {
        const int j = k + 1 + 8 * bj + lj;
        if (i < m && j <= i) T.at(i, j) -= lik * T.at(j, k);
      }
    }
    T.sync();
  }
  return true;
}

// Solve (L Lᵀ) v = rhs in place (rhs in v, LDS), L from wave_cholesky.
template <bool PACKED>
__device__ void wave_chol_solve(const Tri<PACKED>& T, double* v, int lane) {
  const int m = T.m;
  for (int j = 0; j < m; ++j) {
    const double yj = v[j] / T.at(j, j);
    T.sync();
    for (int i = j + 1 + lane; i < m; i += 64) v[i] -= T.at(i, j) * yj;
    if (lane == 0) v[j] = yj;
    T.sync();
  }
  for (int j = m - 1; j >= 0; --j) {
    const double yj = v[j] / T.at(j, j);
    T.sync();
    for (int i = lane; i < j; i += 64) v[i] -= T.at(j, i) * yj;
    if (lane == 0) v[j] = yj;
    T.sync();
  }
}

struct WaveWork {
  double* zz;    // [Np] current δ
  double* nuf;   // [Np] multipliers scattered to horizon slots
  double* nuc;   // [Np] compact right-hand side / solution
  double* rj;    // [Np] per-slot scratch read across lanes (dual rhs, primal W − H t)
  int* ia;       // [Np] compact active slots
  int* iff;      // [Np] compact free slots
  double* S;     // LDS factor workspace (pcap doubles)
  double* Sg;    // [N*N] global factor scratch
  const double* Gs;  // G packed lower-triangular in LDS (N(N+1)/2), or null (G from L2)
};

__device__ __forceinline__ int tri_at(int i, int j) { return ((i * (i + 1)) >> 1) + j; }

// G(r, c) from the LDS copy (symmetric, packed lower) or from global memory.
__device__ __forceinline__ double g_at(const StrictArgs& a, const WaveWork& w, int r, int c) {
  if (w.Gs) return w.Gs[r >= c ? tri_at(r, c) : tri_at(c, r)];
  return a.G[(size_t)r * a.N + c];
}

// acc[c] −= Σ_r M[idx[r]][j_c] · coef[r] for the lane's horizon slots j_c = lane + 64c:
// one coalesced row load per (r, c); four rows in flight per round.  (Global M.)
template <int NJ>
__device__ __forceinline__ void row_combine(const double* M, int N, const int* idx,
                                            const double* coef, int count, double* acc,
                                            int lane) {
  // RB rows (RB·NJ loads) in flight per round: the rows come from L2 at ~2k-cycle latency
  // and one wave per SIMD has nothing else to hide it with
  constexpr int RB = (NJ <= 3) ? 8 : 4;
  int r0 = 0;
  for (; r0 + RB <= count; r0 += RB) {
    double g[RB][NJ];
    double cf[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const double* row = M + (size_t)idx[r0 + u] * N;
      cf[u] = coef[r0 + u];
#pragma unroll
      for (int c = 0; c < NJ; ++c) {
        const int j = lane + 64 * c;
        g[u][c] = row[j < N ? j : 0];
      }
    }
#pragma unroll
    for (int u = 0; u < RB; ++u)
#pragma unroll
      for (int c = 0; c < NJ; ++c) acc[c] = fma(-g[u][c], cf[u], acc[c]);
  }
  for (; r0 < count; ++r0) {
    const double* row = M + (size_t)idx[r0] * N;
    const double cf = coef[r0];
#pragma unroll
    for (int c = 0; c < NJ; ++c) {
      const int j = lane + 64 * c;
      if (j < N) acc[c] = fma(-row[j], cf, acc[c]);
    }
  }
}

// The same with G's packed LDS copy (rows of a symmetric matrix: G[r][j] = Gs[tri(max, min)]).
template <int NJ>
__device__ __forceinline__ void row_combine_lds(const double* Gs, int N, const int* idx,
                                                const double* coef, int count, double* acc,
                                                int lane) {
  for (int r = 0; r < count; ++r) {
    const int ir = idx[r];
    const double cf = coef[r];
#pragma unroll
    for (int c = 0; c < NJ; ++c) {
      const int j = lane + 64 * c;
      if (j < N) acc[c] = fma(-Gs[j <= ir ? tri_at(ir, j) : tri_at(j, ir)], cf, acc[c]);
    }
  }
}

// Gather the reduced matrix (gather(r, c), r >= c) into the packed LDS factor, 8×8 lane
// blocks, every load of a block row in flight before its stores.
template <class Gather>
__device__ __forceinline__ void gather_packed(const Tri<true>& T, Gather gather, int lane) {
  const int m = T.m;
  const int nb = (m + 7) >> 3;
  const int li = lane >> 3, lj = lane & 7;
  constexpr int kMaxNb = 16;  // m <= 128
  for (int bi = 0; bi < nb; ++bi) {
    const int r = 8 * bi + li;
    double v[kMaxNb];
#pragma unroll
    for (int bj = 0; bj < kMaxNb; ++bj) {
      const int c = 8 * bj + lj;
      if (bj <= bi && r < m && c <= r) v[bj] = gather(r, c);
    }
#pragma unroll
    for (int bj = 0; bj < kMaxNb; ++bj) {
      const int c = 8 * bj + lj;
      if (bj <= bi && r < m && c <= r) T.at(r, c) = v[bj];
    }
  }
}

// ---- register-resident reduced solve (m <= 64) ------------------------------------------
// Lane i < m owns row i of the trailing matrix: at column step k, a[j] = element (i, k + j)
// (the array shifts one slot per column, so every register index is static in a rolled
// k-loop).  Column k is broadcast with v_readlane (wave-uniform lane index): a column costs
// MR FMAs + 2·MR readlanes per lane and no memory round trip.  The inner loops carry no
// guards (MR is the smallest of 16/32/48/64 covering m; entries past m stay 0), so they are
// straight-line code.  L's rows go to LDS (packed) for the two triangular solves, which chain
// through v_readlane.
__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Solve M_II y = rhs, M_II[r][c] = gather(r, c) (symmetric positive definite, r >= c asked),
// rhs in LDS (overwritten with y), Ls = LDS scratch of m(m+1)/2 doubles.  False if a pivot is
// not positive.
template <int MR, class Gather>
__device__ __noinline__ bool reg_chol_solve(Gather gather, int m, double* rhs, double* Ls, int lane) {
  double a[MR];
#pragma unroll
  for (int j = 0; j < MR; ++j) a[j] = (j < m && lane < m && j <= lane) ? gather(lane, j) : 0.0;
  double invd = 0.0;
  for (int k = 0; k < m; ++k) {
    const double d = readlane_d(a[0], k);
    if (!(d > 0.0)) return false;
    const double piv = sqrt(d);
    const double inv = 1.0 / piv;
    const double l = (lane == k) ? piv : ((lane > k && lane < m) ? a[0] * inv : 0.0);
    if (lane == k) invd = inv;
    if (lane >= k && lane < m) Ls[tri_at(lane, k)] = l;
#pragma unroll
    for (int j = 1; j < MR; ++j) a[j - 1] = fma(-l, readlane_d(l, (k + j) & 63), a[j]);
    a[MR - 1] = 0.0;
  }
  lds_sync();
  // forward L y = rhs
  double acc = (lane < m) ? rhs[lane] : 0.0;
  double y = 0.0;
  for (int j = 0; j < m; ++j) {
    const double lij = (lane > j && lane < m) ? Ls[tri_at(lane, j)] : 0.0;
    const double yj = readlane_d(acc * invd, j);
    if (lane == j) y = yj;
    acc = fma(-lij, yj, acc);
  }
  // backward Lᵀ x = y (column j of Lᵀ = row j of L)
  acc = y;
  double x = 0.0;
  for (int j = m - 1; j >= 0; --j) {
    const double lji = (lane < j) ? Ls[tri_at(j, lane)] : 0.0;
    const double xj = readlane_d(acc * invd, j);
    if (lane == j) x = xj;
    acc = fma(-lji, xj, acc);
  }
  lds_sync();
  if (lane < m) rhs[lane] = x;
  lds_sync();
  return true;
}

// Factor the reduced matrix gathered by `gather(r, c)` (size m) and solve in place on w.nuc:
// registers for m <= 32, the packed LDS factor while it fits, else the wave's global scratch.
template <class Gather>
__device__ __forceinline__ bool reduced_solve(const StrictArgs& a, const WaveWork& w, int m, Gather gather,
                              int lane) {
  PhaseClock clk(a.dbg);
  clk.count(12, m, lane);
  clk.count(m <= 16 ? 16 : m <= 32 ? 17 : m <= 48 ? 18 : m <= 64 ? 19 : 20, 1, lane);
  if (m <= 64 && m * (m + 1) / 2 <= a.pcap && !a.lds_chol) {
    const bool ok = m <= 16   ? reg_chol_solve<16>(gather, m, w.nuc, w.S, lane)
                    : m <= 32 ? reg_chol_solve<32>(gather, m, w.nuc, w.S, lane)
                    : m <= 48 ? reg_chol_solve<48>(gather, m, w.nuc, w.S, lane)
                              : reg_chol_solve<64>(gather, m, w.nuc, w.S, lane);
    clk.lap(3, lane);
    return ok;
  }
  if (m * (m + 1) / 2 <= a.pcap && m <= 128) {
    Tri<true> T{w.S, m};
    gather_packed(T, gather, lane);
    lds_sync();
    clk.lap(2, lane);
    if (!wave_cholesky(T, lane)) return false;
    clk.lap(3, lane);
    wave_chol_solve(T, w.nuc, lane);
    clk.lap(4, lane);
  } else {
    clk.count(14, 1, lane);
    Tri<false> T{w.Sg, m};
    for (int t = lane; t < m * m; t += 64) {
      const int r = t / m, c = t % m;
      if (c <= r) T.at(r, c) = gather(r, c);
    }
    wave_sync();
    if (!wave_cholesky(T, lane)) return false;
    wave_chol_solve(T, w.nuc, lane);
  }
  return true;
}

// One strict QP solve for one instance.  D holds G·W on entry; st is the instance's
// warm-start status array (0 free, 1 upper, 2 lower), updated in place.  Returns u0 and
// ORs failure flags into *flags.  The lane's own horizon slots (j = lane + 64c) keep D and
// the shifted bounds in registers; only what other lanes read goes through LDS.
template <int NJ>
__device__ __forceinline__ double solve_instance(const StrictArgs& a, int64_t inst, int64_t i, const double* x,
                                 const double* D, signed char* st, const WaveWork& w, int lane,
                                 int* flags) {
  const int N = a.N;
  PhaseClock clk(a.dbg);
  double zs[NJ], hi[NJ], lo[NJ];  // D, z_max − c, z_min − c on the lane's slots
  {
    double bh[NJ], bl[NJ];
#pragma unroll
    for (int c = 0; c < NJ; ++c) {
      const int j = lane + 64 * c;
      const int64_t e = bound_index(a, inst, i, j < N ? j : N - 1);
      bh[c] = a.zmax[e];
      bl[c] = a.zmin[e];
    }
#pragma unroll
    for (int c = 0; c < NJ; ++c) {
      const int j = lane + 64 * c;
      zs[c] = hi[c] = lo[c] = 0.0;
      if (j < N) {
        const double cj = px_dot(a, j, x);
        hi[c] = bh[c] - cj;
        lo[c] = bl[c] - cj;
        zs[c] = D[j];
        w.zz[j] = zs[c];
        w.nuf[j] = 0.0;
      }
    }
  }
  lds_sync();
  clk.lap(0, lane);
  clk.count(11, 1, lane);
  const double tolz = 1e-13, tolnu = 1e-13;
  bool done = false;
  for (int it = 0; it < SMAXIT; ++it) {
    clk.count(9, 1, lane);
    // compact the active and the free slots
    int m = 0, f = 0;
#pragma unroll
    for (int c = 0; c < NJ; ++c) {
      const int j = lane + 64 * c;
      const bool act = (j < N) && st[j] != 0;
      const bool fre = (j < N) && st[j] == 0;
      const unsigned long long ba = __ballot(act), bf = __ballot(fre);
      const unsigned long long below = (1ull << lane) - 1ull;
      if (act) w.ia[m + __popcll(ba & below)] = j;
      if (fre) w.iff[f + __popcll(bf & below)] = j;
      m += __popcll(ba);
      f += __popcll(bf);
    }
    lds_sync();
    clk.lap(1, lane);
    clk.count(10, m, lane);
    if (m > f) clk.count(13, 1, lane);
    if (m == 0) {
#pragma unroll
      for (int c = 0; c < NJ; ++c) {
        const int j = lane + 64 * c;
        if (j < N) {
          w.zz[j] = zs[c];
          w.nuf[j] = 0.0;
        }
      }
    } else if (m <= f) {
      // dual: G_AA ν = D_A − t_A
#pragma unroll
      for (int c = 0; c < NJ; ++c) {
        const int j = lane + 64 * c;
        if (j < N && st[j] != 0) w.rj[j] = zs[c] - (st[j] == 1 ? hi[c] : lo[c]);
      }
      lds_sync();
      for (int r = lane; r < m; r += 64) w.nuc[r] = w.rj[w.ia[r]];
      lds_sync();
      const int* ia = w.ia;
      if (!reduced_solve(a, w, m, [&](int r, int c) { return g_at(a, w, ia[r], ia[c]); },
                         lane)) {
        *flags |= ZMPC_ST_FACTOR;
        break;
      }
      // δ = D − G_{:,A} ν_A   (G symmetric: row ia_r is column ia_r)
      double acc[NJ];
#pragma unroll
      for (int c = 0; c < NJ; ++c) {
        const int j = lane + 64 * c;
        acc[c] = zs[c];
        if (j < N) w.nuf[j] = 0.0;
      }
      lds_sync();
      for (int r = lane; r < m; r += 64) w.nuf[w.ia[r]] = w.nuc[r];
      if (w.Gs)
        row_combine_lds<NJ>(w.Gs, N, w.ia, w.nuc, m, acc, lane);
      else
        row_combine<NJ>(a.G, N, w.ia, w.nuc, m, acc, lane);
#pragma unroll
      for (int c = 0; c < NJ; ++c) {
        const int j = lane + 64 * c;
        if (j < N) w.zz[j] = acc[c];
      }
    } else {
      // primal: H_FF δ_F = W_F − (H t_A)_F,  ν_A = W_A − (H δ)_A
      double y[NJ];
#pragma unroll
      for (int c = 0; c < NJ; ++c) {
        const int j = lane + 64 * c;
        y[c] = 0.0;
        if (j < N) w.zz[j] = (st[j] == 1) ? hi[c] : ((st[j] == 2) ? lo[c] : 0.0);
      }
      lds_sync();
      for (int r = lane; r < m; r += 64) w.nuc[r] = -w.zz[w.ia[r]];
      lds_sync();
      row_combine<NJ>(a.Hz, N, w.ia, w.nuc, m, y, lane);  // y = H t_A (scattered)
      // W_j − y_j for every slot (W = Q (z_ref − c) = Q (hi + lo) / 2)
      double wy[NJ];
#pragma unroll
      for (int c = 0; c < NJ; ++c) {
        const int j = lane + 64 * c;
        wy[c] = a.Q * ((hi[c] + lo[c]) / 2) - y[c];
        if (j < N) w.rj[j] = wy[c];
      }
      lds_sync();
      for (int r = lane; r < f; r += 64) w.nuc[r] = w.rj[w.iff[r]];
      lds_sync();
      const int* iff = w.iff;
      const double* H = a.Hz;
      if (f > 0 &&
          !reduced_solve(a, w, f, [&](int r, int c) { return H[(size_t)iff[r] * N + iff[c]]; },
                         lane)) {
        *flags |= ZMPC_ST_FACTOR;
        break;
      }
      for (int r = lane; r < f; r += 64) w.zz[w.iff[r]] = w.nuc[r];
      // ν_A = (W − H t_A)_A − (H_{:,F} δ_F)_A ; 0 on the free slots
      double v2[NJ];
#pragma unroll
      for (int c = 0; c < NJ; ++c) v2[c] = 0.0;
      for (int r = lane; r < f; r += 64) w.nuc[r] = -w.nuc[r];
      lds_sync();
      row_combine<NJ>(a.Hz, N, w.iff, w.nuc, f, v2, lane);
#pragma unroll
      for (int c = 0; c < NJ; ++c) {
        const int j = lane + 64 * c;
        if (j < N) w.nuf[j] = (st[j] != 0) ? (wy[c] - v2[c]) : 0.0;
      }
    }
    lds_sync();
    clk.lap(5, lane);
    // primal-dual set update: release active slots with wrong-signed multipliers, activate
    // violated free slots
    signed char ns[NJ];
    bool changed = false;
#pragma unroll
    for (int c = 0; c < NJ; ++c) {
      const int j = lane + 64 * c;
      ns[c] = 0;
      if (j < N) {
        const signed char o = st[j];
        signed char v = o;
        const double zj = w.zz[j], nj = w.nuf[j];
        if (o == 1) {
          if (nj < -tolnu) v = 0;
        } else if (o == 2) {
          if (nj > tolnu) v = 0;
        } else if (zj > hi[c] + tolz) {
          v = 1;
        } else if (zj < lo[c] - tolz) {
          v = 2;
        }
        ns[c] = v;
        changed |= (v != o);
      }
    }
    changed = __any(changed);
    clk.lap(6, lane);
    if (!changed) {
      done = true;
      break;
    }
#pragma unroll
    for (int c = 0; c < NJ; ++c) {
      const int j = lane + 64 * c;
      if (j < N) st[j] = ns[c];
    }
    lds_sync();
  }
  if (!done) *flags |= ZMPC_ST_MAXITER;
  const double u0 = w.zz[0] / a.p0;
  lds_sync();
  return u0;
}

// D[:, 16 instances] = M · Win for the row tiles rt = wave + 4t (t < NJ) of one wave;
// results returned in acc (MFMA D layout: col = lane&15, row = (lane>>4) + 4q).
// The next k-group's M loads are issued before the current group's MFMAs.
template <int NJ>
__device__ __forceinline__ void tile_gemm(const double* __restrict__ M, int N, int Np,
                                          const double* Win, int ld, int wave, int lane,
                                          dbl4* acc) {
  const int r = lane & 15, kq = lane >> 4;
  const int nrt = Np >> 4;
  const double* rows[NJ];
  bool ok[NJ];
#pragma unroll
  for (int t = 0; t < NJ; ++t) {
    acc[t] = dbl4{0.0, 0.0, 0.0, 0.0};
    const int rt = wave + SWAVES * t;
    const int row = rt * 16 + r;
    ok[t] = (rt < nrt) && (row < N);
    rows[t] = M + (ok[t] ? row : 0);
  }
  double gc[NJ][4], gn[NJ][4];
  auto load_group = [&](int k0, double (&g)[NJ][4]) {
#pragma unroll
    for (int t = 0; t < NJ; ++t)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + 4 * u + kq;
        g[t][u] = (ok[t] && k < N) ? rows[t][(size_t)k * N] : 0.0;
      }
  };
  load_group(0, gc);
  for (int k0 = 0; k0 < Np; k0 += 16) {
    if (k0 + 16 < Np) load_group(k0 + 16, gn);
    double wv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) wv[u] = Win[r * ld + k0 + 4 * u + kq];
#pragma unroll
    for (int t = 0; t < NJ; ++t) {
      if (wave + SWAVES * t < nrt) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(gc[t][u], wv[u], acc[t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < NJ; ++t)
#pragma unroll
      for (int u = 0; u < 4; ++u) gc[t][u] = gn[t][u];
  }
}

template <int NJ>
__global__ void __launch_bounds__(256) zmpc_strict_kernel(StrictArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int Np = a.Np, ld = a.ld;
  // LDS carve: Gs [gsz] (G packed lower, when it fits) | Wt [SNB][ld] | xs [SNB][4] |
  //            flags [SNB] (as doubles) | per wave {zz,nuf,nuc,rj}[Np], ia/iff[Np] ints,
  //            S[pcap] | st [SNB][Np] B
  double* Gs = smem;
  double* Wt = Gs + a.gsz;
  double* xs = Wt + SNB * ld;
  int* fl = reinterpret_cast<int*>(xs + SNB * 4);
  double* wbase = xs + SNB * 4 + SNB;
  const int per_wave = 5 * Np + a.pcap;
  double* my = wbase + wave * per_wave;
  WaveWork w;
  w.zz = my;
  w.nuf = my + Np;
  w.nuc = my + 2 * Np;
  w.rj = my + 3 * Np;
  w.ia = reinterpret_cast<int*>(my + 4 * Np);
  w.iff = w.ia + Np;
  w.S = my + 5 * Np;
  w.Sg = a.scratch + ((size_t)blockIdx.x * SWAVES + wave) * (size_t)a.sg_stride;
  w.Gs = nullptr;
  if (a.gsz > 0) {
    // G (symmetric, batch-invariant) packed into LDS once per workgroup: every reduced-matrix
    // gather and row combination of the active-set solves then reads LDS, not L2
    for (int r = wave; r < a.N; r += SWAVES)
      for (int c = lane; c <= r; c += 64) Gs[tri_at(r, c)] = a.G[(size_t)r * a.N + c];
    w.Gs = Gs;
    __syncthreads();
  }
  signed char* stall = reinterpret_cast<signed char*>(wbase + SWAVES * per_wave);

  const int64_t ntiles = (a.ninst + SNB - 1) / SNB;
  const int64_t nsteps = a.window_mode ? 1 : a.n - 1;
  const int nrt = Np / 16;

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // ---- tile setup: states, warm-start sets, first W --------------------------------
    for (int q = 0; q < SPW; ++q) {
      const int s = wave * SPW + q;
      const int64_t inst = tile * SNB + s;
      double* x = xs + s * 4;
      signed char* st = stall + s * Np;
      for (int j = lane; j < Np; j += 64) st[j] = 0;
      if (lane == 0) fl[s] = 0;
      if (lane < 3) x[lane] = (inst < a.ninst) ? a.x0[inst * 3 + lane] : 0.0;
      wave_sync();
      if (!a.window_mode && inst < a.ninst && lane < 3) {
        // hist[b, 0, axis, :] = x0
        a.out[((inst >> 1) * a.n * 2 + (inst & 1)) * 3 + lane] = x[lane];
      }
      if (inst < a.ninst) {
        const double xv[3] = {x[0], x[1], x[2]};
        build_w<NJ>(a, inst, 0, xv, Wt + s * ld, lane);
      } else {
        for (int j = lane; j < ld; j += 64) Wt[s * ld + j] = 0.0;
      }
    }
    __syncthreads();

    for (int64_t i = 0; i < nsteps; ++i) {
      PhaseClock kclk(a.dbg);
      // ---- GEMM: D = G · W for the 16 instances of the tile (MFMA f64) ----------------
      dbl4 acc[NJ];
      tile_gemm<NJ>(a.G, a.N, Np, Wt, ld, wave, lane, acc);
      __syncthreads();
#pragma unroll
      for (int t = 0; t < NJ; ++t) {
        const int rt = wave + SWAVES * t;
        if (rt < nrt) {
          const int col = lane & 15;
#pragma unroll
          for (int q = 0; q < 4; ++q) Wt[col * ld + rt * 16 + (lane >> 4) + 4 * q] = acc[t][q];
        }
      }
      __syncthreads();
      kclk.lap(7, lane);

      // ---- per-instance active set, state advance, next W ------------------------------
      for (int q = 0; q < SPW; ++q) {
        const int s = wave * SPW + q;
        const int64_t inst = tile * SNB + s;
        if (inst >= a.ninst) continue;
        double* x = xs + s * 4;
        signed char* st = stall + s * Np;
        const double xv[3] = {x[0], x[1], x[2]};
        // warm start: shift the previous set one slot towards the present
        if (i > 0) {
          signed char v[NJ];
#pragma unroll
          for (int c = 0; c < NJ; ++c) {
            const int j = lane + 64 * c;
            v[c] = (j + 1 < a.N) ? st[j + 1] : ((j < a.N) ? st[j] : 0);
          }
          lds_sync();
#pragma unroll
          for (int c = 0; c < NJ; ++c)
            if (lane + 64 * c < a.N) st[lane + 64 * c] = v[c];
          lds_sync();
        }
        int fq = 0;
        const double u0 = solve_instance<NJ>(a, inst, i, xv, Wt + s * ld, st, w, lane, &fq);
        double xn[3];
        lipm_step(a.lc, xv, u0, xn);
        if (!a.window_mode && (inst & 1) && a.kick != nullptr &&
            i == (a.kick_steps ? a.kick_steps[inst >> 1] : a.kick_step))
          xn[1] -= a.kick[inst >> 1];
        if (!(isfinite(xn[0]) && isfinite(xn[1]) && isfinite(xn[2]))) fq |= ZMPC_ST_NONFINITE;
        if (lane == 0) fl[s] |= fq;
        lds_sync();
        if (lane < 3) x[lane] = xn[lane];
        if (a.window_mode) {
          if (lane < 3) a.out[inst * 3 + lane] = xn[lane];
        } else if (lane < 3) {
          a.out[(((inst >> 1) * a.n + i + 1) * 2 + (inst & 1)) * 3 + lane] = xn[lane];
        }
        lds_sync();
        if (i + 1 < nsteps) build_w<NJ>(a, inst, i + 1, xn, Wt + s * ld, lane);
      }
      kclk.lap(8, lane);
      __syncthreads();
      kclk.lap(15, lane);
    }
    // ---- status: OR over the axes of a walk -------------------------------------------
    if (a.status != nullptr) {
      for (int q = 0; q < SPW; ++q) {
        const int s = wave * SPW + q;
        const int64_t inst = tile * SNB + s;
        if (inst < a.ninst && lane == 0) {
          if (a.window_mode)
            a.status[inst] = fl[s];
          else if (fl[s] != 0)
            atomicOr(&a.status[inst >> 1], fl[s]);
        }
      }
    }
    __syncthreads();
  }
}

// ---- small batches: one instance per wavefront (north_star's mapping) -------------------------
// The tile kernel above amortises the unconstrained solution over 16 instances with an MFMA GEMM;
// with a handful of walks (the drop-in's single walk) most of those columns are empty and every
// timestep pays the GEMM's and the gathers' L2 round trips.  Here a wave owns one instance
// (walk, axis) for the whole rollout and a workgroup's waves share nothing but G, packed into LDS
// once per workgroup (the lower triangle, N(N+1)/2 doubles: 90 KB at N = 150), so the
// unconstrained solve D = G·W (each lane its horizon slots j = lane + 64c, G's row/column from
// LDS), the reduced-matrix gathers and the row combinations of the active-set passes
// (solve_instance, shared with the tile kernel) are LDS reads.  Same primal-dual active-set
// iteration and warm start as the tile kernel and the LQ kernel: the same sets and solutions.
constexpr int WWAVES = 4;  // instances (waves) per workgroup of the wave kernel

template <int NJ>
__global__ void __launch_bounds__(64 * WWAVES) zmpc_strict_wave_kernel(StrictArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int N = a.N, Np = a.Np;
  // LDS carve: Gs [gsz] | per wave {W, zz, nuf, nuc, rj [Np], ia/iff [Np] ints, S [pcap],
  //            x [4]} | st [WWAVES][Np] bytes
  double* Gs = smem;
  const int per_wave = 6 * Np + a.pcap + 4;
  double* my = Gs + a.gsz + wave * per_wave;
  double* W = my;
  WaveWork w;
  w.zz = my + Np;
  w.nuf = my + 2 * Np;
  w.nuc = my + 3 * Np;
  w.rj = my + 4 * Np;
  w.ia = reinterpret_cast<int*>(my + 5 * Np);
  w.iff = w.ia + Np;
  w.S = my + 6 * Np;
  double* xs = w.S + a.pcap;
  w.Sg = a.scratch + ((size_t)blockIdx.x * WWAVES + wave) * (size_t)a.sg_stride;
  w.Gs = nullptr;
  signed char* st = reinterpret_cast<signed char*>(Gs + a.gsz + WWAVES * per_wave) + wave * Np;
  if (a.gsz > 0) {
    for (int r = wave; r < N; r += WWAVES)
      for (int c = lane; c <= r; c += 64) Gs[tri_at(r, c)] = a.G[(size_t)r * N + c];
    w.Gs = Gs;
  }
  __syncthreads();  // (the last barrier: from here on every wave runs on its own)
  const int64_t inst = (int64_t)blockIdx.x * WWAVES + wave;
  if (inst >= a.ninst) return;
  const int64_t nsteps = a.window_mode ? 1 : a.n - 1;
  for (int j = lane; j < Np; j += 64) st[j] = 0;
  if (lane < 3) xs[lane] = a.x0[inst * 3 + lane];
  lds_sync();
  if (!a.window_mode && lane < 3)  // hist[b, 0, axis, :] = x0
    a.out[((inst >> 1) * a.n * 2 + (inst & 1)) * 3 + lane] = xs[lane];
  const int64_t kstep = (!a.window_mode && (inst & 1) && a.kick != nullptr)
                            ? (a.kick_steps ? a.kick_steps[inst >> 1] : a.kick_step)
                            : -1;
  const double kv = (kstep >= 0) ? a.kick[inst >> 1] : 0.0;
  int fq = 0;
  for (int64_t i = 0; i < nsteps; ++i) {
    const double xv[3] = {xs[0], xs[1], xs[2]};
    // W = Q (z_ref − c) of this window (zmp_controller.py:184, 197), then D = G W on the lane's
    // horizon slots (G symmetric: G[j][k] from the packed lower triangle)
    build_w<NJ>(a, inst, i, xv, W, lane);
    lds_sync();
    double d[NJ];
#pragma unroll
    for (int c = 0; c < NJ; ++c) d[c] = 0.0;
    for (int j = 0; j < N; ++j) {
      const double wj = W[j];
#pragma unroll
      for (int c = 0; c < NJ; ++c) {
        const int k = lane + 64 * c;
        if (k < N) d[c] = fma(g_at(a, w, k, j), wj, d[c]);
      }
    }
    lds_sync();
#pragma unroll
    for (int c = 0; c < NJ; ++c)
      if (lane + 64 * c < N) W[lane + 64 * c] = d[c];
    // warm start: the previous set shifted one slot towards the present (slot N−1 kept)
    if (i > 0) {
      signed char v[NJ];
#pragma unroll
      for (int c = 0; c < NJ; ++c) {
        const int j = lane + 64 * c;
        v[c] = (j + 1 < N) ? st[j + 1] : ((j < N) ? st[j] : 0);
      }
      lds_sync();
#pragma unroll
      for (int c = 0; c < NJ; ++c)
        if (lane + 64 * c < N) st[lane + 64 * c] = v[c];
    }
    lds_sync();
    const double u0 = solve_instance<NJ>(a, inst, i, xv, W, st, w, lane, &fq);
    double xn[3];
    lipm_step(a.lc, xv, u0, xn);  // x⁺ = A x + B u0 (zmp_controller.py:199)
    if (i == kstep) xn[1] -= kv;  // force kick (zmp_controller.py:90,105-106)
    if (!(isfinite(xn[0]) && isfinite(xn[1]) && isfinite(xn[2]))) fq |= ZMPC_ST_NONFINITE;
    lds_sync();
    if (lane < 3) {
      xs[lane] = xn[lane];
      if (a.window_mode)
        a.out[inst * 3 + lane] = xn[lane];
      else
        a.out[(((inst >> 1) * a.n + i + 1) * 2 + (inst & 1)) * 3 + lane] = xn[lane];
    }
    lds_sync();
  }
  if (a.status != nullptr && lane == 0) {
    if (a.window_mode)
      a.status[inst] = fq;
    else if (fq != 0)
      atomicOr(&a.status[inst >> 1], fq);
  }
}

size_t wave_lds_bytes(int Np, int pcap, int gsz) {
  return ((size_t)gsz + WWAVES * (6 * (size_t)Np + pcap + 4)) * sizeof(double) +
         (size_t)WWAVES * Np;
}

size_t strict_lds_bytes(int Np, int ld, int pcap, int gsz) {
  const size_t per_wave = 5 * Np + (size_t)pcap;
  return ((size_t)gsz + SNB * ld + SNB * 4 + SNB + SWAVES * per_wave) * sizeof(double) +
         SNB * Np;
}

}  // namespace

hipError_t zmpc_strict_set_attrs() {
  hipError_t e = hipSuccess;
#define ZMPC_SATTR(J)                                                                   \
  if (e == hipSuccess)                                                                  \
    e = hipFuncSetAttribute((const void*)zmpc_strict_kernel<J>,                        \
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  ZMPC_SATTR(1) ZMPC_SATTR(2) ZMPC_SATTR(3) ZMPC_SATTR(4) ZMPC_SATTR(5) ZMPC_SATTR(6)
  ZMPC_SATTR(7) ZMPC_SATTR(8)
#undef ZMPC_SATTR
#define ZMPC_WATTR(J)                                                                   \
  if (e == hipSuccess)                                                                  \
    e = hipFuncSetAttribute((const void*)zmpc_strict_wave_kernel<J>,                   \
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  ZMPC_WATTR(1) ZMPC_WATTR(2) ZMPC_WATTR(3) ZMPC_WATTR(4) ZMPC_WATTR(5) ZMPC_WATTR(6)
  ZMPC_WATTR(7) ZMPC_WATTR(8)
#undef ZMPC_WATTR
  return e;
}

static hipError_t launch_strict(const zmpc_plan* p, StrictArgs a, hipStream_t s,
                                std::string* why) {
  if (p->N > 512) {
    *why = "strict solver supports horizon N <= 512";
    return hipErrorInvalidValue;
  }
  a.N = p->N;
  a.Np = (p->N + 15) & ~15;
  a.ld = a.Np + 4;
  const size_t budget = 160 * 1024 - 512;
  if (strict_lds_bytes(a.Np, a.ld, 0, 0) > budget) {
    *why = "horizon too long for the strict solver's LDS tile (N=" + std::to_string(p->N) + ")";
    return hipErrorInvalidValue;
  }
  // G packed in LDS when it fits beside a factor room for m <= 32 — N <= ~150; the rest of
  // the room then holds the packed factor
  // (A/B in the diagnostics build only: measured slower at N = 150 — the factor room it
  // leaves is too small)
#ifdef ZMPC_DIAG
  static const bool lds_g = getenv("ZMPC_STRICT_LDS_G") != nullptr;
#else
  constexpr bool lds_g = false;
#endif
  const int gsz = ((p->N * (p->N + 1) / 2) + 1) & ~1;
  a.gsz = (lds_g && strict_lds_bytes(a.Np, a.ld, 32 * 33 / 2, gsz) <= budget) ? gsz : 0;
  // packed factor room for min(|A|, |F|) <= N/2 when it fits, else as much as fits
  const int half = p->N / 2;
  int pcap = half * (half + 1) / 2;
  const size_t fixed = strict_lds_bytes(a.Np, a.ld, 0, a.gsz);
  const int fit = (int)((budget - fixed) / (SWAVES * sizeof(double)));
  if (pcap > fit) pcap = fit;
  a.pcap = pcap & ~1;
  a.Q = p->Q;
  a.hg = p->hg;
  a.lc = p->lc;
  a.G = p->G;
  a.Hz = p->Hz;
  // p(0) = T³/6·1 − T h/g  (zmp_controller.py:171 with i = j)
  a.p0 = p->T3_6 - p->Thg;
  const int64_t ntiles = (a.ninst + SNB - 1) / SNB;
  int grid = (int)std::min<int64_t>(ntiles, (int64_t)p->strict_slots);
  // the global factor room of the waves (reduced systems that fit neither registers nor the
  // packed LDS factor) is allocated per launch, stream-ordered, so concurrent launches of one
  // plan on different streams never share it; m = min(|A|, |F|) <= N/2 bounds its size
  const int64_t half1 = p->N / 2 + 1;
  a.sg_stride = half1 * half1;
  const size_t sg_bytes = (size_t)grid * SWAVES * (size_t)a.sg_stride * sizeof(double);
  if (hipMallocAsync((void**)&a.scratch, sg_bytes, s) != hipSuccess) {
    (void)hipGetLastError();
    return hipErrorOutOfMemory;
  }
  const size_t lds = strict_lds_bytes(a.Np, a.ld, a.pcap, a.gsz);
#ifdef ZMPC_DIAG
  static const bool lds_chol = getenv("ZMPC_STRICT_LDS_CHOL") != nullptr;  // A/B only
  static const bool dbg_on = getenv("ZMPC_DEBUG_STRICT") != nullptr;       // diagnostics only
#else
  constexpr bool lds_chol = false, dbg_on = false;
#endif
  a.lds_chol = lds_chol ? 1 : 0;
  static unsigned long long* dbgbuf = nullptr;
  if (dbg_on && !dbgbuf) (void)hipMalloc((void**)&dbgbuf, 32 * sizeof(unsigned long long));
  if (dbg_on && dbgbuf) {
    (void)hipMemsetAsync(dbgbuf, 0, 32 * sizeof(unsigned long long), s);
    a.dbg = dbgbuf;
  }
  const int nj = (a.N + 63) / 64;
  switch (nj) {
#define ZMPC_SCASE(J)                                                                        \
  case J:                                                                                    \
    hipLaunchKernelGGL(zmpc_strict_kernel<J>, dim3(grid), dim3(256), lds, s, a);             \
    break;
    ZMPC_SCASE(1) ZMPC_SCASE(2) ZMPC_SCASE(3) ZMPC_SCASE(4) ZMPC_SCASE(5) ZMPC_SCASE(6)
    ZMPC_SCASE(7) ZMPC_SCASE(8)
#undef ZMPC_SCASE
    default:
      (void)hipFreeAsync(a.scratch, s);
      *why = "unsupported horizon";
      return hipErrorInvalidValue;
  }
  hipError_t e = hipGetLastError();
  const hipError_t ef = hipFreeAsync(a.scratch, s);
  if (e == hipSuccess) e = ef;
  if (dbg_on && dbgbuf && e == hipSuccess) {
    unsigned long long h[32];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h, dbgbuf, sizeof(h), hipMemcpyDeviceToHost);
    fprintf(stderr,
            "[zmpc strict dbg] grid=%d pcap=%d cycles: prep=%llu compact=%llu gather=%llu "
            "chol=%llu cholsolve=%llu branch=%llu setupd=%llu gemm=%llu inst_all=%llu "
            "barrier=%llu | solves=%llu iters=%llu sum_m=%llu primal=%llu sum_fact=%llu "
            "global_fact=%llu\n",
            grid, a.pcap, h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[15], h[11],
            h[9], h[10], h[13], h[12], h[14]);
    fprintf(stderr, "[zmpc strict dbg] reduced sizes: <=16 %llu, 17-32 %llu, 33-48 %llu, "
            "49-64 %llu, >64 %llu; gsz=%d\n", h[16], h[17], h[18], h[19], h[20], a.gsz);
  }
  return e;
}

// The strict solver of a launch over `ninst` instances (ZMPC_OPT_STRICT_SOLVER: 1 the tile
// kernel above, 2 the reduced-Cholesky one-instance-per-wave kernel, 3 the LQ lane-per-instance
// kernel of strict_lq.hip, 4 the parallel-in-time one-instance-per-wave kernel of
// strict_scan.hip, 0 = auto): small batches take the parallel-in-time kernel and large ones the
// LQ kernel, whose per-pass work is O(N) per lane but serial within it.  The reduced-Cholesky
// wave kernel is a cross-check (profiles/r4/r4e_strict_small_batch.jsonl, N = 150, n = 420: 1
// walk 27.6 ms vs the LQ kernel's 29.0, 8 walks 92.8 vs 46.4 — its passes are long when a
// kicked walk pins many slots).
// Option 4 / auto at up to kScanMaxInst instances: the parallel-in-time kernel of
// strict_scan.hip (one instance per wave, the horizon over the lanes).  Crossover measured at
// N = 150, n = 420 (profiles/r4/r4h_crossover.jsonl): 4096 walks 19.9 vs 55.2 ms (LQ), 8192
// walks 35.6 vs 56.8, 16384 walks 65.2 vs 57.8 — the LQ kernel won from ≈14 000 walks.  Round 5
// (profiles/r5r/cross.jsonl; both kernels faster): 8192 walks 45.0 vs 47.0 ms, 12288 walks 64.9
// vs 47.6 — the LQ kernel wins from ≈8 600 walks.
constexpr int64_t kScanMaxInst = 16384;
enum { kTile = 1, kWave = 2, kLq = 3, kScan = 4 };

static int strict_mode(const zmpc_plan* p, int64_t ninst) {
  const int opt = p->opt[ZMPC_OPT_STRICT_SOLVER];
  const bool lq_ok = zmpc_strict_lq_supported(p);
  const bool scan_ok = zmpc_strict_scan_supported(p);
  if (opt == 1) return kTile;
  if (opt == 2) return kWave;
  if (opt == 3) return kLq;    // (zmpc_plan_set_option accepts 3 and 4 only where they run)
  if (opt == 4) return kScan;
  if (scan_ok && (ninst <= kScanMaxInst || !lq_ok)) return kScan;
  return lq_ok ? kLq : kTile;
}

static hipError_t launch_strict_wave(const zmpc_plan* p, StrictArgs a, hipStream_t s,
                                     std::string* why) {
  if (p->N > 512) {
    *why = "strict solver supports horizon N <= 512";
    return hipErrorInvalidValue;
  }
  a.N = p->N;
  a.Np = (p->N + 15) & ~15;
  a.ld = a.Np;
  a.Q = p->Q;
  a.hg = p->hg;
  a.lc = p->lc;
  a.G = p->G;
  a.Hz = p->Hz;
  a.p0 = p->T3_6 - p->Thg;  // p(0) (zmp_controller.py:171, i = j)
  a.lds_chol = 0;
  a.dbg = nullptr;
  const size_t budget = 160 * 1024 - 512;
  // G packed in LDS when it fits beside a factor room for reduced systems of 32
  const int gsz = ((p->N * (p->N + 1) / 2) + 1) & ~1;
  a.gsz = wave_lds_bytes(a.Np, 32 * 33 / 2, gsz) <= budget ? gsz : 0;
  if (wave_lds_bytes(a.Np, 0, a.gsz) > budget) {
    *why = "horizon too long for the strict wave kernel's LDS (N=" + std::to_string(p->N) + ")";
    return hipErrorInvalidValue;
  }
  // packed factor room for min(|A|, |F|) <= N/2 when it fits, else as much as fits (larger
  // reduced systems factor in the wave's global scratch)
  const int half = p->N / 2;
  int pcap = half * (half + 1) / 2;
  const int fit = (int)((budget - wave_lds_bytes(a.Np, 0, a.gsz)) / (WWAVES * sizeof(double)));
  if (pcap > fit) pcap = fit;
  a.pcap = pcap & ~1;
  const int64_t grid = (a.ninst + WWAVES - 1) / WWAVES;
  const int64_t half1 = p->N / 2 + 1;
  a.sg_stride = half1 * half1;
  const size_t sg_bytes = (size_t)grid * WWAVES * (size_t)a.sg_stride * sizeof(double);
  if (hipMallocAsync((void**)&a.scratch, sg_bytes, s) != hipSuccess) {
    (void)hipGetLastError();
    return hipErrorOutOfMemory;
  }
  const size_t lds = wave_lds_bytes(a.Np, a.pcap, a.gsz);
  switch ((a.N + 63) / 64) {
#define ZMPC_WCASE(J)                                                                       \
  case J:                                                                                   \
    hipLaunchKernelGGL(zmpc_strict_wave_kernel<J>, dim3((unsigned)grid), dim3(64 * WWAVES), \
                       lds, s, a);                                                          \
    break;
    ZMPC_WCASE(1) ZMPC_WCASE(2) ZMPC_WCASE(3) ZMPC_WCASE(4) ZMPC_WCASE(5) ZMPC_WCASE(6)
    ZMPC_WCASE(7) ZMPC_WCASE(8)
#undef ZMPC_WCASE
    default:
      (void)hipFreeAsync(a.scratch, s);
      *why = "unsupported horizon";
      return hipErrorInvalidValue;
  }
  hipError_t e = hipGetLastError();
  const hipError_t ef = hipFreeAsync(a.scratch, s);
  return e != hipSuccess ? e : ef;
}

hipError_t zmpc_launch_rollout_strict(const zmpc_plan* p, int64_t B, int64_t n,
                                      const double* zmax, const double* zmin, int64_t bstride,
                                      const double* x0, const double* kick, int64_t kick_step,
                                      const int64_t* kick_steps, double* hist, int32_t* status,
                                      hipStream_t s, std::string* why) {
  const int mode = strict_mode(p, 2 * B);
  if (mode == kScan && n > 1)
    return zmpc_launch_rollout_strict_scan(p, B, n, zmax, zmin, bstride, x0, kick, kick_step,
                                           kick_steps, hist, status, s, why);
  if (mode == kLq && n > 1)
    return zmpc_launch_rollout_strict_lq(p, B, n, zmax, zmin, bstride, x0, kick, kick_step,
                                         kick_steps, hist, status, s, why);
  if (!p->G) {
    *why = "plan was created without strict workspace";
    return hipErrorInvalidValue;
  }
  if (n == 1) {
    hipError_t e = hipMemcpyAsync(hist, x0, 6 * sizeof(double) * (size_t)B,
                                  hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
    if (status) return hipMemsetAsync(status, 0, sizeof(int32_t) * B, s);
    return hipSuccess;
  }
  if (status) {
    hipError_t e = hipMemsetAsync(status, 0, sizeof(int32_t) * B, s);
    if (e != hipSuccess) return e;
  }
  StrictArgs a{};
  a.window_mode = 0;
  a.n = n;
  a.bstride = bstride;
  a.ninst = 2 * B;
  a.zmax = zmax;
  a.zmin = zmin;
  a.x0 = x0;
  a.kick = kick;
  a.kick_step = kick_step;
  a.kick_steps = kick_steps;
  a.out = hist;
  a.status = status;
  return mode == kWave ? launch_strict_wave(p, a, s, why) : launch_strict(p, a, s, why);
}

hipError_t zmpc_launch_step_strict(const zmpc_plan* p, int64_t B, const double* x,
                                   const double* zmax_win, const double* zmin_win,
                                   double* x_next, int32_t* status, hipStream_t s,
                                   std::string* why) {
  const int mode = strict_mode(p, B);
  if (mode == kScan)
    return zmpc_launch_step_strict_scan(p, B, x, zmax_win, zmin_win, x_next, status, s, why);
  if (mode == kLq)
    return zmpc_launch_step_strict_lq(p, B, x, zmax_win, zmin_win, x_next, status, s, why);
  if (!p->G) {
    *why = "plan was created without strict workspace";
    return hipErrorInvalidValue;
  }
  StrictArgs a{};
  a.window_mode = 1;
  a.n = 0;
  a.ninst = B;
  a.zmax = zmax_win;
  a.zmin = zmin_win;
  a.x0 = x;
  a.kick = nullptr;
  a.kick_step = -1;
  a.out = x_next;
  a.status = status;
  return mode == kWave ? launch_strict_wave(p, a, s, why) : launch_strict(p, a, s, why);
}
