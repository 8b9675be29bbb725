// Unconstrained Wieber rollout on the device (config.strict == False).
//
// Reference (per walk, sequential, one QP per axis per timestep):
//   generate_com_trajectory_wieber   zmp_controller.py:59-108
//   generate_state_trajectory_wieber zmp_controller.py:110-147
//   predict_wieber_axis (strict=False) zmp_controller.py:196-201
//     X = -inv(PuᵀPu + R/Q·I) Puᵀ (Px x - z_ref);  x⁺ = A x + B X[0]
// Only X[0] is used, so with the plan's gain row k (= row 0 of inv(M) Puᵀ) and kx = k·Px:
//     u_i = f_i - kx·x_i,   f_i = Σ_j k_j z_ref[i+1+j]   (window rows i+1..i+N, :95-104)
// f does not depend on the state, so the N-long dot products of all timesteps are computed
// in parallel (a sliding correlation), and only the 3-dim state recursion is sequential;
// that recursion is run as a lane-parallel affine scan.
//
// Mapping: one 64-lane wavefront per walk (both axes):
//   1. the walk's bounds (16-B coalesced, whole walk in flight) → z_ref = (z_max + z_min)/2
//      (:197) for both axes in LDS, padded with the last row (:81-88); the gain row k is
//      staged in LDS next to it;
//   2. correlation: lane l owns timesteps [l·CW, l·CW + CW), a CW-deep register sliding
//      window, k read as a wave-uniform LDS broadcast: one z_ref read per CW FMAs per axis;
//   3. chunked affine scan over the 64 lanes with P = Ā^CW (Ā = A - B kxᵀ, powers from the
//      plan), Kogge-Stone;
//   4. each lane replays its chunk in the reference form x⁺ = A x + B u with the F_ext kick
//      (:105-106); history rows are staged in LDS and leave as contiguous 1-KiB wave stores.
// Walks longer than 64·8+1 samples take several correlation passes with f kept in LDS.
#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "zmpc_internal.h"

namespace {

struct Mat3 {
  double m[9];
};

__device__ __forceinline__ Mat3 matmul3(const Mat3& a, const Mat3& b) {
  Mat3 c;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      c.m[3 * i + j] = fma(a.m[3 * i + 0], b.m[0 + j],
                           fma(a.m[3 * i + 1], b.m[3 + j], a.m[3 * i + 2] * b.m[6 + j]));
  return c;
}

__device__ __forceinline__ void matvec3(const Mat3& a, const double* x, double* y) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
    y[i] = fma(a.m[3 * i + 0], x[0], fma(a.m[3 * i + 1], x[1], a.m[3 * i + 2] * x[2]));
}

// A double moved across lanes by DPP (two 32-bit halves); `ctrl` a DPP control word,
// row_mask the rows written (the others keep 0), out-of-row reads 0 (bound_ctrl).
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWS, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWS, 0xF, true);
  return __hiloint2double(hi, lo);
}

// Inclusive affine Kogge-Stone scan over the 64 lanes, T_l = Σ_{m≤l} P^(l−m) s_m, on the VALU's
// DPP lane moves instead of LDS-pipe shuffles: four row_shr levels (1, 2, 4, 8) inside each
// 16-lane row with the uniform P^(2^r), then row_bcast:15 (rows 1, 3 take lanes 15, 47) and
// row_bcast:31 (rows 2, 3 take lane 31) with each lane's own power P^k from the plan
// (pw = [33][9], k = its distance to the source lane).
__device__ __forceinline__ void dpp_level(double* sv, const Mat3& M, double u0, double u1,
                                          double u2) {
  const double u[3] = {u0, u1, u2};
  double t[3];
  matvec3(M, u, t);
  sv[0] += t[0];
  sv[1] += t[1];
  sv[2] += t[2];
}

__device__ __forceinline__ void scan_dpp(double* sv, int lane, const double* __restrict__ Pp,
                                         const double* __restrict__ pw) {
#define ZMPC_DPP_ROW(R2, CTRL)                                                             \
  {                                                                                        \
    Mat3 Pd;                                                                               \
    _Pragma("unroll") for (int q = 0; q < 9; ++q) Pd.m[q] = Pp[(R2) * 9 + q];              \
    dpp_level(sv, Pd, dpp_f64<CTRL, 0xF>(sv[0]), dpp_f64<CTRL, 0xF>(sv[1]),                \
              dpp_f64<CTRL, 0xF>(sv[2]));                                                  \
  }
  ZMPC_DPP_ROW(0, 0x111)  // row_shr:1
  ZMPC_DPP_ROW(1, 0x112)  // row_shr:2
  ZMPC_DPP_ROW(2, 0x114)  // row_shr:4
  ZMPC_DPP_ROW(3, 0x118)  // row_shr:8
#undef ZMPC_DPP_ROW
  {  // rows 1 and 3 take lane 15 / 47 at distance (lane & 15) + 1
    const double* m = pw + ((lane & 15) + 1) * 9;
    Mat3 M;
#pragma unroll
    for (int q = 0; q < 9; ++q) M.m[q] = m[q];
    dpp_level(sv, M, dpp_f64<0x142, 0xA>(sv[0]), dpp_f64<0x142, 0xA>(sv[1]),
              dpp_f64<0x142, 0xA>(sv[2]));
  }
  {  // rows 2 and 3 take lane 31 at distance lane − 31
    const double* m = pw + (lane >= 32 ? lane - 31 : 0) * 9;
    Mat3 M;
#pragma unroll
    for (int q = 0; q < 9; ++q) M.m[q] = m[q];
    dpp_level(sv, M, dpp_f64<0x143, 0xC>(sv[0]), dpp_f64<0x143, 0xC>(sv[1]),
              dpp_f64<0x143, 0xC>(sv[2]));
  }
}

// Reference state update x⁺ = A x + B u (zmp_controller.py:199).
__device__ __forceinline__ void lipm_step(const LipmConsts& c, const double* x, double u,
                                          double* y) {
  y[0] = x[0] + c.T * x[1] + c.T2_2 * x[2] + c.T3_6 * u;
  y[1] = x[1] + c.T * x[2] + c.T2_2 * u;
  y[2] = x[2] + c.T * u;
}

// Correlation tile width: outputs per lane per pass, chosen per walk length so that
// passes·64·CW barely covers the n−1 timesteps (n = 420 → CW = 7: 448 outputs, 1 pass).
int pick_cw(int64_t nsteps) {
  int best = 8;
  int64_t best_cost = INT64_MAX;
  for (int cw = 8; cw >= 1; --cw) {
    const int64_t cost = ((nsteps + 64 * cw - 1) / (64 * cw)) * cw;
    if (cost < best_cost) {
      best_cost = cost;
      best = cw;
    }
  }
  return best;
}

// LDS layout of z_ref: lane l's chunk starts at t = l·CW; for even CW one pad double per CW
// keeps the 64 lanes' ds_read_b64 on distinct banks (lane stride CW+1 doubles, odd).
template <int CW>
struct ZrLayout {
  static constexpr int kPad = (CW % 2 == 0) ? 1 : 0;
  __host__ __device__ static constexpr int idx(int t) { return t + kPad * (t / CW); }
};

// History staging of the split kernels: row 0 the initial state, row m + 1 the state after
// step m (6 doubles: both axes), written by the lane owning step m.  For even CW the lanes'
// rows are CW·48 bytes apart, a multiple of 128 B, so the 16 lanes of a ds_write_b64 group hit
// one or two banks (16-way at CW = 8); two pad doubles after every 2·CW rows (every second
// lane) spread them over eight bank pairs (2-way, as odd CW) for CW = 2..8, at 2 % more LDS
// (after every CW rows the same 2-way costs twice the pad, which at n = 476 took one of the seven
// workgroups a CU holds).  The copy-out skips the pads.
template <int CW>
struct HistLayout {
  static constexpr int kPad = (CW % 2 == 0) ? 2 : 0;  // doubles after every 2·CW step rows
  static constexpr int kSpan = 2 * CW;
  __host__ __device__ static constexpr int row(int r) {  // first double of staged row r
    return r * 6 + (r >= 1 ? kPad * ((r - 1) / kSpan) : 0);
  }
  __host__ __device__ static constexpr size_t doubles(int n) {
    return (size_t)n * 6 + (size_t)kPad * ((n + kSpan - 1) / kSpan);
  }
};

struct RolloutGeom {
  int cw, passes, kc, lz, lzp, nf;
  int kfm;  // fast-FIR steps (odd CW; axis_correlate_ffa), 0 otherwise
  int kcp;  // doubles of LDS for the staged gain row (kc rounded up to even)
};

RolloutGeom rollout_geom(int N, int64_t n) {
  RolloutGeom g;
  const int64_t nsteps = n - 1;
  g.cw = pick_cw(nsteps);
  g.passes = (int)((nsteps + 64 * g.cw - 1) / (64 * g.cw));
  g.kc = (N + g.cw - 1) / g.cw * g.cw;           // k loop bound (k zero-padded)
  g.lz = g.passes * 64 * g.cw + g.kc + 1;         // z_ref samples staged (padded with last)
  g.kfm = 0;
  if (g.cw & 1) {
    // the fast-FIR form (odd CW) reads up to sample 64·CW + 2·kfm + W of the walk
    const int U = g.cw / 2 + 1, mm = (N + 2) / 2;
    g.kfm = (mm + U - 1) / U * U;
    g.lz = std::max(g.lz, g.passes * 64 * g.cw + 2 * g.kfm + 2 * U + 2);
  }
  const int pad = (g.cw % 2 == 0) ? 1 : 0;
  g.lzp = g.lz + pad * (g.lz / g.cw) + 1;         // LDS doubles per axis
  // the z_ref area doubles as the history staging buffer: at least a third of a walk of rows
  const int64_t stage_min = ((n + 2) / 3 * 6 + 1) / 2;
  if (g.lzp < stage_min) g.lzp = (int)stage_min;
  g.lzp = (g.lzp + 1) & ~1;
  g.nf = g.passes == 1 ? 0 : (int)((nsteps + 2) & ~1LL);  // f lives in LDS only if passes > 1
  g.kcp = (g.kc + 1) & ~1;
  return g;
}

size_t lds_bytes(const RolloutGeom& g) {
  return (size_t)(g.kcp + 2 * g.lzp + 2 * g.nf) * sizeof(double);
}

struct RolloutArgs {
  int kc, kcp, lz, lzp, n;
  int64_t B;
  LipmConsts lc;
  const double* k;
  const double* kx;
  const double* zmax;
  const double* zmin;
  int64_t bstride;
  const double* x0;
  const double* kick;
  int64_t kick_step;
  double* hist;
  int32_t* status;
  const double* scanP;  // [8][kScanLevels][9]: (Ā^C)^(2^r) for C = 1..8 (plan), or null
  int dbg;
  int srows;  // history rows the split-axis kernels stage per copy-out round
  const int64_t* kick_steps;  // [B] per-walk kick steps (ragged walks), or null: kick_step
  const double* fsh;  // shared CoP (bounds stride 0): f of both axes, [2][fstride], or null
  int fstride;
  const double2* fft_tw;  // plan twiddles e^{−2πi m/kFftPT} (FFT correlation, wide kernel)
  const double2* fft_g;   // plan gain spectrum DFT(g)/P for this launch's P
  const double* kffa;     // plan fast-FIR taps [kffa_rows(N)][4] (axis_correlate_ffa)
  int kfm;                // fast-FIR steps per walk, ⌈(N+1)/2⌉ rounded up to the unroll
  const double* ksum;     // plan suffix sums of k [ksum_rows(N)] (axis_correlate_sparse), or null
  int hN;                 // horizon N (ksum layout)
  int64_t pf_ahead;       // one walk per workgroup: touch walk b + pf_ahead's bounds (the next
                          // dispatch round's) into the caches early; 0 = off
  unsigned long long* tl;  // diagnostics build only (ZMPC_ROLLOUT_TL): per-walk phase stamps
};

// Diagnostic ablation bits (ZMPC_DEBUG_ROLLOUT: 1 no correlation, 2 no scan, 4 no history
// stores, 8 bounds from row 0) — compiled only into the diagnostics build (make diag,
// -DZMPC_DIAG); the product library has none of them.
#ifdef ZMPC_DIAG
__device__ __forceinline__ int dbgb(const RolloutArgs& a, int bit) { return a.dbg & bit; }
// phase stamps of walk b (wave 0's view, the 100 MHz constant clock): [0] start, [1] bounds in
// LDS, [2] correlation done, [3] history staged, [4] copy-out issued
__device__ __forceinline__ void tl_stamp(const RolloutArgs& a, int64_t b, int k) {
  if (a.tl != nullptr && threadIdx.x == 0) a.tl[b * 5 + k] = (unsigned long long)wall_clock64();
}
#else
__device__ __forceinline__ constexpr int dbgb(const RolloutArgs&, int) { return 0; }
__device__ __forceinline__ void tl_stamp(const RolloutArgs&, int64_t, int) {}
#endif

// a 16-byte store with the non-temporal hint (streamed past the caches)
__device__ __forceinline__ void st_nt2(double2* p, double2 v) {
  typedef double v2d __attribute__((ext_vector_type(2)));
  const v2d t = {v.x, v.y};
  __builtin_nontemporal_store(t, reinterpret_cast<v2d*>(p));
}

// The kick step of walk b: per walk (ragged batches) or the launch-wide one.
__device__ __forceinline__ int64_t kick_step_of(const RolloutArgs& a, int64_t b) {
  return a.kick_steps != nullptr ? a.kick_steps[b] : a.kick_step;
}


// Bounds of one walk held in registers: PF rounds of 64 samples, one 16-B (x, y) pair of
// each bound array per lane and round.
template <int PF>
struct BoundRegs {
  double2 hi[PF], lo[PF];
};

template <int PF>
__device__ __forceinline__ void load_bounds(const RolloutArgs& a, int64_t b, int lane,
                                            BoundRegs<PF>& r) {
  const double2* zmx = reinterpret_cast<const double2*>(a.zmax + b * a.bstride);
  const double2* zmn = reinterpret_cast<const double2*>(a.zmin + b * a.bstride);
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    const int t = u * 64 + lane;
    if (t < a.n) {
      r.hi[u] = zmx[t];
      r.lo[u] = zmn[t];
    }
  }
}

// z_ref = (z_max + z_min) / 2 into the (padded) LDS layout, then the last row repeated up to
// lz (the window padding of zmp_controller.py:81-88).
template <int CW, int PF>
__device__ __forceinline__ void store_zref(const RolloutArgs& a, const BoundRegs<PF>& r,
                                           double* zr0, double* zr1, int lane) {
  using ZL = ZrLayout<CW>;
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    const int t = u * 64 + lane;
    if (t < a.n) {
      zr0[ZL::idx(t)] = (r.hi[u].x + r.lo[u].x) / 2;
      zr1[ZL::idx(t)] = (r.hi[u].y + r.lo[u].y) / 2;
    }
  }
  // the last sample lives in lane (n-1)%64 of round (n-1)/64: broadcast it
  const int ul = (a.n - 1) >> 6, ll = (a.n - 1) & 63;
  double h0 = 0.0, h1 = 0.0, l0 = 0.0, l1 = 0.0;
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u == ul) {
      h0 = r.hi[u].x;
      h1 = r.hi[u].y;
      l0 = r.lo[u].x;
      l1 = r.lo[u].y;
    }
  h0 = __shfl(h0, ll, 64);
  h1 = __shfl(h1, ll, 64);
  l0 = __shfl(l0, ll, 64);
  l1 = __shfl(l1, ll, 64);
  const double last0 = (h0 + l0) / 2, last1 = (h1 + l1) / 2;
  for (int t = a.n + lane; t < a.lz; t += 64) {
    zr0[ZL::idx(t)] = last0;
    zr1[ZL::idx(t)] = last1;
  }
}

// f for lane l's CW timesteps of one pass starting at i0 (both axes).
// k is read from the wave's LDS copy (ks): wave-uniform broadcast reads keep every lgkm
// operation of the loop an in-order LDS access, so waits stay counted (a scalar load here
// would force lgkmcnt(0) drains of the z_ref reads in flight).
template <int CW>
__device__ __forceinline__ void correlate(const RolloutArgs& a, const double* ks,
                                          const double* zr0, const double* zr1, int i0,
                                          double* a0, double* a1) {
  using ZL = ZrLayout<CW>;
  // i0 is a multiple of CW, so idx(i0 + c) = idx(i0) + idx(c): compile-time offsets
  const double* z0 = zr0 + ZL::idx(i0);
  const double* z1 = zr1 + ZL::idx(i0);
  double w0[CW], w1[CW];
#pragma unroll
  for (int m = 0; m < CW; ++m) {
    a0[m] = 0.0;
    a1[m] = 0.0;
    w0[m] = z0[ZL::idx(1 + m)];
    w1[m] = z1[ZL::idx(1 + m)];
  }
  const double* k = ks;
  for (int j = 0; j < a.kc; j += CW) {
#pragma unroll
    for (int jj = 0; jj < CW; ++jj) {
      const double kj = k[j + jj];
#pragma unroll
      for (int m = 0; m < CW; ++m) {
        a0[m] = fma(kj, w0[(jj + m) % CW], a0[m]);
        a1[m] = fma(kj, w1[(jj + m) % CW], a1[m]);
      }
      w0[jj] = z0[ZL::idx(1 + jj + CW)];
      w1[jj] = z1[ZL::idx(1 + jj + CW)];
    }
    z0 += CW + ZL::kPad;
    z1 += CW + ZL::kPad;
  }
}

// Scan, replay and store of one walk whose f is in registers (REGF: a0/a1[q] = f of
// timestep lane·CW + q) or in LDS (f0/f1).  `stage` (>= 2·lzp doubles) is free LDS.
template <int CW, bool REGF>
__device__ __forceinline__ void scan_replay_store(const RolloutArgs& a, int64_t b, int lane,
                                                  const double* a0, const double* a1,
                                                  const double* f0, const double* f1,
                                                  double* stage, const double* xi0,
                                                  const double* xi1, double kk) {
  const int n = a.n, nsteps = n - 1;
  const LipmConsts lc = a.lc;
  const double kx0 = a.kx[0], kx1 = a.kx[1], kx2 = a.kx[2];
  const double Bv[3] = {lc.T3_6, lc.T2_2, lc.T};
  Mat3 Ab;  // Ā = A - B kxᵀ
  {
    const double A[9] = {1.0, lc.T, lc.T2_2, 0.0, 1.0, lc.T, 0.0, 0.0, 1.0};
    const double kx[3] = {kx0, kx1, kx2};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) Ab.m[3 * i + j] = A[3 * i + j] - Bv[i] * kx[j];
  }
  const int C = REGF ? CW : (nsteps + 63) / 64;  // steps per lane chunk
  const int mbeg = lane * C;
  const int64_t kick_step = kick_step_of(a, b);

  // ---- 3. affine scan of x_{i+1} = Ā x_i + B f_i (+ kick) over 64 lane chunks ----------
  double s0[3] = {0.0, 0.0, 0.0}, s1[3] = {0.0, 0.0, 0.0};
  auto scan_step = [&](int m, double fx, double fy) {
    double t[3];
    matvec3(Ab, s0, t);
    s0[0] = fma(Bv[0], fx, t[0]);
    s0[1] = fma(Bv[1], fx, t[1]);
    s0[2] = fma(Bv[2], fx, t[2]);
    matvec3(Ab, s1, t);
    s1[0] = fma(Bv[0], fy, t[0]);
    s1[1] = fma(Bv[1], fy, t[1]);
    s1[2] = fma(Bv[2], fy, t[2]);
    if (m == kick_step) s1[1] -= kk;
  };
  if constexpr (REGF) {
#pragma unroll
    for (int q = 0; q < CW; ++q)
      if (mbeg + q < nsteps) scan_step(mbeg + q, a0[q], a1[q]);
  } else {
    for (int m = mbeg; m < min(mbeg + C, nsteps); ++m) scan_step(m, f0[m], f1[m]);
  }
  Mat3 P;  // P = Ā^C (from the plan for C <= 8)
  const bool pre = REGF && a.scanP != nullptr;
  if (pre) {
#pragma unroll
    for (int q = 0; q < 9; ++q) P.m[q] = a.scanP[(C - 1) * kScanStride + q];
  } else {
    P = Ab;
    for (int q = 1; q < C; ++q) P = matmul3(P, Ab);
  }
  if (lane == 0) {
    double t[3];
    matvec3(P, xi0, t);
    for (int i = 0; i < 3; ++i) s0[i] += t[i];
    matvec3(P, xi1, t);
    for (int i = 0; i < 3; ++i) s1[i] += t[i];
  }
  // inclusive Kogge-Stone: T_l += P^d T_{l-d}
  Mat3 Pd = P;
  int r2 = 0;
  for (int d = 1; d < (dbgb(a, 2) ? 1 : 64); d <<= 1, ++r2) {
    double u0[3], u1[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      u0[i] = __shfl_up(s0[i], d, 64);
      u1[i] = __shfl_up(s1[i], d, 64);
    }
    if (lane >= d) {
      double t[3];
      matvec3(Pd, u0, t);
      for (int i = 0; i < 3; ++i) s0[i] += t[i];
      matvec3(Pd, u1, t);
      for (int i = 0; i < 3; ++i) s1[i] += t[i];
    }
    if (pre && r2 < 5) {
#pragma unroll
      for (int q = 0; q < 9; ++q) Pd.m[q] = a.scanP[(C - 1) * kScanStride + (r2 + 1) * 9 + q];
    } else {
      Pd = matmul3(Pd, Pd);
    }
  }
  double x[3], y[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double p0 = __shfl_up(s0[i], 1, 64);
    const double p1 = __shfl_up(s1[i], 1, 64);
    x[i] = (lane == 0) ? xi0[i] : p0;
    y[i] = (lane == 0) ? xi1[i] : p1;
  }

  // ---- 4. replay in the reference form x⁺ = A x + B u; store through LDS ------------
  // Lane l produces history rows l·C+1 .. l·C+C, i.e. 48-B pieces 48·C bytes apart across
  // lanes; written directly that is one L2 request per lane per 16 B.  Instead the rows
  // are staged in LDS, `rows_per_round` at a time, and copied out as contiguous 1-KiB wave
  // stores; the cheap replay is recomputed once per round.
  const int rows_per_round = (2 * a.lzp) / 6;
  double* hb = a.hist + b * (int64_t)n * 6;
  const double xs0[3] = {x[0], x[1], x[2]}, ys0[3] = {y[0], y[1], y[2]};
  for (int r0 = 0; r0 < n; r0 += rows_per_round) {
    const int r1 = min(r0 + rows_per_round, n);
    if (lane == 0 && r0 == 0) {
      stage[0] = xi0[0];
      stage[1] = xi0[1];
      stage[2] = xi0[2];
      stage[3] = xi1[0];
      stage[4] = xi1[1];
      stage[5] = xi1[2];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      x[i] = xs0[i];
      y[i] = ys0[i];
    }
    auto replay_step = [&](int m, double fx, double fy) {
      const double ux = fx - (kx0 * x[0] + kx1 * x[1] + kx2 * x[2]);
      const double uy = fy - (kx0 * y[0] + kx1 * y[1] + kx2 * y[2]);
      double xn[3], yn[3];
      lipm_step(lc, x, ux, xn);
      lipm_step(lc, y, uy, yn);
      if (m == kick_step) yn[1] -= kk;
      const int row = m + 1;
      if (row >= r0 && row < r1) {
        double* o = stage + (row - r0) * 6;
        o[0] = xn[0];
        o[1] = xn[1];
        o[2] = xn[2];
        o[3] = yn[0];
        o[4] = yn[1];
        o[5] = yn[2];
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        x[i] = xn[i];
        y[i] = yn[i];
      }
    };
    if constexpr (REGF) {
#pragma unroll
      for (int q = 0; q < CW; ++q)
        if (mbeg + q < nsteps) replay_step(mbeg + q, a0[q], a1[q]);
    } else {
      for (int m = mbeg; m < min(mbeg + C, nsteps); ++m) replay_step(m, f0[m], f1[m]);
    }
    __syncthreads();
    if (!dbgb(a, 4)) {
      const int nd2 = (r1 - r0) * 3;  // double2 items
      const double2* src = reinterpret_cast<const double2*>(stage);
      double2* dst = reinterpret_cast<double2*>(hb + (int64_t)r0 * 6);
      for (int e = lane; e < nd2; e += 64) dst[e] = src[e];
    }
    __syncthreads();
  }
  if (a.status != nullptr) {
    const bool finite = isfinite(x[0]) && isfinite(x[1]) && isfinite(x[2]) &&
                        isfinite(y[0]) && isfinite(y[1]) && isfinite(y[2]);
    const unsigned long long bad = __ballot(!finite);
    if (lane == 0) a.status[b] = bad ? ZMPC_ST_NONFINITE : 0;
  }
}

// Walks of at most 64·CW+1 samples (one correlation pass): one wave per walk, f stays in
// registers (lane l's CW outputs are exactly its scan chunk).
template <int CW>
__global__ void __launch_bounds__(64) zmpc_rollout_unc_kernel(RolloutArgs a) {
  constexpr int PF = CW + 1;  // 64·(CW+1) >= n
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  double* ks = smem;
  double* zr0 = smem + a.kcp;
  double* zr1 = zr0 + a.lzp;
  BoundRegs<PF> r;
  if (!dbgb(a, 8)) load_bounds<PF>(a, b, lane, r);
  // everything the tail needs is requested up front, behind the bound loads
  const double* xb = a.x0 + b * 6;
  const double xi0[3] = {xb[0], xb[1], xb[2]};
  const double xi1[3] = {xb[3], xb[4], xb[5]};
  const double kk = (a.kick != nullptr) ? a.kick[b] : 0.0;
  for (int j = lane; j < a.kcp; j += 64) ks[j] = a.k[j];
  store_zref<CW, PF>(a, r, zr0, zr1, lane);
  __syncthreads();
  double a0[CW], a1[CW];
  if (!dbgb(a, 1)) {
    correlate<CW>(a, ks, zr0, zr1, lane * CW, a0, a1);
  } else {
#pragma unroll
    for (int m = 0; m < CW; ++m) a0[m] = a1[m] = 0.0;
  }
  __syncthreads();
  scan_replay_store<CW, true>(a, b, lane, a0, a1, nullptr, nullptr, zr0, xi0, xi1, kk);
}

// Split-axis single-pass kernels: a 128-thread workgroup per walk, wave 0 solves the x axis
// and wave 1 the y axis (half the registers and twice the waves of the one-wave kernel, for
// latency hiding); they share the staged z_ref and the history staging rows, so loads and
// stores stay whole-walk coalesced.
template <int CW>
struct AxisBounds {
  static constexpr int PF2 = (CW + 2) / 2;  // 128·PF2 >= 64·(CW+1) >= n
  double2 hi[PF2], lo[PF2];
};

template <int CW>
__device__ __forceinline__ void axis_load(const RolloutArgs& a, int64_t b, int tid,
                                          AxisBounds<CW>& r) {
  const double2* zmx = reinterpret_cast<const double2*>(a.zmax + b * a.bstride);
  const double2* zmn = reinterpret_cast<const double2*>(a.zmin + b * a.bstride);
#pragma unroll
  for (int u = 0; u < AxisBounds<CW>::PF2; ++u) {
    const int t = u * 128 + tid;
    // clamped rather than predicated (predicated double2 loads here crash the gfx950 backend
    // of ROCm 7.2 in machine copy propagation); dbg bit 8 turns every load into row 0
    const int tc = dbgb(a, 8) ? 0 : min(t, a.n - 1);
    r.hi[u] = zmx[tc];
    r.lo[u] = zmn[tc];
  }
}

template <int CW>
__device__ __forceinline__ void axis_correlate(const RolloutArgs& a, const double* __restrict__ ks,
                                               const double* zr, int lane, double* f) {
  using ZL = ZrLayout<CW>;
  const double* z = zr + ZL::idx(lane * CW);
  double w[CW];
#pragma unroll
  for (int m = 0; m < CW; ++m) {
    f[m] = 0.0;
    w[m] = z[ZL::idx(1 + m)];
  }
  for (int j = 0; j < (dbgb(a, 1) ? 0 : a.kc); j += CW) {
#pragma unroll
    for (int jj = 0; jj < CW; ++jj) {
      const double kj = ks[j + jj];
#pragma unroll
      for (int m = 0; m < CW; ++m) f[m] = fma(kj, w[(jj + m) % CW], f[m]);
      w[jj] = z[ZL::idx(1 + jj + CW)];
    }
    z += CW + ZL::kPad;
  }
}

// The same correlation in two-parallel fast-FIR form (odd CW).  With g_j = z_ref[s + 1 + j]
// (s = lane·CW), E_m = k_{2m}, O_m = k_{2m+1} and h_j = g_j + g_{j+1}, the half-length sums
//   A(t) = Σ_m E_m g_{t+2m},  Bo(t) = Σ_m O_m g_{t+2m+1},  C(t) = Σ_m (E_m + O_{m−1}) h_{t+2m}
// give f_t = A(t) + Bo(t) and f_{t+1} = C(t) − A(t) − Bo(t+2) (C(t) = A(t) + f_{t+1} + Bo(t+2)).
// The lane's CW outputs are ⌊CW/2⌋ pairs (t = s + 2i) and one single (t = s + CW − 1, which
// reuses the last pair's Bo(t+2)): ⌈CW/2⌉ A, ⌈CW/2⌉ Bo and ⌊CW/2⌋ C sums of ⌈(N+1)/2⌉ taps —
// 11 × 76 FMAs + 76 additions (h) at CW = 7, N = 150, against 7 × 154 for the direct form.
// A window of W = CW + 1 samples slides two per step (ring of W registers, renamed by the U-step
// unroll), the h values a ring of U; one 16-byte pair of samples per step from LDS, the taps
// (E_m, O_m, E_m + O_{m−1}) one wave-uniform row of the plan's table.
template <int CW>
__device__ __forceinline__ void axis_correlate_ffa(const RolloutArgs& a,
                                                   const double* __restrict__ kt,
                                                   const double* zr, int lane, double* f) {
  static_assert(CW & 1, "the fast-FIR correlation takes odd chunk widths (no LDS padding)");
  constexpr int NP = CW / 2, NA = NP + 1, NB = NP + 1, NC = NP, U = NP + 1, W = 2 * U;
  const double* g = zr + lane * CW + 1;
  double w[W], hr[U], A[NA], Bo[NB], C[NC > 0 ? NC : 1];
#pragma unroll
  for (int j = 0; j < W; ++j) w[j] = g[j];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    A[i] = 0.0;
    Bo[i] = 0.0;
  }
#pragma unroll
  for (int i = 0; i < NC; ++i) C[i] = 0.0;
#pragma unroll
  for (int i = 0; i + 1 < NC; ++i) hr[i] = w[2 * i] + w[2 * i + 1];  // h_{s+2i}
  const int mloop = dbgb(a, 1) ? 0 : a.kfm;
  const double* tr = kt;
  for (int m0 = 0; m0 < mloop; m0 += U, tr += 4 * U) {
#pragma unroll
    for (int mm = 0; mm < U; ++mm) {
      const double E = tr[4 * mm], O = tr[4 * mm + 1], EO = tr[4 * mm + 2];
      const int b = 2 * mm;  // ring base (2m mod W: m0 is a multiple of U)
      if (NC > 0) hr[(mm + NC - 1) % U] = w[(b + 2 * NC - 2) % W] + w[(b + 2 * NC - 1) % W];
#pragma unroll
      for (int i = 0; i < NA; ++i) A[i] = fma(E, w[(b + 2 * i) % W], A[i]);
#pragma unroll
      for (int i = 0; i < NB; ++i) Bo[i] = fma(O, w[(b + 2 * i + 1) % W], Bo[i]);
#pragma unroll
      for (int i = 0; i < NC; ++i) C[i] = fma(EO, hr[(mm + i) % U], C[i]);
      w[b % W] = g[2 * (m0 + mm) + W];
      w[(b + 1) % W] = g[2 * (m0 + mm) + W + 1];
    }
  }
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    f[2 * i] = A[i] + Bo[i];
    f[2 * i + 1] = (C[i] - A[i]) - Bo[i + 1];
  }
  f[CW - 1] = A[NP] + Bo[NP];
}

// v_readlane of a double at a wave-uniform lane index
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// The correlation by summation by parts over the walk's z_ref changes.  With S_j = Σ_{j'≥j} k_j'
// and d_m = z_ref[m+1] − z_ref[m],
//   f_t = Σ_j k_j z_ref[t+1+j] = S_0 z_ref[t+1] + Σ_{j=1}^{N−1} S_j d_{t+j},
// and the CoP references the footstep generators produce (cop_generator.py:34-115: one box per
// support phase) are piecewise constant, so d is zero except at the support-phase switches —
// ≈16 changes per axis in a 420-sample default.json walk against 150 taps per output.  The wave
// finds its axis's changes with one ballot per chunk column (lane l tests m = l·CW + q), then
// walks the set bits: every lane adds S_{m−t}·d_m to its CW outputs t (Ts = the plan's ksum
// table staged in LDS; entries outside 1 ≤ j ≤ N−1 are zero, so lanes the change does not reach
// read zeros at a clamped offset).  Exact for any input; a wave whose axis changes more than
// kSparseMax times (dense bounds) returns false and takes the dense form instead.  Rounding
// differs from the direct sum by ≈ε·Σ|S_j d_j| (test_sparse_correlation_equals_dense).
constexpr int kSparseMax = 40;

template <int CW>
__device__ __forceinline__ bool axis_correlate_sparse(const RolloutArgs& a, const double* zr,
                                                      const double* Ts, int lane, double* f) {
  using ZL = ZrLayout<CW>;
  const double* z = zr + ZL::idx(lane * CW);
  double gv[CW + 1], d[CW];
  unsigned long long mk[CW];
  int cnt = 0;
#pragma unroll
  for (int j = 0; j <= CW; ++j) gv[j] = z[ZL::idx(j)];
#pragma unroll
  for (int q = 0; q < CW; ++q) {
    d[q] = gv[q + 1] - gv[q];
    mk[q] = __ballot(d[q] != 0.0);
    cnt += __popcll(mk[q]);
  }
  if (cnt > kSparseMax) return false;
  const int N = a.hN, s = lane * CW;
  const double S0 = Ts[ksum_s0(N)];
#pragma unroll
  for (int r = 0; r < CW; ++r) f[r] = S0 * gv[r + 1];
#pragma unroll
  for (int q = 0; q < CW; ++q) {
    unsigned long long m = mk[q];
    while (m) {
      const int L = __builtin_ctzll(m);
      m &= m - 1;
      const double dv = readlane_f64(d[q], L);
      // f_{s+r} += S_{e−r} d with e = m − s, S_{e−r} = Ts[e − r + 8]
      const int e = min(max(L * CW + q - s, 0), N + CW - 1);
      const double* p = Ts + e + 9 - CW;
#pragma unroll
      for (int r = 0; r < CW; ++r) f[r] = fma(p[CW - 1 - r], dv, f[r]);
    }
  }
  return true;
}

// Split-axis kernel, one walk per 128-thread workgroup: wave 0 solves the x axis and wave 1 the
// y axis (half the registers and twice the waves of the one-wave kernel, for latency hiding);
// they share the staged z_ref and the history staging rows, so loads and stores stay whole-walk
// coalesced.  The fewest serial steps: every global load (bounds, the last sample for the window
// padding, x0, kick) issued up front, z_ref + padding in one pass, one replay writing the whole
// walk's history rows into the dead z_ref area (LDS sized for it), and one coalesced copy-out —
// three barriers per walk.  The tables read on wave-uniform addresses come in as __restrict__
// pointers so the compiler keeps them on scalar loads even inside a loop that stores the history.
// SHF: shared CoP, f precomputed once per launch (zmpc_shared_f_kernel).
// PM (the persistent kernel): the walk's global loads and its history copy-out are issued at
// raised wave priority, so a CU's co-resident walks get their memory traffic out ahead of the
// others' correlation (config 2: 45.3 → 43.8 µs; the one-walk-per-workgroup grid is not helped).
// FFA: odd chunk widths take the two-parallel fast-FIR form of the dense correlation.
template <int CW, bool SHF, bool PM, bool FFA>
__device__ __forceinline__ void split_walk(const RolloutArgs& a, int64_t b, double* smem,
                                           int* flag, const double* __restrict__ kg,
                                           const double* __restrict__ scanP,
                                           const double* __restrict__ kxp,
                                           double* __restrict__ hist) {
  using ZL = ZrLayout<CW>;
  const int tid = threadIdx.x, lane = tid & 63, axis = tid >> 6;
  const int n = a.n, nsteps = n - 1;
  double f[CW];
  double pf0 = 0.0, pf1 = 0.0;  // prefetch results (kept alive to the end, never used)
  tl_stamp(a, b, 0);
  const double* xb = a.x0 + b * 6 + 3 * axis;
  const double xi[3] = {xb[0], xb[1], xb[2]};
  const double kk = (axis == 1 && a.kick != nullptr) ? a.kick[b] : 0.0;
  if constexpr (SHF) {
    // shared CoP: f of this lane's timesteps, computed once per launch (zmpc_shared_f_kernel)
    const double* fp = a.fsh + axis * a.fstride + lane * CW;
#pragma unroll
    for (int q = 0; q < CW; ++q) f[q] = fp[q];
  } else {
    double* zr0 = smem;
    double* zr1 = zr0 + a.lzp;
    // ---- 1. loads --------------------------------------------------------------------------
    if constexpr (PM) __builtin_amdgcn_s_setprio(3);  // issue the walk's loads first
    AxisBounds<CW> r;
    axis_load<CW>(a, b, tid, r);
    const double2 hl = reinterpret_cast<const double2*>(a.zmax + b * a.bstride)[n - 1];
    const double2 ll = reinterpret_cast<const double2*>(a.zmin + b * a.bstride)[n - 1];
    // the plan's suffix-sum table (sparse-difference correlation) behind the two z_ref areas
    double* Ts = smem + 2 * a.lzp;
    if (a.ksum != nullptr)
      for (int i = tid; i < ksum_rows(a.hN); i += 128) Ts[i] = a.ksum[i];
    // the bounds of the walk the next dispatch round puts on this slot, one double per 64 B
    // (threads 0..63 z_max, 64..127 z_min; two loads cover n ≤ 512 samples), so that round's
    // loads hit L2 / Infinity Cache instead of HBM under this round's compute (issued after the
    // walk's own loads have landed it gained nothing: 29.9 vs 29.5 µs, profiles/r3pf2/)
    if (a.pf_ahead > 0 && b + a.pf_ahead < a.B) {
      const double* src = (tid < 64 ? a.zmax : a.zmin) + (b + a.pf_ahead) * a.bstride;
      const int ln = tid & 63, nd = 2 * n;
      pf0 = src[min(ln * 8, nd - 1)];
      pf1 = src[min(ln * 8 + 512, nd - 1)];
    }
    if constexpr (PM) __builtin_amdgcn_s_setprio(0);
    // ---- 2. z_ref rows + window padding (zmp_controller.py:81-88) --------------------------
#pragma unroll
    for (int u = 0; u < AxisBounds<CW>::PF2; ++u) {
      const int t = u * 128 + tid;
      if (t < n) {
        zr0[ZL::idx(t)] = (r.hi[u].x + r.lo[u].x) / 2;
        zr1[ZL::idx(t)] = (r.hi[u].y + r.lo[u].y) / 2;
      }
    }
    {
      const double l0 = (hl.x + ll.x) / 2, l1 = (hl.y + ll.y) / 2;
      for (int t = n + tid; t < a.lz; t += 128) {
        zr0[ZL::idx(t)] = l0;
        zr1[ZL::idx(t)] = l1;
      }
    }
    __syncthreads();
    tl_stamp(a, b, 1);
    // ---- 3. correlation (this wave's axis) -------------------------------------------------
    // sparse z_ref differences (piecewise-constant CoP) first, else the dense forms
    const bool sparse = a.ksum != nullptr && !dbgb(a, 1) &&
                        axis_correlate_sparse<CW>(a, axis ? zr1 : zr0, Ts, lane, f);
    if (sparse) {
    } else if constexpr (FFA && (CW & 1))
      axis_correlate_ffa<CW>(a, kg, axis ? zr1 : zr0, lane, f);  // kg = the fast-FIR taps
    else
      axis_correlate<CW>(a, kg, axis ? zr1 : zr0, lane, f);  // k: wave-uniform scalar loads
    __syncthreads();  // z_ref dead: the area becomes the history staging (n rows of 6)
    tl_stamp(a, b, 2);
  }
  // ---- 4. lane-chunk affine scan -----------------------------------------------------------
  const int64_t kick_step = (axis == 1) ? kick_step_of(a, b) : -1;
  const LipmConsts lc = a.lc;
  const double kx0 = kxp[0], kx1 = kxp[1], kx2 = kxp[2];
  const int mbeg = lane * CW;
  double sv[3] = {0.0, 0.0, 0.0};
  {
    // the chunk's end state from a zero start as one sum, Σ_q Ā^(CW−1−q) B f_q (plan columns;
    // 3 FMAs per step instead of the 12 of the recursion), plus the kick's −kk Ā^(CW−1−q) e1.
    // Steps past nsteps count too: only lanes whose chunk holds no output follow such a lane.
    const double* Gc = scanP + kScanGOff;
#pragma unroll
    for (int q = 0; q < CW; ++q) {
      const double* gq = Gc + (CW - 1 - q) * 6;
#pragma unroll
      for (int i = 0; i < 3; ++i) sv[i] = fma(gq[i], f[q], sv[i]);
    }
    const int64_t qk = kick_step - mbeg;
    if (qk >= 0 && qk < CW && kick_step < nsteps) {
      const double* ek = Gc + (CW - 1 - (int)qk) * 6 + 3;
#pragma unroll
      for (int i = 0; i < 3; ++i) sv[i] = fma(-kk, ek[i], sv[i]);
    }
  }
  const double* Pp = scanP + (CW - 1) * kScanStride;  // (Ā^CW)^(2^r), r = 0..5, from the plan
  if (lane == 0) {
    double t[3];
    Mat3 P;
#pragma unroll
    for (int q = 0; q < 9; ++q) P.m[q] = Pp[q];
    matvec3(P, xi, t);
    for (int i = 0; i < 3; ++i) sv[i] += t[i];
  }
  if (!dbgb(a, 2)) scan_dpp(sv, lane, Pp, scanP + kScanPowOff + (CW - 1) * 33 * 9);
  double x[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double p = dpp_f64<0x138, 0xF>(sv[i]);  // wave_shr:1
    x[i] = (lane == 0) ? xi[i] : p;
  }
  // ---- 5. replay (reference form) straight into the staged history ------------------------
  double* stage = smem;
  if (lane == 0) {
    stage[3 * axis + 0] = xi[0];
    stage[3 * axis + 1] = xi[1];
    stage[3 * axis + 2] = xi[2];
  }
#pragma unroll
  for (int q = 0; q < CW; ++q) {
    const int m = mbeg + q;
    if (m < nsteps) {
      const double u = f[q] - (kx0 * x[0] + kx1 * x[1] + kx2 * x[2]);
      double xn[3];
      lipm_step(lc, x, u, xn);
      if (m == kick_step) xn[1] -= kk;  // force kick (zmp_controller.py:90,105-106)
      double* o = stage + HistLayout<CW>::row(m + 1) + 3 * axis;
      o[0] = xn[0];
      o[1] = xn[1];
      o[2] = xn[2];
#pragma unroll
      for (int i = 0; i < 3; ++i) x[i] = xn[i];
    }
  }
  if (a.status != nullptr) {
    const bool finite = isfinite(x[0]) && isfinite(x[1]) && isfinite(x[2]);
    const unsigned long long bad = __ballot(!finite);
    if (lane == 0) flag[axis] = bad ? ZMPC_ST_NONFINITE : 0;
  }
  __syncthreads();
  tl_stamp(a, b, 3);
  // ---- 6. coalesced copy-out ---------------------------------------------------------------
  if (!dbgb(a, 4)) {
    if constexpr (PM) __builtin_amdgcn_s_setprio(3);
    const double2* src = reinterpret_cast<const double2*>(stage);
    double2* dst = reinterpret_cast<double2*>(hist + b * (int64_t)n * 6);
    const int ne = n * 3;
    // four rows in flight per thread (LDS reads batched ahead of the stores); the history is
    // written once and never re-read here: non-temporal stores (config 4 unconstrained
    // 0.547 → 0.497 ms in an A/B on one box; config 2 unchanged)
    int e = tid;
    if constexpr (HistLayout<CW>::kPad == 0) {
      for (; e + 3 * 128 < ne; e += 4 * 128) {
        const double2 v0 = src[e], v1 = src[e + 128], v2 = src[e + 256], v3 = src[e + 384];
        st_nt2(&dst[e], v0);
        st_nt2(&dst[e + 128], v1);
        st_nt2(&dst[e + 256], v2);
        st_nt2(&dst[e + 384], v3);
      }
      for (; e < ne; e += 128) st_nt2(&dst[e], src[e]);
    } else {
      // element e (a double2) of row r = e / 3 sits behind (r − 1) / (2·CW) pads of one double2
      auto at = [](int e2) {
        const int r = e2 / 3;
        return e2 + (r >= 1 ? (r - 1) / HistLayout<CW>::kSpan : 0) * (HistLayout<CW>::kPad / 2);
      };
      for (; e + 3 * 128 < ne; e += 4 * 128) {
        const double2 v0 = src[at(e)], v1 = src[at(e + 128)], v2 = src[at(e + 256)],
                      v3 = src[at(e + 384)];
        st_nt2(&dst[e], v0);
        st_nt2(&dst[e + 128], v1);
        st_nt2(&dst[e + 256], v2);
        st_nt2(&dst[e + 384], v3);
      }
      for (; e < ne; e += 128) st_nt2(&dst[e], src[at(e)]);
    }
    if constexpr (PM) __builtin_amdgcn_s_setprio(0);
  }
  tl_stamp(a, b, 4);
  if (a.status != nullptr && tid == 0) a.status[b] = flag[0] | flag[1];
  if (a.dbg < 0) hist[tid] = pf0 + pf1;  // never (dbg ≥ 0): keeps the prefetch loads
}

// Shared CoP (bounds stride 0, e.g. an F_ext sweep over one walk): z_ref, and so f, is the
// same for every walk, so the correlation runs once per launch — one thread per (axis,
// timestep), the taps in the per-walk kernels' order (fma chain from 0 over j = 0..kc−1) — and
// the rollout kernel reads it instead (split_walk<CW, true>); histories equal the per-walk
// kernels' to rounding (≈1e-15 relative: the compiler contracts the two kernels differently).
__global__ void __launch_bounds__(256) zmpc_shared_f_kernel(const double* __restrict__ zmax,
                                                            const double* __restrict__ zmin,
                                                            int n, const double* __restrict__ k,
                                                            int kc, double* fsh, int fstride) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // timestep
  const int axis = blockIdx.y;
  if (i >= fstride) return;
  double acc = 0.0;
  for (int j = 0; j < kc; ++j) {
    const int t = min(i + 1 + j, n - 1);  // window padding with the last row (:81-88)
    const double z = (zmax[2 * t + axis] + zmin[2 * t + axis]) / 2;
    acc = fma(k[j], z, acc);
  }
  fsh[axis * fstride + i] = acc;
}

// The persistent split kernel (grid = resident workgroups × CUs, walks strided over it): even
// chunk widths at 1–3 walks per resident slot (config 2 before the fast-FIR form: 45 vs 49 µs).
// (The tables come through the argument struct: as __restrict__ arguments they go to SGPRs
// and the DPP scan's per-lane powers push the kernel into spills.)
template <int CW>
__global__ void __launch_bounds__(128, 4)
    zmpc_rollout_unc_persd_kernel(RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ int flag[2];
  for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {
    split_walk<CW, false, true, false>(a, b, smem, flag, a.k, a.scanP, a.kx, a.hist);
    __syncthreads();  // staging read out before the next walk's z_ref overwrites it
  }
}

// One walk per workgroup (the default; odd chunk widths with the fast-FIR dense form), and the
// shared-CoP form (SHF).
template <int CW, bool SHF>
__global__ void __launch_bounds__(128, 4) zmpc_rollout_unc_splitd_kernel(RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ int flag[2];
  split_walk<CW, SHF, false, true>(a, blockIdx.x, smem, flag, (CW & 1) ? a.kffa : a.k, a.scanP,
                                   a.kx, a.hist);
}

// ---- FFT correlation (long walks) ------------------------------------------------------------
// f_i = Σ_{d=1..N} g[d] s[i+d] with g[d] = k_{d−1} and s = z_x + i z_y (both axes in one complex
// signal; g is real, so Re and Im stay separate): a circular cross-correlation of period
// P = 2^p ≥ n − 1 + N, so no output i ≤ n − 2 wraps.  Its spectrum is S·conj(DFT g); with
// T = conj(S)·DFT(g)/P (the plan's fft_g) f = conj(DFT(T)): two forward transforms.  O(P log P)
// instead of the direct form's N per output (N = 512: ≈10× fewer FP64 operations).
// Stockham autosort, radix 4 (+ one radix-2 stage when p is odd), in place in LDS: each stage
// reads all of its inputs, barrier, writes, barrier.  NT threads, E = P/NT points each.
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}

// 8-point DFT in registers, forward sign (e^{−2πi/8} = (1 − i)/√2).
__device__ __forceinline__ void dft8(double2 (&v)[8]) {
  constexpr double h = 0.70710678118654752440;  // 1/√2
  double2 a[4], c[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    a[r] = make_double2(v[r].x + v[r + 4].x, v[r].y + v[r + 4].y);
    c[r] = make_double2(v[r].x - v[r + 4].x, v[r].y - v[r + 4].y);
  }
  // c1 ·= w8, c2 ·= −i, c3 ·= w8³
  c[1] = make_double2((c[1].x + c[1].y) * h, (c[1].y - c[1].x) * h);
  c[2] = make_double2(c[2].y, -c[2].x);
  c[3] = make_double2((c[3].y - c[3].x) * h, -(c[3].x + c[3].y) * h);
  // 4-point DFTs: evens from a, odds from c
  auto dft4 = [](const double2 (&q)[4], double2& y0, double2& y1, double2& y2, double2& y3) {
    const double2 t0 = make_double2(q[0].x + q[2].x, q[0].y + q[2].y);
    const double2 t1 = make_double2(q[0].x - q[2].x, q[0].y - q[2].y);
    const double2 t2 = make_double2(q[1].x + q[3].x, q[1].y + q[3].y);
    const double2 t3 = make_double2(q[1].y - q[3].y, q[3].x - q[1].x);  // (q1 − q3)·(−i)
    y0 = make_double2(t0.x + t2.x, t0.y + t2.y);
    y2 = make_double2(t0.x - t2.x, t0.y - t2.y);
    y1 = make_double2(t1.x + t3.x, t1.y + t3.y);
    y3 = make_double2(t1.x - t3.x, t1.y - t3.y);
  };
  dft4(a, v[0], v[2], v[4], v[6]);
  dft4(c, v[1], v[3], v[5], v[7]);
}

// In-place-in-registers Stockham FFT of P = 2^p points (forward), radix 8 (+ one radix-2 or
// radix-4 stage when p mod 3 ≠ 0), by the first NF = P/8 threads of the workgroup: thread t
// holds points t + NF·u (u = 0..7) on entry and the transform's points t + NF·u on exit, so
// the first stage reads and the last stage writes registers; between stages the points pass
// through LDS (buf, P complex).  Every thread of the workgroup must call it (barriers).
template <int P>
__device__ __forceinline__ void fft8(double2 (&v)[8], double2* buf,
                                     const double2* __restrict__ tw, int tid) {
  constexpr int NF = P / 8;
  constexpr int LOGP = __builtin_ctz(P);
  constexpr int A8 = LOGP / 3;  // radix-8 stages
  constexpr int RL = LOGP % 3;  // last stage radix 2^RL (0: none)
  constexpr int R = 1 << RL;
  const bool act = tid < NF;
#pragma unroll
  for (int st = 0; st < A8; ++st) {
    const int Ns = 1 << (3 * st);
    const int k = tid & (Ns - 1);
    if (act) {
      if (st > 0) {
        const double2 w1 = tw[k * (kFftPT / (8 * Ns))];
        const double2 w2 = cmul(w1, w1), w3 = cmul(w2, w1), w4 = cmul(w2, w2);
        v[1] = cmul(v[1], w1);
        v[2] = cmul(v[2], w2);
        v[3] = cmul(v[3], w3);
        v[4] = cmul(v[4], w4);
        v[5] = cmul(v[5], cmul(w4, w1));
        v[6] = cmul(v[6], cmul(w4, w2));
        v[7] = cmul(v[7], cmul(w4, w3));
      }
      dft8(v);
    }
    const bool last = (st == A8 - 1) && RL == 0;
    if (!last) {
      if (act) {
        const int base = ((tid - k) << 3) + k;
#pragma unroll
        for (int r = 0; r < 8; ++r) buf[base + r * Ns] = v[r];
      }
      __syncthreads();
      if (act) {
        if (st + 1 < A8) {
#pragma unroll
          for (int r = 0; r < 8; ++r) v[r] = buf[tid + r * NF];
        } else {
          // the radix-R stage: butterflies j = tid + NF·m (m < 8/R), inputs j + r·P/R
#pragma unroll
          for (int m = 0; m < 8 / R; ++m)
#pragma unroll
            for (int r = 0; r < R; ++r) v[m * R + r] = buf[tid + NF * m + r * (P / R)];
        }
      }
      __syncthreads();
    }
  }
  if constexpr (RL > 0) {
    // last stage (Ns = P/R, k = j): twiddles w^{r j}, w = e^{−2πi/P}; outputs j + r·P/R =
    // tid + NF·(m + r·8/R)
    double2 y[8];
    if (act) {
#pragma unroll
      for (int m = 0; m < 8 / R; ++m) {
        const int j = tid + NF * m;
        const double2 w1 = tw[j * (kFftPT / P)];
        double2 q[4];
#pragma unroll
        for (int r = 0; r < R; ++r) q[r] = v[m * R + r];
        if constexpr (R == 2) {
          q[1] = cmul(q[1], w1);
          y[m] = make_double2(q[0].x + q[1].x, q[0].y + q[1].y);
          y[m + 4] = make_double2(q[0].x - q[1].x, q[0].y - q[1].y);
        } else {
          const double2 w2 = cmul(w1, w1), w3 = cmul(w2, w1);
          q[1] = cmul(q[1], w1);
          q[2] = cmul(q[2], w2);
          q[3] = cmul(q[3], w3);
          const double2 t0 = make_double2(q[0].x + q[2].x, q[0].y + q[2].y);
          const double2 t1 = make_double2(q[0].x - q[2].x, q[0].y - q[2].y);
          const double2 t2 = make_double2(q[1].x + q[3].x, q[1].y + q[3].y);
          const double2 t3 = make_double2(q[1].y - q[3].y, q[3].x - q[1].x);
          y[m] = make_double2(t0.x + t2.x, t0.y + t2.y);
          y[m + 2] = make_double2(t1.x + t3.x, t1.y + t3.y);
          y[m + 4] = make_double2(t0.x - t2.x, t0.y - t2.y);
          y[m + 6] = make_double2(t1.x - t3.x, t1.y - t3.y);
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = y[u];
    }
  }
}

// s (points t + NF·u in v, NF = P/8 threads) → f = conj(DFT(conj(DFT s)·G)) into buf (P complex,
// natural order), G = the plan's DFT(g)/P.  Every thread of the workgroup must call it.
template <int P>
__device__ __forceinline__ void fft_correlate8(double2 (&v)[8], double2* buf,
                                               const double2* __restrict__ tw,
                                               const double2* __restrict__ G, int tid) {
  constexpr int NF = P / 8;
  fft8<P>(v, buf, tw, tid);
  if (tid < NF) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const double2 S = v[u], g = G[tid + NF * u];
      v[u] = make_double2(fma(S.x, g.x, S.y * g.y), fma(S.x, g.y, -S.y * g.x));  // conj(S)·g
    }
  }
  __syncthreads();  // the last exchange's reads are done before buf is rewritten
  fft8<P>(v, buf, tw, tid);
  if (tid < NF) {
#pragma unroll
    for (int u = 0; u < 8; ++u) buf[tid + NF * u] = v[u];
  }
  __syncthreads();
}

// The sparse-difference correlation (axis_correlate_sparse) for the wide kernel: the changes a
// lane's outputs need lie up to N − 1 samples ahead, in other waves' ranges, so each axis's
// changes go to an LDS list first (per-wave counts → prefix → positions, deterministic order)
// and every lane walks its axis's list.  Returns false, uniformly over the workgroup, when
// either axis has more than kSparseMaxWide changes (both axes then take the dense form: the FFT
// correlates them together).  Both calls' barriers are reached by every thread.
constexpr int kSparseMaxWide = 64;

template <int CW, int W>
__device__ __forceinline__ bool wide_correlate_sparse(const RolloutArgs& a, const double* zr,
                                                      const double* Ts, double* ld, int* lm,
                                                      int (*scnt)[W], int axis, int w, int lane,
                                                      double* f) {
  using ZL = ZrLayout<CW>;
  const int s = (w * 64 + lane) * CW;
  const double* z = zr + ZL::idx(s);
  double gv[CW + 1], d[CW];
  unsigned long long mk[CW];
  int cnt = 0;
#pragma unroll
  for (int j = 0; j <= CW; ++j) gv[j] = z[ZL::idx(j)];
#pragma unroll
  for (int q = 0; q < CW; ++q) {
    d[q] = gv[q + 1] - gv[q];
    mk[q] = __ballot(d[q] != 0.0);
    cnt += __popcll(mk[q]);
  }
  if (lane == 0) scnt[axis][w] = cnt;
  __syncthreads();
  int tot0 = 0, tot1 = 0, base = 0;
#pragma unroll
  for (int v = 0; v < W; ++v) {
    tot0 += scnt[0][v];
    tot1 += scnt[1][v];
    if (v < w) base += scnt[axis][v];
  }
  if (tot0 > kSparseMaxWide || tot1 > kSparseMaxWide || dbgb(a, 1)) return false;
  const unsigned long long lt = (1ull << lane) - 1ull;
  double* la = ld + axis * kSparseMaxWide;
  int* lma = lm + axis * kSparseMaxWide;
#pragma unroll
  for (int q = 0; q < CW; ++q) {
    if ((mk[q] >> lane) & 1ull) {
      const int pos = base + __popcll(mk[q] & lt);
      la[pos] = d[q];
      lma[pos] = s + q;
    }
    base += __popcll(mk[q]);
  }
  __syncthreads();
  const int N = a.hN, tot = axis ? tot1 : tot0;
  const double S0 = Ts[ksum_s0(N)];
#pragma unroll
  for (int r = 0; r < CW; ++r) f[r] = S0 * gv[r + 1];
  for (int c = 0; c < tot; ++c) {
    const int e = min(max(lma[c] - s, 0), N + CW - 1);
    const double dv = la[c];
    const double* p = Ts + e + 9 - CW;
#pragma unroll
    for (int r = 0; r < CW; ++r) f[r] = fma(p[CW - 1 - r], dv, f[r]);
  }
  return true;
}

// LDS doubles the wide kernel's sparse attempt adds behind the two z_ref areas: the suffix-sum
// table, the two change lists (values, then int positions)
__host__ __device__ constexpr int wide_sparse_doubles(int N) {
  return ((ksum_rows(N) + 1) & ~1) + 2 * kSparseMaxWide + kSparseMaxWide;
}

// Long walks (64·8+1 < n ≤ 64·8·8+1): the split-axis structure widened to W waves per axis
// (workgroup = 2·W waves; wave w of an axis owns timesteps [w·64·CW, (w+1)·64·CW)).  Each
// wave scans its range from a zero state; the true start state of wave w is chained over the
// waves' end states with M = (Ā^CW)^64 (plan level 6), and lane l adds (Ā^CW)^(l+1)·x_start by
// binary powering.  History staged through the z_ref area in rounds (replay per round).
template <int CW, int W, int E = 0>
__global__ void __launch_bounds__(128 * W, E == 4 ? 6 : 4) zmpc_rollout_unc_wide_kernel(RolloutArgs a) {
  using ZL = ZrLayout<CW>;
  constexpr int NT = 128 * W;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ int flag[2 * W];
  __shared__ double send[2][W][3];  // zero-start end state of each wave (wave 0: true)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int axis = wv / W, w = wv % W;
  const int64_t b = blockIdx.x;
  const int n = a.n, nsteps = n - 1;
  double* zr0 = smem;
  double* zr1 = zr0 + a.lzp;
  __shared__ int scnt[2][W];  // per-wave z_ref change counts (sparse attempt)
  // (diagnostics timeline: [0] start, [1] correlation inputs staged, [2] correlation done,
  // [3] scan and cross-wave chain done, [4] last copy-out issued)
  tl_stamp(a, b, 0);
  double* Ts = smem + 2 * a.lzp;  // sparse attempt: suffix sums, then the change lists
  double* ld = Ts + ((ksum_rows(a.hN) + 1) & ~1);
  int* lm = reinterpret_cast<int*>(ld + 2 * kSparseMaxWide);
  // ---- 1. z_ref rows + window padding (zmp_controller.py:81-88) ----------------------------
  double f[CW];
  const int mbeg = (w * 64 + lane) * CW;
  // next-dispatch-round prefetch (as split_walk): one double per 64 B of walk b + pf_ahead's
  // bounds, results kept alive to the end and never used
  double pf0 = 0.0, pf1 = 0.0;
  if (a.pf_ahead > 0 && b + a.pf_ahead < a.B) {
    const int nd = 2 * n, half = NT / 2, tl = tid % half;
    const double* src = (tid < half ? a.zmax : a.zmin) + (b + a.pf_ahead) * a.bstride;
    pf0 = src[min(tl * 8, nd - 1)];
    pf1 = src[min((tl + half) * 8, nd - 1)];
  }
  // the sparse-difference correlation first (piecewise-constant CoP), else the dense forms;
  // the FFT form stages only the rows the change scan reads (its transform loads its own)
  bool dense = true;
  if constexpr (E > 0) {
    if (a.ksum != nullptr) {
      const double2* zmx = reinterpret_cast<const double2*>(a.zmax + b * a.bstride);
      const double2* zmn = reinterpret_cast<const double2*>(a.zmin + b * a.bstride);
      // the bound loads issued GB rows per thread at a time ahead of their LDS stores (one HBM
      // round trip per group instead of per row; two-row groups at CW ≥ 7, whose state would
      // spill at four)
      constexpr int lzs = W * 64 * CW + 1, IT = (lzs + NT - 1) / NT, GB = CW >= 7 ? 2 : 4;
#pragma unroll
      for (int u0 = 0; u0 < IT; u0 += GB) {
        double2 hi[GB], lo[GB];
#pragma unroll
        for (int u = 0; u < GB; ++u) {
          const int tc = min(tid + (u0 + u) * NT, n - 1);  // padding = last row
          hi[u] = zmx[tc];
          lo[u] = zmn[tc];
        }
        if (u0 == 0)
          for (int i = tid; i < ksum_rows(a.hN); i += NT) Ts[i] = a.ksum[i];
#pragma unroll
        for (int u = 0; u < GB; ++u) {
          const int t = tid + (u0 + u) * NT;
          if (u0 + u < IT && t < lzs) {
            zr0[ZL::idx(t)] = (hi[u].x + lo[u].x) / 2;
            zr1[ZL::idx(t)] = (hi[u].y + lo[u].y) / 2;
          }
        }
      }
      __syncthreads();
      tl_stamp(a, b, 1);
      dense = !wide_correlate_sparse<CW, W>(a, axis ? zr1 : zr0, Ts, ld, lm, scnt, axis, w, lane,
                                             f);
    }
  }
  if (!dense) {
  } else if constexpr (E > 0) {
    // FFT correlation: s[t] = (z_x, z_y) for t < P (rows past n − 1: the last row)
    double2* buf = reinterpret_cast<double2*>(smem);
    const double2* zmx = reinterpret_cast<const double2*>(a.zmax + b * a.bstride);
    const double2* zmn = reinterpret_cast<const double2*>(a.zmin + b * a.bstride);
    constexpr int P = NT * E, NF = P / 8;  // the first NF threads run the transform
    double2 v[8];
    if (tid < NF) {
      double2 hi[8], lo[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int tc = min(tid + NF * u, n - 1);
        hi[u] = zmx[tc];
        lo[u] = zmn[tc];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = make_double2((hi[u].x + lo[u].x) / 2, (hi[u].y + lo[u].y) / 2);
    }
    fft_correlate8<P>(v, buf, a.fft_tw, a.fft_g, tid);
#pragma unroll
    for (int q = 0; q < CW; ++q) {
      const double2 c = buf[min(mbeg + q, NT * E - 1)];
      f[q] = axis ? -c.y : c.x;  // f = conj(DFT T): f_y = −Im
    }
  } else {
    const double2* zmx = reinterpret_cast<const double2*>(a.zmax + b * a.bstride);
    const double2* zmn = reinterpret_cast<const double2*>(a.zmin + b * a.bstride);
    for (int t0 = 0; t0 < a.lz; t0 += 4 * NT) {
      double2 hi[4], lo[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int tc = dbgb(a, 8) ? 0 : min(t0 + u * NT + tid, n - 1);  // padding = last row
        hi[u] = zmx[tc];
        lo[u] = zmn[tc];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + u * NT + tid;
        if (t < a.lz) {
          zr0[ZL::idx(t)] = (hi[u].x + lo[u].x) / 2;
          zr1[ZL::idx(t)] = (hi[u].y + lo[u].y) / 2;
        }
      }
    }
    if (a.ksum != nullptr)
      for (int i = tid; i < ksum_rows(a.hN); i += NT) Ts[i] = a.ksum[i];
    __syncthreads();
    // ---- 2. correlation ----------------------------------------------------------------------
    if (a.ksum == nullptr ||
        !wide_correlate_sparse<CW, W>(a, axis ? zr1 : zr0, Ts, ld, lm, scnt, axis, w, lane, f))
      axis_correlate<CW>(a, a.k, (axis ? zr1 : zr0) + ZL::idx(w * 64 * CW), lane, f);
  }
  tl_stamp(a, b, 2);
  const double* xb = a.x0 + b * 6 + 3 * axis;
  const double xi[3] = {xb[0], xb[1], xb[2]};
  const double kk = (axis == 1 && a.kick != nullptr) ? a.kick[b] : 0.0;
  // ---- 3. scan: per-wave zero-start Kogge-Stone, then the cross-wave offsets ---------------
  const int64_t kick_step = (axis == 1) ? kick_step_of(a, b) : -1;
  const LipmConsts lc = a.lc;
  const double kx0 = a.kx[0], kx1 = a.kx[1], kx2 = a.kx[2];
  const double Bv[3] = {lc.T3_6, lc.T2_2, lc.T};
  Mat3 Ab;
  {
    const double A[9] = {1.0, lc.T, lc.T2_2, 0.0, 1.0, lc.T, 0.0, 0.0, 1.0};
    const double kx[3] = {kx0, kx1, kx2};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) Ab.m[3 * i + j] = A[3 * i + j] - Bv[i] * kx[j];
  }
  double sv[3] = {0.0, 0.0, 0.0};
#pragma unroll
  for (int q = 0; q < CW; ++q) {
    if (mbeg + q < nsteps) {
      double t[3];
      matvec3(Ab, sv, t);
      sv[0] = fma(Bv[0], f[q], t[0]);
      sv[1] = fma(Bv[1], f[q], t[1]);
      sv[2] = fma(Bv[2], f[q], t[2]);
      if (mbeg + q == kick_step) sv[1] -= kk;
    }
  }
  const double* Pp = a.scanP + (CW - 1) * kScanStride;  // (Ā^CW)^(2^r), r = 0..6
  if (lane == 0 && w == 0) {
    double t[3];
    Mat3 P;
#pragma unroll
    for (int q = 0; q < 9; ++q) P.m[q] = Pp[q];
    matvec3(P, xi, t);
    for (int i = 0; i < 3; ++i) sv[i] += t[i];
  }
  // (the 6-waves-per-SIMD FFT instances at CW ≥ 7 keep the shuffle scan and binary powering:
  // the DPP scan's per-lane powers would spill them, 12–36 B)
  constexpr bool kShflScan = E == 4 && CW >= 7;
  if constexpr (kShflScan) {
#pragma unroll
    for (int r2 = 0; r2 < 6; ++r2) {
      const int d = 1 << r2;
      if (dbgb(a, 2)) break;
      double u[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) u[i] = __shfl_up(sv[i], d, 64);
      if (lane >= d) {
        Mat3 Pd;
#pragma unroll
        for (int q = 0; q < 9; ++q) Pd.m[q] = Pp[r2 * 9 + q];
        double t[3];
        matvec3(Pd, u, t);
        for (int i = 0; i < 3; ++i) sv[i] += t[i];
      }
    }
  } else if (!dbgb(a, 2)) {
    scan_dpp(sv, lane, Pp, a.scanP + kScanPowOff + (CW - 1) * 33 * 9);
  }
  if (lane == 63) {
    send[axis][w][0] = sv[0];
    send[axis][w][1] = sv[1];
    send[axis][w][2] = sv[2];
  }
  __syncthreads();  // end states published; z_ref dead (staging from here on)
  double xs[3] = {xi[0], xi[1], xi[2]};  // this wave's start state
  if (w > 0) {
    Mat3 M64;
#pragma unroll
    for (int q = 0; q < 9; ++q) M64.m[q] = Pp[6 * 9 + q];
    for (int i = 0; i < 3; ++i) xs[i] = send[axis][0][i];
    for (int v = 1; v < w; ++v) {
      double t[3];
      matvec3(M64, xs, t);
      for (int i = 0; i < 3; ++i) xs[i] = send[axis][v][i] + t[i];
    }
    // lane l adds (Ā^CW)^(l+1)·x_start: the plan's per-lane powers k ≤ 32, times (Ā^CW)^32
    // (scan level 5) first for lanes 32..63
    double vv[3] = {xs[0], xs[1], xs[2]};
    int e = lane + 1;
    if constexpr (kShflScan) {  // binary powering over the scan levels
#pragma unroll
      for (int r2 = 0; r2 < 7; ++r2) {
        if ((e >> r2) & 1) {
          Mat3 Pd;
#pragma unroll
          for (int q = 0; q < 9; ++q) Pd.m[q] = Pp[r2 * 9 + q];
          double t[3];
          matvec3(Pd, vv, t);
          for (int i = 0; i < 3; ++i) vv[i] = t[i];
        }
      }
      for (int i = 0; i < 3; ++i) sv[i] += vv[i];
    } else {
      if (e > 32) {
        Mat3 P32;
#pragma unroll
        for (int q = 0; q < 9; ++q) P32.m[q] = Pp[5 * 9 + q];
        double t[3];
        matvec3(P32, vv, t);
        for (int i = 0; i < 3; ++i) vv[i] = t[i];
        e -= 32;
      }
      const double* m = a.scanP + kScanPowOff + ((CW - 1) * 33 + e) * 9;
      Mat3 M;
#pragma unroll
      for (int q = 0; q < 9; ++q) M.m[q] = m[q];
      double t[3];
      matvec3(M, vv, t);
      for (int i = 0; i < 3; ++i) sv[i] += t[i];
    }
  }
  double xs0[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double p = kShflScan ? __shfl_up(sv[i], 1, 64) : dpp_f64<0x138, 0xF>(sv[i]);
    xs0[i] = (lane == 0) ? xs[i] : p;
  }
  tl_stamp(a, b, 3);
  // ---- 4. replay (reference form) into the staging rows, coalesced copy-out per round --------
  // staging rows padded as the split kernels' (HistLayout: two doubles after every CW local
  // rows, even CW), so the lanes' ds_write rows are not 128 B multiples apart
  double* stage = smem;
  constexpr int HP = HistLayout<CW>::kPad;
  constexpr int HS = HistLayout<CW>::kSpan;
  const int rows_per_round = (2 * a.lzp) * HS / (6 * HS + HP);
  auto srow = [](int lr) { return lr * 6 + HP * (lr / HS); };
  double* hb = a.hist + b * (int64_t)n * 6;
  double x[3];
  for (int r0 = 0; r0 < n; r0 += rows_per_round) {
    const int r1 = min(r0 + rows_per_round, n);
    if (lane == 0 && w == 0 && r0 == 0) {
      stage[3 * axis + 0] = xi[0];
      stage[3 * axis + 1] = xi[1];
      stage[3 * axis + 2] = xi[2];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = xs0[i];
#pragma unroll
    for (int q = 0; q < CW; ++q) {
      const int m = mbeg + q;
      if (m < nsteps) {
        const double u = f[q] - (kx0 * x[0] + kx1 * x[1] + kx2 * x[2]);
        double xn[3];
        lipm_step(lc, x, u, xn);
        if (m == kick_step) xn[1] -= kk;
        const int row = m + 1;
        if (row >= r0 && row < r1) {
          double* o = stage + srow(row - r0) + 3 * axis;
          o[0] = xn[0];
          o[1] = xn[1];
          o[2] = xn[2];
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) x[i] = xn[i];
      }
    }
    __syncthreads();
    if (!dbgb(a, 4)) {
      const int nd2 = (r1 - r0) * 3;
      const double2* src = reinterpret_cast<const double2*>(stage);
      double2* dst = reinterpret_cast<double2*>(hb + (int64_t)r0 * 6);
      for (int e = tid; e < nd2; e += NT)  // written once
        st_nt2(&dst[e], src[e + (HP / 2) * ((e / 3) / HS)]);
    }
    __syncthreads();
  }
  if (a.status != nullptr) {
    const bool finite = isfinite(x[0]) && isfinite(x[1]) && isfinite(x[2]);
    const unsigned long long bad = __ballot(!finite);
    if (lane == 0) flag[wv] = bad ? ZMPC_ST_NONFINITE : 0;
    __syncthreads();
    if (tid == 0) {
      int fl = 0;
      for (int v = 0; v < 2 * W; ++v) fl |= flag[v];
      a.status[b] = fl;
    }
  }
  tl_stamp(a, b, 4);
  if (a.dbg < 0) a.hist[tid] = pf0 + pf1;  // never (dbg ≥ 0): keeps the prefetch loads
}

// Geometry of the wide kernel: W waves per axis (2, 4 or 8), CW = ceil((n−1)/(64·W)) ≤ 8.
struct WideGeom {
  int w, cw, kc, lz, lzp;
};

#ifndef ZMPC_WIDE8  // (A/B builds only)
#define ZMPC_WIDE8 0
#endif
constexpr bool kWide8 = ZMPC_WIDE8 != 0;

// The wide kernel's dynamic-LDS ceiling: 64 KiB (the 4-waves-per-SIMD bound leaves no room above
// it for W = 2 and 4), but 159 KiB for W = 8 — a 16-wave workgroup fills a CU's wave slots at that
// bound alone, so its LDS costs no occupancy (walks of 2561..4096 samples at N >= 920 took the
// chunk kernel at 8x the time, profiles/r6fin/configs/sweep_full.jsonl).  The kernel's static LDS
// (≈0.5 KiB) comes on top: hipFuncSetAttribute refuses a dynamic limit of the full 160 KiB.
size_t wide_lds_cap(int w) { return (size_t)(w == 8 ? 159 : 64) * 1024; }

bool wide_geom(int N, int64_t n, WideGeom* g) {
  const int64_t ns = n - 1;
  // (449..512 timesteps: the single-pass split kernel's CW = 8 runs 1.7× slower per walk than
  // its CW = 7, profiles/r4/r4hp_*; the wide kernel takes them at CW = 4 per wave pair)
  if (ns <= 64 * 7 || ns > 64 * 8 * 8) return false;
  g->w = ns <= 64 * 8 * 2 ? 2 : (ns <= 64 * 8 * 4 ? 4 : 8);
  g->cw = (int)((ns + 64 * g->w - 1) / (64 * g->w));
  g->kc = (N + g->cw - 1) / g->cw * g->cw;
  g->lz = g->w * 64 * g->cw + g->kc + 1;
  const int pad = (g->cw % 2 == 0) ? 1 : 0;
  g->lzp = ((g->lz + pad * (g->lz / g->cw) + 1) + 1) & ~1;
  return (size_t)2 * g->lzp * sizeof(double) <= wide_lds_cap(g->w);
}

// Walks of any length (the fallback beyond the wide kernel's 64·8·8 + 1 samples): one wave per
// walk, the walk processed in chunks of `lc` timesteps with the two axes' states carried in
// registers from chunk to chunk, so the LDS footprint does not grow with n.  Per chunk: the
// z_ref rows it reads (t0 .. t0 + lc + kc, clamped to the last sample — the window padding of
// zmp_controller.py:81-88), the correlation passes into f (LDS), the lane-chunk affine scan
// from the carried state, and the replay in the reference form through the dead z_ref area.
template <int CW>
__device__ __forceinline__ void chunk_scan_replay(const RolloutArgs& a, int lane, const double* f0,
                                                  const double* f1, double* stage, int rows_pr,
                                                  double* xs, double* ys, double kk,
                                                  int64_t kstep, int64_t t0, int ns,
                                                  double* hb) {
  const LipmConsts lc = a.lc;
  const double kx0 = a.kx[0], kx1 = a.kx[1], kx2 = a.kx[2];
  const double Bv[3] = {lc.T3_6, lc.T2_2, lc.T};
  Mat3 Ab;  // Ā = A − B kxᵀ
  {
    const double A[9] = {1.0, lc.T, lc.T2_2, 0.0, 1.0, lc.T, 0.0, 0.0, 1.0};
    const double kx[3] = {kx0, kx1, kx2};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) Ab.m[3 * i + j] = A[3 * i + j] - Bv[i] * kx[j];
  }
  const int C = (ns + 63) / 64;  // steps per lane chunk
  const int mbeg = lane * C, mend = min(mbeg + C, ns);
  // zero-start composition of the lane's steps, then Kogge-Stone with P = Ā^C
  double s0[3] = {0.0, 0.0, 0.0}, s1[3] = {0.0, 0.0, 0.0};
  for (int m = mbeg; m < mend; ++m) {
    double t[3];
    matvec3(Ab, s0, t);
    for (int i = 0; i < 3; ++i) s0[i] = fma(Bv[i], f0[m], t[i]);
    matvec3(Ab, s1, t);
    for (int i = 0; i < 3; ++i) s1[i] = fma(Bv[i], f1[m], t[i]);
    if (t0 + m == kstep) s1[1] -= kk;
  }
  Mat3 P = Ab;
  for (int q = 1; q < C; ++q) P = matmul3(P, Ab);
  if (lane == 0) {
    double t[3];
    matvec3(P, xs, t);
    for (int i = 0; i < 3; ++i) s0[i] += t[i];
    matvec3(P, ys, t);
    for (int i = 0; i < 3; ++i) s1[i] += t[i];
  }
  Mat3 Pd = P;
  for (int d = 1; d < 64; d <<= 1) {
    double u0[3], u1[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      u0[i] = __shfl_up(s0[i], d, 64);
      u1[i] = __shfl_up(s1[i], d, 64);
    }
    if (lane >= d) {
      double t[3];
      matvec3(Pd, u0, t);
      for (int i = 0; i < 3; ++i) s0[i] += t[i];
      matvec3(Pd, u1, t);
      for (int i = 0; i < 3; ++i) s1[i] += t[i];
    }
    Pd = matmul3(Pd, Pd);
  }
  double xb0[3], yb0[3];  // state at the start of this lane's steps
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double p0 = __shfl_up(s0[i], 1, 64);
    const double p1 = __shfl_up(s1[i], 1, 64);
    xb0[i] = (lane == 0) ? xs[i] : p0;
    yb0[i] = (lane == 0) ? ys[i] : p1;
  }
  // replay x⁺ = A x + B u (zmp_controller.py:199) in rounds of staged rows t0+1 .. t0+ns
  double x[3], y[3];
  for (int r0 = 0; r0 < ns; r0 += rows_pr) {
    const int r1 = min(r0 + rows_pr, ns);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      x[i] = xb0[i];
      y[i] = yb0[i];
    }
    for (int m = mbeg; m < mend; ++m) {
      const double ux = f0[m] - (kx0 * x[0] + kx1 * x[1] + kx2 * x[2]);
      const double uy = f1[m] - (kx0 * y[0] + kx1 * y[1] + kx2 * y[2]);
      double xn[3], yn[3];
      lipm_step(lc, x, ux, xn);
      lipm_step(lc, y, uy, yn);
      if (t0 + m == kstep) yn[1] -= kk;  // F_ext impulse (:105-106)
      if (m >= r0 && m < r1) {
        double* o = stage + (m - r0) * 6;
        o[0] = xn[0];
        o[1] = xn[1];
        o[2] = xn[2];
        o[3] = yn[0];
        o[4] = yn[1];
        o[5] = yn[2];
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        x[i] = xn[i];
        y[i] = yn[i];
      }
    }
    __syncthreads();
    const double2* src = reinterpret_cast<const double2*>(stage);
    double2* dst = reinterpret_cast<double2*>(hb + (t0 + r0 + 1) * 6);
    for (int e = lane; e < (r1 - r0) * 3; e += 64) st_nt2(&dst[e], src[e]);
    __syncthreads();
  }
  // carry the chunk's end state: the lane that ran step ns − 1
  const int last = (ns - 1) / C;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    xs[i] = __shfl(x[i], last, 64);
    ys[i] = __shfl(y[i], last, 64);
  }
}

template <int CW>
__global__ void __launch_bounds__(64) zmpc_rollout_unc_chunk_kernel(RolloutArgs a, int lc) {
  using ZL = ZrLayout<CW>;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = a.n;
  const int64_t nsteps = n - 1;
  double* ks = smem;
  double* zr0 = smem + a.kcp;
  double* zr1 = zr0 + a.lzp;
  double* f0 = zr1 + a.lzp;
  double* f1 = f0 + lc;
  const int rows_pr = (2 * a.lzp) / 6;  // history rows per staging round (z_ref area)
  for (int j = lane; j < a.kcp; j += 64) ks[j] = a.k[j];
  const double2* zmx = reinterpret_cast<const double2*>(a.zmax + b * a.bstride);
  const double2* zmn = reinterpret_cast<const double2*>(a.zmin + b * a.bstride);
  const double* xb = a.x0 + b * 6;
  double xs[3] = {xb[0], xb[1], xb[2]}, ys[3] = {xb[3], xb[4], xb[5]};
  const double kk = (a.kick != nullptr) ? a.kick[b] : 0.0;
  const int64_t kstep = kick_step_of(a, b);
  double* hb = a.hist + b * (int64_t)n * 6;
  if (lane < 6) hb[lane] = xb[lane];  // row 0 = x0
  for (int64_t t0 = 0; t0 < nsteps; t0 += lc) {
    const int ns = (int)min((int64_t)lc, nsteps - t0);
    const int passes = (ns + 64 * CW - 1) / (64 * CW);
    const int lz = passes * 64 * CW + a.kc + 1;
    __syncthreads();  // the previous chunk's staging rows are out
    for (int t = lane; t < lz; t += 64) {
      const int64_t row = min(t0 + t, (int64_t)n - 1);
      const double2 h = zmx[row], l = zmn[row];
      zr0[ZL::idx(t)] = (h.x + l.x) / 2;
      zr1[ZL::idx(t)] = (h.y + l.y) / 2;
    }
    __syncthreads();
    for (int pass = 0; pass < passes; ++pass) {
      const int i0 = pass * 64 * CW + lane * CW;
      double a0[CW], a1[CW];
      correlate<CW>(a, ks, zr0, zr1, i0, a0, a1);
#pragma unroll
      for (int m = 0; m < CW; ++m) {
        if (i0 + m < ns) {
          f0[i0 + m] = a0[m];
          f1[i0 + m] = a1[m];
        }
      }
    }
    __syncthreads();  // f complete; the z_ref area becomes the history staging
    chunk_scan_replay<CW>(a, lane, f0, f1, zr0, rows_pr, xs, ys, kk, kstep, t0, ns, hb);
  }
  if (a.status != nullptr) {
    const bool finite = isfinite(xs[0]) && isfinite(xs[1]) && isfinite(xs[2]) &&
                        isfinite(ys[0]) && isfinite(ys[1]) && isfinite(ys[2]);
    if (lane == 0) a.status[b] = finite ? 0 : ZMPC_ST_NONFINITE;
  }
}

// Chunk geometry: CW = 8, chunks of lc = 2·64·CW timesteps (two correlation passes), LDS =
// k + z_ref (2 axes, lc + kc + 1 padded rows) + f (2 axes × lc): ≈ 45 KB at N = 512.
struct ChunkGeom {
  int lc, kc, kcp, lz, lzp;
};

ChunkGeom chunk_geom(int N) {
  constexpr int CW = 8;
  ChunkGeom g;
  g.lc = 2 * 64 * CW;
  g.kc = (N + CW - 1) / CW * CW;
  g.kcp = (g.kc + CW + 1) & ~1;  // the correlation's sliding window reads one group past kc
  g.lz = g.lc + g.kc + 1;
  g.lzp = ((g.lz + g.lz / CW + 1) + 1) & ~1;
  return g;
}

size_t chunk_lds_bytes(const ChunkGeom& g) {
  return (size_t)(g.kcp + 2 * g.lzp + 2 * g.lc) * sizeof(double);
}

// Batched predict_wieber_axis (strict=False): one wave per instance.
__global__ void __launch_bounds__(256) zmpc_step_unc_kernel(
    int64_t B, int N, LipmConsts lc, const double* __restrict__ k, const double* __restrict__ kxp,
    const double* __restrict__ x, const double* __restrict__ zmax_win,
    const double* __restrict__ zmin_win, double* __restrict__ x_next,
    int32_t* __restrict__ status) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const double* zx = zmax_win + b * N;
  const double* zn = zmin_win + b * N;
  double acc = 0.0;
  for (int j = lane; j < N; j += 64) acc = fma(k[j], (zx[j] + zn[j]) / 2, acc);
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (lane == 0) {
    const double* xb = x + b * 3;
    const double xs[3] = {xb[0], xb[1], xb[2]};
    const double u = acc - (kxp[0] * xs[0] + kxp[1] * xs[1] + kxp[2] * xs[2]);
    double y[3];
    lipm_step(lc, xs, u, y);
    x_next[b * 3 + 0] = y[0];
    x_next[b * 3 + 1] = y[1];
    x_next[b * 3 + 2] = y[2];
    if (status != nullptr)
      status[b] = (isfinite(y[0]) && isfinite(y[1]) && isfinite(y[2])) ? 0 : ZMPC_ST_NONFINITE;
  }
}

// Any walk length: the chunked kernel (its own CW = 8 geometry).
void launch_chunk(hipStream_t s, const RolloutArgs& a0, int N) {
  const ChunkGeom g = chunk_geom(N);
  RolloutArgs a = a0;
  a.kc = g.kc;
  a.kcp = g.kcp;
  a.lz = g.lz;
  a.lzp = g.lzp;
  hipLaunchKernelGGL(zmpc_rollout_unc_chunk_kernel<8>, dim3((unsigned)a.B), dim3(64),
                     chunk_lds_bytes(g), s, a, g.lc);
}

// Resident workgroups per CU of a kernel at an LDS size (a small per-host-thread cache keyed by
// kernel, block size and LDS; every device of the pool is the same gfx950 part).
int occupancy(const void* kernel, int threads, size_t lds) {
  struct Entry {
    const void* k;
    size_t lds;
    int threads, occ;
  };
  static thread_local Entry cache[32];
  static thread_local int used = 0;
  const int n = used < 32 ? used : 32;
  for (int i = 0; i < n; ++i)
    if (cache[i].k == kernel && cache[i].lds == lds && cache[i].threads == threads)
      return cache[i].occ;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, threads, lds) != hipSuccess)
    occ = 0;
  cache[used++ % 32] = Entry{kernel, lds, threads, occ};
  return occ;
}

// The wide kernel, with the next-dispatch-round prefetch when the batch takes at most two
// rounds of resident workgroups (config 5 at ≈2.7 rounds: 64.4 vs 54.3 µs with it, so off there;
// profiles/r3pfw/).
template <int C, int W, int E>
void launch_wide(hipStream_t s, RolloutArgs q, size_t lds, int64_t B, int cus) {
  if (lds > 64 * 1024) {  // (W = 8 only, wide_lds_cap): raise the kernel's dynamic-LDS limit
    static size_t raised = 64 * 1024;
    if (lds > raised &&
        hipFuncSetAttribute(reinterpret_cast<const void*>(zmpc_rollout_unc_wide_kernel<C, W, E>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess)
      raised = lds;
  }
  const int occ = occupancy(reinterpret_cast<const void*>(zmpc_rollout_unc_wide_kernel<C, W, E>),
                            128 * W, lds);
  const int64_t R = (int64_t)std::max(cus, 1) * occ;
  q.pf_ahead = (R > 0 && q.n <= 512 * W && B <= 2 * R) ? R : 0;
  hipLaunchKernelGGL((zmpc_rollout_unc_wide_kernel<C, W, E>), dim3((unsigned)B), dim3(128 * W),
                     lds, s, q);
}

// The wide kernel's instance for E points per thread.  E = 8 exists only where its transform
// (P = 8·128·W points of 16 B) fits the 64 KiB LDS ceiling the launcher enforces, i.e. W ≤ 4:
// an 8-wave E = 8 instance could never launch.
template <int C, int W>
void launch_wide_e(int E, hipStream_t s, const RolloutArgs& q, size_t lds, int64_t B, int cus) {
  if (E == 4) {
    launch_wide<C, W, 4>(s, q, lds, B, cus);
    return;
  }
  if constexpr (8 * 128 * W * 16 <= 64 * 1024) {
    if (E == 8) {
      launch_wide<C, W, 8>(s, q, lds, B, cus);
      return;
    }
  }
  launch_wide<C, W, 0>(s, q, lds, B, cus);
}

// Walks of at most 64·8+1 samples (one correlation pass).  The split kernels (a 128-thread
// workgroup per walk, one wave per axis) when their LDS fits the default 64 KiB ceiling:
//   shared CoP (f precomputed): zmpc_rollout_unc_splitd_kernel<CW, true>;
//   otherwise one walk per workgroup (odd CW: the fast-FIR dense form), with the next-round
//     prefetch when the batch takes at most two dispatch rounds (config 2: 29.6 → 26.9 µs,
//     profiles/r3pf/; with more rounds the touched lines are evicted before use, B = 16384:
//     92 → 117 µs).  Round 4: even CW no longer take the persistent kernel (it has no prefetch;
//     the horizon sweep's even-CW horizons were the slow ones, profiles/r4/); the diagnostics
//     build keeps it behind ZMPC_PERSISTENT for A/B.
// Otherwise (very long horizons) or with ZMPC_OPT_ROLLOUT_KERNEL = 1 (the cross-check):
// zmpc_rollout_unc_kernel, one wave per walk.
template <int CW>
void launch_unc(const RolloutGeom& g, size_t lds, hipStream_t s, RolloutArgs a, int cus,
                bool generic) {
  const size_t lds_axis = lds - (size_t)a.kcp * sizeof(double);  // no staged gain row
  size_t lds_split = std::max<size_t>(lds_axis, HistLayout<CW>::doubles(a.n) * sizeof(double));
  // the sparse-difference correlation stages the plan's suffix sums behind the z_ref areas
  const size_t lds_sparse = std::max(lds_axis + (size_t)ksum_rows(a.hN) * sizeof(double),
                                     lds_split);
  if (a.ksum != nullptr && lds_sparse <= 64 * 1024)
    lds_split = lds_sparse;
  else
    a.ksum = nullptr;
  if (a.fsh != nullptr) {
    // shared CoP, f precomputed: scan, replay and the history stores only
    hipLaunchKernelGGL((zmpc_rollout_unc_splitd_kernel<CW, true>), dim3((unsigned)a.B),
                       dim3(128), HistLayout<CW>::doubles(a.n) * sizeof(double), s, a);
    return;
  }
  if (generic || lds_split > 64 * 1024) {
    hipLaunchKernelGGL(zmpc_rollout_unc_kernel<CW>, dim3((unsigned)a.B), dim3(64), lds, s, a);
    return;
  }
#ifdef ZMPC_DIAG
  static const bool pers = getenv("ZMPC_PERSISTENT") != nullptr;  // A/B: round-3 even-CW rule
  if ((CW & 1) == 0 && pers) {
    const int per_cu = occupancy(
        reinterpret_cast<const void*>(zmpc_rollout_unc_persd_kernel<CW>), 128, lds_split);
    const int64_t grid = (int64_t)std::max(cus, 1) * per_cu;
    if (per_cu > 0 && grid < a.B && a.B <= 3 * grid) {
      hipLaunchKernelGGL(zmpc_rollout_unc_persd_kernel<CW>, dim3((unsigned)grid), dim3(128),
                         lds_split, s, a);
      return;
    }
  }
#endif
  const int occ = occupancy(
      reinterpret_cast<const void*>(zmpc_rollout_unc_splitd_kernel<CW, false>), 128, lds_split);
  const int64_t R = (int64_t)std::max(cus, 1) * occ;
  a.pf_ahead = (R > 0 && a.n <= 512 && a.B <= 2 * R) ? R : 0;
  hipLaunchKernelGGL((zmpc_rollout_unc_splitd_kernel<CW, false>), dim3((unsigned)a.B),
                     dim3(128), lds_split, s, a);
}

}  // namespace

size_t zmpc_rollout_unc_lds_bytes(int N, int64_t n) { return lds_bytes(rollout_geom(N, n)); }

#ifdef ZMPC_DIAG
// diagnostics: the phase stamps of the last launch to $ZMPC_ROLLOUT_TL ([B][5] u64)
static void tl_write(const unsigned long long* tl, int64_t B, hipStream_t s, hipError_t e) {
  const char* path = getenv("ZMPC_ROLLOUT_TL");
  if (tl == nullptr || path == nullptr || e != hipSuccess) return;
  std::vector<unsigned long long> h((size_t)B * 5);
  (void)hipStreamSynchronize(s);
  (void)hipMemcpy(h.data(), tl, h.size() * 8, hipMemcpyDeviceToHost);
  if (FILE* f = fopen(path, "wb")) {
    fwrite(h.data(), 8, h.size(), f);
    fclose(f);
  }
}
#endif

hipError_t zmpc_launch_rollout_unc(const zmpc_plan* p, int64_t B, int64_t n, const double* zmax,
                                   const double* zmin, int64_t bstride, const double* x0,
                                   const double* kick, int64_t kick_step,
                                   const int64_t* kick_steps, double* hist, int32_t* status,
                                   hipStream_t s, std::string* why) {
  if (n == 1) {
    // no QP solve: the history is the initial state only
    hipError_t e = hipMemcpyAsync(hist, x0, 6 * sizeof(double) * (size_t)B,
                                  hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
    if (status) return hipMemsetAsync(status, 0, sizeof(int32_t) * B, s);
    return hipSuccess;
  }
  const RolloutGeom g = rollout_geom(p->N, n);
  const size_t lds = lds_bytes(g);
#ifdef ZMPC_DIAG
  static const int dbg = [] {
    const char* e = getenv("ZMPC_DEBUG_ROLLOUT");  // diagnostics build: ablation bits
    return e ? atoi(e) : 0;
  }();
#else
  constexpr int dbg = 0;
#endif
  RolloutArgs a{};
  a.kc = g.kc;
  a.kcp = g.kcp;
  a.lz = g.lz;
  a.lzp = g.lzp;
  a.n = (int)n;
  a.B = B;
  a.lc = p->lc;
  a.k = p->k;
  a.kx = p->kx;
  a.zmax = zmax;
  a.zmin = zmin;
  a.bstride = bstride;
  a.x0 = x0;
  a.kick = kick;
  a.kick_step = kick_step;
  a.hist = hist;
  a.status = status;
  a.scanP = p->scanP;
  a.dbg = dbg;
  a.kick_steps = kick_steps;
  a.kffa = p->kffa;
  a.kfm = g.kfm;
  // ZMPC_OPT_CORRELATION = 1: the dense correlation forms only (cross-checks, and bench.py's
  // dense-form timing beside the default)
  a.ksum = p->opt[ZMPC_OPT_CORRELATION] == 1 ? nullptr : p->ksum;
  a.hN = p->N;
#ifdef ZMPC_DIAG
  // diagnostics: per-walk phase stamps of the split and wide kernels, written to $ZMPC_ROLLOUT_TL after
  // every launch ([B][5] u64, wall_clock64 ticks)
  static unsigned long long* tl_buf = nullptr;
  static int64_t tl_cap = 0;
  if (getenv("ZMPC_ROLLOUT_TL") && B > tl_cap) {
    if (tl_buf) (void)hipFree(tl_buf);
    tl_buf = nullptr;
    tl_cap = hipMalloc((void**)&tl_buf, (size_t)B * 5 * 8) == hipSuccess ? B : 0;
  }
  if (tl_buf) {
    (void)hipMemsetAsync(tl_buf, 0, (size_t)B * 5 * 8, s);
    a.tl = tl_buf;
  }
#endif
  const int long_form = p->opt[ZMPC_OPT_LONG_WALK];  // 0 auto, 1 direct, 2 FFT, 3 chunk kernel
  WideGeom wg;
  if (g.passes > 1 && (long_form == 3 || !wide_geom(p->N, n, &wg))) {
    launch_chunk(s, a, p->N);  // any length (the whole walk does not fit one pass)
    return hipGetLastError();
  }
  if (lds > 160 * 1024) {  // single-pass geometry beyond LDS (very long horizon N)
    launch_chunk(s, a, p->N);
    return hipGetLastError();
  }
  const bool generic = p->opt[ZMPC_OPT_ROLLOUT_KERNEL] == 1;
  // per-walk bounds whose single pass would run at CW = 8 take the wide kernel (wide_geom)
  const bool wide8 = kWide8 && g.passes == 1 && g.cw == 8 && bstride != 0 && !generic &&
                     wide_geom(p->N, n, &wg);
  if (g.passes > 1 || wide8) {
    RolloutArgs q = a;
    q.kc = wg.kc;
    q.lz = wg.lz;
    q.lzp = wg.lzp;
    size_t lds_w = 2 * (size_t)wg.lzp * sizeof(double);
    // FFT correlation when the transform maps onto the workgroup (E = P/NT points per thread,
    // 4 or 8), fits the default LDS ceiling and costs less than the direct form: measured
    // crossover (n − 1)·N ≥ 9·P·log2 P — N = 150 walks of 1000/2000 samples
    // are faster direct, N ≥ 200 faster by FFT.  ZMPC_OPT_LONG_WALK 1 / 2 forces the direct
    // form / the FFT wherever it fits.
    int P = kFftPmin;
    while (P < n - 1 + p->N) P *= 2;
    const int NT = 128 * wg.w;
    int E = (P % NT == 0) ? P / NT : 0;
    if (long_form == 1 || (E != 4 && E != 8) || P > kFftPT || (size_t)P * 16 > 64 * 1024) E = 0;
    if (long_form == 0 && (double)(n - 1) * p->N < 9.0 * P * __builtin_ctz((unsigned)P)) E = 0;
    if (E) {
      q.fft_tw = reinterpret_cast<const double2*>(p->fft_tw);
      q.fft_g = reinterpret_cast<const double2*>(p->fft_g) + (P - kFftPmin);
      lds_w = std::max(lds_w, (size_t)P * 16);
    }
    // the sparse attempt's table and change lists behind the z_ref areas (within the default
    // 64 KiB dynamic-LDS ceiling, else dense only)
    const size_t lds_sp = (2 * (size_t)wg.lzp + wide_sparse_doubles(p->N)) * sizeof(double);
    if (q.ksum != nullptr && lds_sp <= wide_lds_cap(wg.w))
      lds_w = std::max(lds_w, lds_sp);
    else
      q.ksum = nullptr;
    switch (wg.w * 16 + wg.cw) {
#define ZMPC_WCASE(W, C)                                \
  case W * 16 + C:                                      \
    launch_wide_e<C, W>(E, s, q, lds_w, B, p->cus);     \
    break;
      ZMPC_WCASE(2, 4) ZMPC_WCASE(2, 5) ZMPC_WCASE(2, 6) ZMPC_WCASE(2, 7) ZMPC_WCASE(2, 8)
      ZMPC_WCASE(4, 5) ZMPC_WCASE(4, 6) ZMPC_WCASE(4, 7) ZMPC_WCASE(4, 8)
      ZMPC_WCASE(8, 5) ZMPC_WCASE(8, 6) ZMPC_WCASE(8, 7) ZMPC_WCASE(8, 8)
#undef ZMPC_WCASE
      default:
        return hipErrorInvalidValue;
    }
    const hipError_t ew = hipGetLastError();
#ifdef ZMPC_DIAG
    tl_write(a.tl, B, s, ew);
#endif
    return ew;
  }
  // shared CoP (bounds stride 0) with a single-pass geometry: f once per launch
  double* fsh = nullptr;
  if (bstride == 0 && !generic && (6 * (size_t)n + 2 * (size_t)n) * sizeof(double) <= 64 * 1024) {
    a.fstride = ((64 * g.cw) + 63) & ~63;  // every lane's CW values, padded
    hipError_t e = hipMallocAsync((void**)&fsh, 2 * (size_t)a.fstride * sizeof(double), s);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return hipErrorOutOfMemory;
    }
    hipLaunchKernelGGL(zmpc_shared_f_kernel, dim3((unsigned)((a.fstride + 255) / 256), 2),
                       dim3(256), 0, s, zmax, zmin, (int)n, p->k, g.kc, fsh, a.fstride);
    a.fsh = fsh;
  }
  switch (g.cw) {
#define ZMPC_CW(C)                                   \
  case C:                                            \
    launch_unc<C>(g, lds, s, a, p->cus, generic);    \
    break;
    ZMPC_CW(1) ZMPC_CW(2) ZMPC_CW(3) ZMPC_CW(4) ZMPC_CW(5) ZMPC_CW(6) ZMPC_CW(7) ZMPC_CW(8)
#undef ZMPC_CW
    default:
      if (fsh) (void)hipFreeAsync(fsh, s);
      return hipErrorInvalidValue;
  }
  hipError_t e = hipGetLastError();
#ifdef ZMPC_DIAG
  tl_write(a.tl, B, s, e);
#endif
  if (fsh) {
    const hipError_t ef = hipFreeAsync(fsh, s);
    if (e == hipSuccess) e = ef;
  }
  return e;
}

hipError_t zmpc_launch_step_unc(const zmpc_plan* p, int64_t B, const double* x,
                                const double* zmax_win, const double* zmin_win, double* x_next,
                                int32_t* status, hipStream_t s) {
  hipLaunchKernelGGL(zmpc_step_unc_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, B,
                     p->N, p->lc, p->k, p->kx, x, zmax_win, zmin_win, x_next, status);
  return hipGetLastError();
}

// The dynamic-LDS ceiling must be raised once per device for > 64 KiB requests (the split
// kernels stay within the default 64 KiB).
hipError_t zmpc_rollout_unc_set_attrs() {
  hipError_t e = hipSuccess;
#define ZMPC_ATTR(C)                                                                        \
  if (e == hipSuccess)                                                                      \
    e = hipFuncSetAttribute((const void*)zmpc_rollout_unc_kernel<C>,                       \
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  ZMPC_ATTR(1) ZMPC_ATTR(2) ZMPC_ATTR(3) ZMPC_ATTR(4) ZMPC_ATTR(5) ZMPC_ATTR(6) ZMPC_ATTR(7)
  ZMPC_ATTR(8)
#undef ZMPC_ATTR
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)zmpc_rollout_unc_chunk_kernel<8>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  return e;
}
