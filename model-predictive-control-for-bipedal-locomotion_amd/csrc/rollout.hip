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
#include <cstdlib>

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

struct RolloutGeom {
  int cw, passes, kc, lz, lzp, nf;
  int kcp;  // doubles of LDS for the staged gain row (kc rounded up to even)
};

RolloutGeom rollout_geom(int N, int64_t n) {
  RolloutGeom g;
  const int64_t nsteps = n - 1;
  g.cw = pick_cw(nsteps);
  g.passes = (int)((nsteps + 64 * g.cw - 1) / (64 * g.cw));
  g.kc = (N + g.cw - 1) / g.cw * g.cw;           // k loop bound (k zero-padded)
  g.lz = g.passes * 64 * g.cw + g.kc + 1;         // z_ref samples staged (padded with last)
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
  const double* scanP;  // [8][6][9]: (Ā^C)^(2^r) for C = 1..8 (plan), or null
  int dbg;
};

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
  const int64_t kick_step = a.kick_step;

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
    for (int q = 0; q < 9; ++q) P.m[q] = a.scanP[(C - 1) * 54 + q];
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
  for (int d = 1; d < ((a.dbg & 2) ? 1 : 64); d <<= 1, ++r2) {
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
      for (int q = 0; q < 9; ++q) Pd.m[q] = a.scanP[(C - 1) * 54 + (r2 + 1) * 9 + q];
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
    if (!(a.dbg & 4)) {
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
  if (!(a.dbg & 8)) load_bounds<PF>(a, b, lane, r);
  // everything the tail needs is requested up front, behind the bound loads
  const double* xb = a.x0 + b * 6;
  const double xi0[3] = {xb[0], xb[1], xb[2]};
  const double xi1[3] = {xb[3], xb[4], xb[5]};
  const double kk = (a.kick != nullptr) ? a.kick[b] : 0.0;
  for (int j = lane; j < a.kcp; j += 64) ks[j] = a.k[j];
  store_zref<CW, PF>(a, r, zr0, zr1, lane);
  __syncthreads();
  double a0[CW], a1[CW];
  if (!(a.dbg & 1)) {
    correlate<CW>(a, ks, zr0, zr1, lane * CW, a0, a1);
  } else {
#pragma unroll
    for (int m = 0; m < CW; ++m) a0[m] = a1[m] = 0.0;
  }
  __syncthreads();
  scan_replay_store<CW, true>(a, b, lane, a0, a1, nullptr, nullptr, zr0, xi0, xi1, kk);
}

// Split-axis variant of the single-pass kernel: a 128-thread workgroup per walk, wave 0
// solves the x axis and wave 1 the y axis (half the registers and twice the waves of the
// one-wave kernel, for latency hiding); they share the staged z_ref, gain row and history
// staging buffer, so loads and stores stay whole-walk coalesced.
template <int CW>
__global__ void __launch_bounds__(128, 8) zmpc_rollout_unc_axis_kernel(RolloutArgs a) {
  using ZL = ZrLayout<CW>;
  constexpr int PF2 = (CW + 2) / 2;  // 128·PF2 >= 64·(CW+1) >= n
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ int flag[2];
  const int tid = threadIdx.x, axis = tid >> 6, lane = tid & 63;
  const int64_t b = blockIdx.x;
  const int n = a.n, nsteps = n - 1;
  // k stays in global memory (wave-uniform scalar loads): at 8 waves per SIMD the scalar
  // waits hide, and the LDS it would take keeps 16 walks per CU resident
  const double* __restrict__ ks = a.k;
  double* zr0 = smem;
  double* zr1 = zr0 + a.lzp;
  // ---- 1. bounds → z_ref (both waves, 128 samples per round) ---------------------------
  {
    const double2* zmx = reinterpret_cast<const double2*>(a.zmax + b * a.bstride);
    const double2* zmn = reinterpret_cast<const double2*>(a.zmin + b * a.bstride);
    double2 hi[PF2], lo[PF2];
#pragma unroll
    for (int u = 0; u < PF2; ++u) {
      const int t = u * 128 + tid;
      if (t < n && !(a.dbg & 8)) {
        hi[u] = zmx[t];
        lo[u] = zmn[t];
      } else {
        hi[u] = lo[u] = make_double2(0.0, 0.0);
      }
    }
#pragma unroll
    for (int u = 0; u < PF2; ++u) {
      const int t = u * 128 + tid;
      if (t < n) {
        zr0[ZL::idx(t)] = (hi[u].x + lo[u].x) / 2;
        zr1[ZL::idx(t)] = (hi[u].y + lo[u].y) / 2;
      }
    }
    const double2 h = zmx[n - 1], l = zmn[n - 1];
    const double last0 = (h.x + l.x) / 2, last1 = (h.y + l.y) / 2;
    for (int t = n + tid; t < a.lz; t += 128) {
      zr0[ZL::idx(t)] = last0;
      zr1[ZL::idx(t)] = last1;
    }
  }
  __syncthreads();

  // ---- 2. correlation for this wave's axis --------------------------------------------
  double f[CW];
  {
    const double* z = (axis ? zr1 : zr0) + ZL::idx(lane * CW);
    double w[CW];
#pragma unroll
    for (int m = 0; m < CW; ++m) {
      f[m] = 0.0;
      w[m] = z[ZL::idx(1 + m)];
    }
    for (int j = 0; j < ((a.dbg & 1) ? 0 : a.kc); j += CW) {
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
  __syncthreads();  // z_ref is dead from here on: the area becomes the history staging
  const double* xb = a.x0 + b * 6 + 3 * axis;
  const double xi[3] = {xb[0], xb[1], xb[2]};
  const double kk = (axis == 1 && a.kick != nullptr) ? a.kick[b] : 0.0;
  const int64_t kick_step = (axis == 1) ? a.kick_step : -1;

  // ---- 3. lane-chunk affine scan (this axis) -----------------------------------------
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
  const int mbeg = lane * CW;
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
  const double* Pp = a.scanP + (CW - 1) * 54;  // (Ā^CW)^(2^r), r = 0..5, from the plan
  if (lane == 0) {
    double t[3];
    Mat3 P;
#pragma unroll
    for (int q = 0; q < 9; ++q) P.m[q] = Pp[q];
    matvec3(P, xi, t);
    for (int i = 0; i < 3; ++i) sv[i] += t[i];
  }
#pragma unroll
  for (int r2 = 0; r2 < 6; ++r2) {
    const int d = 1 << r2;
    if (a.dbg & 2) break;
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
  double xs0[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double p = __shfl_up(sv[i], 1, 64);
    xs0[i] = (lane == 0) ? xi[i] : p;
  }

  // ---- 4. replay (reference form) into the shared staging rows, coalesced copy-out ----
  double* stage = zr0;
  const int rows_per_round = (2 * a.lzp) / 6;
  double* hb = a.hist + b * (int64_t)n * 6;
  double x[3];
  for (int r0 = 0; r0 < n; r0 += rows_per_round) {
    const int r1 = min(r0 + rows_per_round, n);
    if (lane == 0 && r0 == 0) {
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
          double* o = stage + (row - r0) * 6 + 3 * axis;
          o[0] = xn[0];
          o[1] = xn[1];
          o[2] = xn[2];
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) x[i] = xn[i];
      }
    }
    __syncthreads();
    if (!(a.dbg & 4)) {
      const int nd2 = (r1 - r0) * 3;
      const double2* src = reinterpret_cast<const double2*>(stage);
      double2* dst = reinterpret_cast<double2*>(hb + (int64_t)r0 * 6);
      for (int e = tid; e < nd2; e += 128) dst[e] = src[e];
    }
    __syncthreads();
  }
  if (a.status != nullptr) {
    const bool finite = isfinite(x[0]) && isfinite(x[1]) && isfinite(x[2]);
    const unsigned long long bad = __ballot(!finite);
    if (lane == 0) flag[axis] = bad ? ZMPC_ST_NONFINITE : 0;
    __syncthreads();
    if (tid == 0) a.status[b] = flag[0] | flag[1];
  }
}

// Longer walks (several correlation passes): one walk per wave, f through LDS.
template <int CW>
__global__ void __launch_bounds__(64) zmpc_rollout_unc_long_kernel(RolloutArgs a) {
  using ZL = ZrLayout<CW>;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = a.n, nsteps = n - 1;
  const int passes = (nsteps + 64 * CW - 1) / (64 * CW);
  double* ks = smem;
  double* zr0 = smem + a.kcp;
  double* zr1 = zr0 + a.lzp;
  double* f0 = zr1 + a.lzp;
  double* f1 = f0 + ((nsteps + 2) & ~1);
  for (int j = lane; j < a.kcp; j += 64) ks[j] = a.k[j];
  {
    const double2* zmx = reinterpret_cast<const double2*>(a.zmax + b * a.bstride);
    const double2* zmn = reinterpret_cast<const double2*>(a.zmin + b * a.bstride);
    constexpr int kU = 8;
    for (int t0 = 0; t0 < n; t0 += 64 * kU) {
      double2 hi[kU], lo[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int t = t0 + u * 64 + lane;
        if (t < n) {
          hi[u] = zmx[t];
          lo[u] = zmn[t];
        }
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int t = t0 + u * 64 + lane;
        if (t < n) {
          zr0[ZL::idx(t)] = (hi[u].x + lo[u].x) / 2;
          zr1[ZL::idx(t)] = (hi[u].y + lo[u].y) / 2;
        }
      }
    }
    const double2 hi = zmx[n - 1], lo = zmn[n - 1];
    const double last0 = (hi.x + lo.x) / 2, last1 = (hi.y + lo.y) / 2;
    for (int t = n + lane; t < a.lz; t += 64) {
      zr0[ZL::idx(t)] = last0;
      zr1[ZL::idx(t)] = last1;
    }
  }
  __syncthreads();
  for (int pass = 0; pass < passes; ++pass) {
    const int i0 = pass * 64 * CW + lane * CW;
    double a0[CW], a1[CW];
    correlate<CW>(a, ks, zr0, zr1, i0, a0, a1);
#pragma unroll
    for (int m = 0; m < CW; ++m) {
      if (i0 + m < nsteps) {
        f0[i0 + m] = a0[m];
        f1[i0 + m] = a1[m];
      }
    }
  }
  __syncthreads();
  const double* xb = a.x0 + b * 6;
  const double xi0[3] = {xb[0], xb[1], xb[2]};
  const double xi1[3] = {xb[3], xb[4], xb[5]};
  const double kk = (a.kick != nullptr) ? a.kick[b] : 0.0;
  scan_replay_store<CW, false>(a, b, lane, nullptr, nullptr, f0, f1, zr0, xi0, xi1, kk);
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

int g_cus = 0;  // CUs of the device the attributes were set on (grid sizing)

template <int CW>
void launch_unc(const RolloutGeom& g, size_t lds, hipStream_t s, const RolloutArgs& a) {
  static const bool one_wave = [] {
    const char* e = getenv("ZMPC_ROLLOUT_ONEWAVE");  // diagnostic A/B: one wave per walk
    return e != nullptr && atoi(e) != 0;
  }();
  // the split-axis kernel is built for 8 waves/SIMD: it keeps the default 64 KiB LDS cap
  const size_t lds_axis = lds - (size_t)a.kcp * sizeof(double);  // no staged gain row
  if (g.passes == 1 && !one_wave && lds_axis <= 64 * 1024) {
    hipLaunchKernelGGL(zmpc_rollout_unc_axis_kernel<CW>, dim3((unsigned)a.B), dim3(128), lds_axis,
                       s, a);
  } else if (g.passes == 1) {
    hipLaunchKernelGGL(zmpc_rollout_unc_kernel<CW>, dim3((unsigned)a.B), dim3(64), lds, s, a);
  } else {
    hipLaunchKernelGGL(zmpc_rollout_unc_long_kernel<CW>, dim3((unsigned)a.B), dim3(64), lds, s,
                       a);
  }
}

}  // namespace

size_t zmpc_rollout_unc_lds_bytes(int N, int64_t n) { return lds_bytes(rollout_geom(N, n)); }

hipError_t zmpc_launch_rollout_unc(const zmpc_plan* p, int64_t B, int64_t n, const double* zmax,
                                   const double* zmin, int64_t bstride, const double* x0,
                                   const double* kick, int64_t kick_step, double* hist,
                                   int32_t* status, hipStream_t s, std::string* why) {
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
  if (lds > 160 * 1024) {
    *why = "walk too long for the LDS-resident rollout (n=" + std::to_string(n) + ")";
    return hipErrorInvalidValue;
  }
  static const int dbg = [] {
    const char* e = getenv("ZMPC_DEBUG_ROLLOUT");  // diagnostic ablation bits (0 in production)
    return e ? atoi(e) : 0;
  }();
  RolloutArgs a{g.kc, g.kcp, g.lz,      g.lzp, (int)n,     B,   p->lc,
                p->k, p->kx,  zmax,      zmin,  bstride,    x0,  kick,
                kick_step,    hist, status, p->scanP, dbg};
  switch (g.cw) {
#define ZMPC_CW(C)               \
  case C:                        \
    launch_unc<C>(g, lds, s, a); \
    break;
    ZMPC_CW(1) ZMPC_CW(2) ZMPC_CW(3) ZMPC_CW(4) ZMPC_CW(5) ZMPC_CW(6) ZMPC_CW(7) ZMPC_CW(8)
#undef ZMPC_CW
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t zmpc_launch_step_unc(const zmpc_plan* p, int64_t B, const double* x,
                                const double* zmax_win, const double* zmin_win, double* x_next,
                                int32_t* status, hipStream_t s) {
  hipLaunchKernelGGL(zmpc_step_unc_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, B,
                     p->N, p->lc, p->k, p->kx, x, zmax_win, zmin_win, x_next, status);
  return hipGetLastError();
}

// The dynamic-LDS ceiling must be raised once per device for > 64 KiB requests (not for the
// split-axis kernel, whose 8-waves-per-SIMD bound caps its LDS below that).
hipError_t zmpc_rollout_unc_set_attrs() {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess)
    e = hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
#define ZMPC_ATTR(C)                                                                        \
  if (e == hipSuccess)                                                                      \
    e = hipFuncSetAttribute((const void*)zmpc_rollout_unc_kernel<C>,                       \
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);       \
  if (e == hipSuccess)                                                                      \
    e = hipFuncSetAttribute((const void*)zmpc_rollout_unc_long_kernel<C>,                  \
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  ZMPC_ATTR(1) ZMPC_ATTR(2) ZMPC_ATTR(3) ZMPC_ATTR(4) ZMPC_ATTR(5) ZMPC_ATTR(6) ZMPC_ATTR(7)
  ZMPC_ATTR(8)
#undef ZMPC_ATTR
  return e;
}
