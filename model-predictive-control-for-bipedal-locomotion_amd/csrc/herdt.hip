// Herdt joint footstep QP on the device (config.method == "herdt").
//
// Reference (per walk, sequential; cvxpy → OSQP per timestep, polish=False):
//   generate_com_trajectory_herdt  zmp_controller.py:435-531   rollout + foot bookkeeping
//   predict_herdt_joint            zmp_controller.py:533-826   the joint x/y QP
// Per axis the reference QP in u = [J (N), f (m)] is
//   ½α‖J‖² + ½β‖Pvs x + Pvu J − v_ref‖² + ½γ‖Pzx x + Pzu J − U_c fc − U f‖²          (:599-642)
// s.t. |Pzx x + Pzu J − U_c fc − U f|_k ≤ ½·foot_dim on the non-STANDING rows         (:661-707)
//      zmin_st ≤ (Pzx x + Pzu J)_k ≤ zmax_st on the STANDING rows when the robot stands   (:719-769)
// plus, coupling the axes, the first footstep's offset in the swing foot's polytope   (:771-783).
// With Pzu[k,j] = C A^(k−j) B, Pzx[k] = C A^(k+1), Pvs/Pvu likewise the velocity row of the
// LIPM, every term is a stage cost of the 3-state LIPM x_{k+1} = A x_k + B u_k:
//   ½α u_k² + ½β (e_vᵀx_k + b_v u_k − vr_k)² + ½γ (c1ᵀx_k + p0 u_k − c_k)²,
//   e_v = [0, 1, T], b_v = T²/2 (velocity at k+1), c1 = (CA)ᵀ, p0 = CB (ZMP at k+1),
// where the ZMP centre c_k is the current foot (rows of U_c) or a footstep variable f_j (rows of
// U, one column per support segment).  The footsteps are constant over the horizon, so they
// enter the Riccati recursion as augmented states ξ = [x; f] with identity dynamics; an active
// ZMP row pins u_k = (t_k + c_k − c1ᵀx_k)/p0 (affine in ξ), exactly as in strict_lq.hip.  At
// k = 0 the value function V_0(x_0, f) is minimised over f: the first footstep of the two
// axes (adjacent lanes) meets the polytope in a 2-D QP solved exactly in both lanes; the later
// footsteps follow from the conditional minimiser.  The working set of ZMP rows comes from the
// same primal-dual active-set iteration as the strict solver (release wrong-signed
// multipliers from a costate sweep, add violated rows, stop when the set repeats), warm-started
// with the previous timestep's set shifted one row.
//
// A pass: sweep 1 runs the augmented Riccati (3 + the wave's footstep count) backward for V_0(x, f);
// the footsteps follow; sweep 2 runs the 3-state Riccati with every ZMP centre now known (the
// augmented control law at f = fsol) and keeps 4 doubles per row; the forward sweep rolls out,
// checks the free rows' bounds and the pinned rows' multipliers (from sweep 2's value function,
// no costate sweep).  Only sweep 2 writes and only the forward sweep reads per-row data.
//
// Mapping: one lane per (walk, axis), lanes 2w and 2w+1 = axes x, y of walk w; a one-wave
// workgroup holds 32 walks.  Sweep 2's rows go through a per-wave global slab ([row][4][64]);
// per-row segment index, constraint kind and working-set flag are LDS bytes, the swing
// polygons (half-spaces and facet segments) LDS doubles.
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "zmpc_internal.h"

namespace {

constexpr int HMAXIT = 64;  // default active-set pass cap (zmpc_herdt_params.max_passes)
#ifdef ZMPC_DIAG
constexpr bool kProf = true;  // per-phase clocks (ZMPC_HERDT_PROF), diagnostics build only
#else
constexpr bool kProf = false;
#endif

struct HerdtArgs {
  int N;
  int window_mode;       // 0: rollout over [B, n] inputs; 1: one step on [B, N] windows
  int64_t n;             // samples per walk (rollout)
  int64_t B;             // walks
  // LIPM (zmp_controller.py:18-20) and derived rows
  double T, T2, T3;      // A/B entries as the reference evaluates them
  double c1_2, p0;       // c1 = [1, T, T²/2 − h/g], p0 = T³/6 − T h/g
  double alpha, beta, gamma;
  double bx, by;         // ½ foot_length, ½ foot_width (:666, :680)
  double flen, fwid, fspread;
  int nfl, nfr;          // polytope facets (left, right swing polygon)
  double poly[2][ZMPC_HERDT_MAX_FACETS][3];  // [side][facet] = (a_x, a_y, b): a·d <= b
  // inputs (rollout): v_ref [B,n,2] (stride vs doubles per walk, 0 = shared), states [B,n]
  // int8 (stride ss), nb [B,n] int32 steps to the next footstep change (stride ns)
  const double* vref;
  int64_t vs;
  const int8_t* st;
  int64_t ss;
  const int32_t* nb;
  int64_t ns;
  const double* x0;      // [B,2,3]
  const double* kick;    // [B] or null (y-velocity impulse at kick_step, :525-526)
  int64_t kick_step;
  // step-mode inputs: current state [B] int8, foot position [B,2], foot side [B] int8 (0 left)
  const int8_t* cur0;
  const double* fc0;
  const int8_t* side0;
  // outputs
  double* hist;          // rollout [B,n,2,3]; step: x_next [B,2,3]
  double* foot;          // rollout [B,n,2]; step: first footstep [B,2] (NaN when m = 0)
  int32_t* status;
  double* ws;            // per-wave slab [waves][N][NF][64]
  int nf;                // doubles per row in the slab
  unsigned long long* cnt;  // plan work counters [4..7] (zmpc_plan_counters), may be null
  int maxit;                // active-set pass cap per solve (ZMPC_ST_MAXITER beyond)
  unsigned long long* prof; // diagnostics build only (ZMPC_DIAG, ZMPC_HERDT_PROF): clock per
                            // phase, summed; null in the product library
};

// Slab row k (4 doubles, written by sweep 2, read by the forward sweep):
//   free row:   K (3), kff        — the control law u = −K x − kff at the solved footsteps
//   pinned row: PB̂ (3), B̂ᵀs of V_{k+1} — the costate B̂ᵀλ_{k+1} = B̂ᵀ∇V_{k+1}(x_{k+1}) for the
//               row's multiplier (its u is fixed by the row)
constexpr int SLAB = 4;
constexpr int RB = 8;  // forward sweep: rows whose slab loads are in flight together

// packed symmetric index (a <= b)
template <int NA>
__device__ __forceinline__ constexpr int sidx(int a, int b) {
  return a <= b ? a * NA - a * (a - 1) / 2 + (b - a) : b * NA - b * (b - 1) / 2 + (a - b);
}

// Swing-foot polygons in LDS (per workgroup, both sides): the half-spaces a·d <= b and, per
// facet, the feasible segment of its boundary line [e0, e1] (x0 = NaN: empty).
struct PolyLds {
  double h[2][ZMPC_HERDT_MAX_FACETS][3];
  double seg[2][ZMPC_HERDT_MAX_FACETS][4];
};

// Facet i of side sd: clip its line {a·d = b} by the other half-spaces (one lane per facet).
__device__ void polytope_segment(const double (*P)[3], int nfac, int i, double& o0, double& o1,
                                 double& o2, double& o3) {
  const double ax = P[i][0], ay = P[i][1], b = P[i][2];
  const double n2 = ax * ax + ay * ay;
  const double px = ax * b / n2, py = ay * b / n2;  // foot of the line
  const double dx = -ay, dy = ax;                   // along the line
  double lo = -1e300, hi = 1e300;
  bool ok = true;
  for (int j = 0; j < nfac; ++j) {
    if (j == i) continue;
    const double ad = P[j][0] * dx + P[j][1] * dy;
    const double rr = P[j][2] - (P[j][0] * px + P[j][1] * py);
    if (fabs(ad) < 1e-14) {
      ok = ok && rr >= -1e-12;
    } else if (ad > 0) {
      hi = fmin(hi, rr / ad);
    } else {
      lo = fmax(lo, rr / ad);
    }
  }
  if (!ok || lo > hi || lo < -1e299 || hi > 1e299) {
    o0 = __builtin_nan("");
    o1 = o2 = o3 = 0.0;
    return;
  }
  o0 = px + lo * dx;
  o1 = py + lo * dy;
  o2 = px + hi * dx;
  o3 = py + hi * dy;
}

// Exact minimiser of ½σx(dx − ux)² + ½σy(dy − uy)² over the polygon {d : a_i·d <= b_i}: the
// unconstrained point when feasible, else the best clamped projection onto a facet segment
// (the optimum of a convex QP outside its minimiser lies on the boundary: inside a facet, or
// at a vertex = a segment end).
// Returns false when the point is outside and no facet segment is usable (a degenerate or
// unbounded polygon through the C-ABI): the caller flags the walk (ZMPC_ST_INFEASIBLE).
__device__ bool polytope_qp(const PolyLds& L, int sd, int nfac, double sx, double sy, double ux,
                            double uy, double* dx, double* dy) {
  const double tol = 1e-12;
  bool inside = true;
  for (int i = 0; i < nfac; ++i)
    inside = inside && (L.h[sd][i][0] * ux + L.h[sd][i][1] * uy <= L.h[sd][i][2] + tol);
  if (inside) {
    *dx = ux;
    *dy = uy;
    return true;
  }
  double best = 1e300, bx = ux, by = uy;
  bool any = false;
  for (int i = 0; i < nfac; ++i) {
    const double* e = L.seg[sd][i];
    if (isnan(e[0])) continue;
    any = true;
    const double wx = e[2] - e[0], wy = e[3] - e[1];
    const double rx = e[0] - ux, ry = e[1] - uy;
    const double den = sx * wx * wx + sy * wy * wy;
    double t = den > 0.0 ? -(sx * rx * wx + sy * ry * wy) / den : 0.0;
    t = fmin(fmax(t, 0.0), 1.0);
    const double px = e[0] + t * wx, py = e[1] + t * wy;
    const double v = 0.5 * sx * (px - ux) * (px - ux) + 0.5 * sy * (py - uy) * (py - uy);
    if (v < best) {
      best = v;
      bx = px;
      by = py;
    }
  }
  *dx = bx;
  *dy = by;
  return any;
}

// Cholesky factor of the M×M footstep block F of P (packed, NA-indexed at offset 3): L lower,
// the reciprocal pivots in id.  False when F is not positive definite.
template <int NA, int MM>
__device__ __forceinline__ bool small_chol(const double* P, int M, double (&L)[MM][MM],
                                           double (&id)[MM]) {
#pragma unroll
  for (int i = 0; i < MM; ++i)
#pragma unroll
    for (int j = 0; j < MM; ++j) L[i][j] = (i < M && j <= i) ? P[sidx<NA>(3 + i, 3 + j)] : 0.0;
  bool ok = true;
#pragma unroll
  for (int k = 0; k < MM; ++k) {
    id[k] = 0.0;
    if (k < M) {
      double d = L[k][k];
#pragma unroll
      for (int q = 0; q < MM; ++q)
        if (q < k) d -= L[k][q] * L[k][q];
      ok = ok && d > 0.0;
      const double piv = sqrt(fmax(d, 1e-300));
      L[k][k] = piv;
      id[k] = 1.0 / piv;
#pragma unroll
      for (int i = 0; i < MM; ++i) {
        if (i > k && i < M) {
          double v = L[i][k];
#pragma unroll
          for (int q = 0; q < MM; ++q)
            if (q < k) v -= L[i][q] * L[k][q];
          L[i][k] = v * id[k];
        }
      }
    }
  }
  return ok;
}

// Solve F g' = g in place with the factor of small_chol.
template <int MM>
__device__ __forceinline__ void small_chol_solve(const double (&L)[MM][MM], const double (&id)[MM],
                                                 int M, double* g) {
#pragma unroll
  for (int i = 0; i < MM; ++i) {
    if (i < M) {
      double v = g[i];
#pragma unroll
      for (int q = 0; q < MM; ++q)
        if (q < i) v -= L[i][q] * g[q];
      g[i] = v * id[i];
    }
  }
#pragma unroll
  for (int i = MM - 1; i >= 0; --i) {
    if (i < M) {
      double v = g[i];
#pragma unroll
      for (int q = 0; q < MM; ++q)
        if (q > i && q < M) v -= L[q][i] * g[q];
      g[i] = v * id[i];
    }
  }
}

enum : unsigned char { CK_NONE = 0, CK_FOOT = 1, CK_STAND = 2 };

// Per-lane constants of a Riccati row (see the kernel).
struct RowC {
  double T, T2, T3, bv, p0, ip, al, be, ga, c12;  // ip = 1/p0
  double bnd, shi, slo;  // ZMP bounds: foot rows ±bnd around the centre, standing [slo, shi]
};

// One backward Riccati row on V_{k+1}(ξ) = ½ξᵀPξ − sᵀξ → V_k, in place, ξ = [x; f] (NA − 3
// footstep columns).  Row k's stage cost: ½α u² + ½β(e_vᵀx + b_v u − vr)² + ½γ(c1ᵀx + p0 u −
// c)² with the ZMP centre c = fc0 (jf < 0) or the footstep f_jf; wk ≠ 0 pins the row's ZMP to
// a bound (u = (t + ccon − c1ᵀx)/p0, ccon = the centre on a foot row).  Outputs the row's
// control law u = −K ξ − kff (x part K[0..2]) and V_{k+1}'s (PB̂)_x, B̂ᵀs (the pinned row's
// costate map, see the forward sweep).
template <int NA>
__device__ __forceinline__ void herdt_row(const RowC& c, double* P, double* s, double vr,
                                          double fc0, int jf, int kd, int wk, double* pbx,
                                          double& sbo, double* Kx, double& kffo) {
  const double T = c.T, T2 = c.T2, p0 = c.p0, bv = c.bv;
  const double al = c.al, be = c.be, ga = c.ga;
  const double c1[3] = {1.0, T, c.c12};
  const double ev[3] = {0.0, 1.0, T};
  const double Bv[3] = {c.T3, T2, T};
  // P B̂ (x part of B̂ only)
  double pb[NA];
#pragma unroll
  for (int q = 0; q < NA; ++q)
    pb[q] = P[sidx<NA>(q, 0)] * Bv[0] + P[sidx<NA>(q, 1)] * Bv[1] + P[sidx<NA>(q, 2)] * Bv[2];
  const double bpb = Bv[0] * pb[0] + Bv[1] * pb[1] + Bv[2] * pb[2];
  const double Huu = al + be * bv * bv + ga * p0 * p0 + bpb;
  // H_uξ
  double Hu[NA];
  Hu[0] = pb[0] + be * bv * ev[0] + ga * p0 * c1[0];
  Hu[1] = T * pb[0] + pb[1] + be * bv * ev[1] + ga * p0 * c1[1];
  Hu[2] = T2 * pb[0] + T * pb[1] + pb[2] + be * bv * ev[2] + ga * p0 * c1[2];
#pragma unroll
  for (int q = 3; q < NA; ++q) Hu[q] = pb[q] + ((q - 3 == jf) ? -ga * p0 : 0.0);
  // h_u, h_ξ
  const double sb = Bv[0] * s[0] + Bv[1] * s[1] + Bv[2] * s[2];
  const double hu = sb + be * bv * vr + ga * p0 * fc0;
  double hx[NA];
  hx[0] = s[0] + be * ev[0] * vr + ga * c1[0] * fc0;
  hx[1] = T * s[0] + s[1] + be * ev[1] * vr + ga * c1[1] * fc0;
  hx[2] = T2 * s[0] + T * s[1] + s[2] + be * ev[2] * vr + ga * c1[2] * fc0;
#pragma unroll
  for (int q = 3; q < NA; ++q) hx[q] = s[q];
  // control law u = −K̂ ξ − kff
  double Kh[NA], kff;
  {
    // both laws, merged by selects: a wave with free and pinned lanes would otherwise run both
    // sides of a branch with its exec-mask bookkeeping, at one wave per SIMD
    // free: 1/Huu by the hardware reciprocal + two Newton steps (Huu ≥ α + βb_v² + γp0² > 0)
    double iq = __builtin_amdgcn_rcp(Huu);
    iq = fma(iq, fma(-Huu, iq, 1.0), iq);
    iq = fma(iq, fma(-Huu, iq, 1.0), iq);
    // pinned: c1ᵀx + p0 u − ccon = t  (ccon: the foot centre on a foot row, 0 standing)
    const bool pin = wk != 0, foot = kd == CK_FOOT;
    const double t = (kd == CK_STAND) ? (wk == 1 ? c.shi : c.slo) : (wk == 1 ? c.bnd : -c.bnd);
    const double cc0 = foot ? fc0 : 0.0;
    const double ip = c.ip;
#pragma unroll
    for (int q = 0; q < 3; ++q) Kh[q] = pin ? c1[q] * ip : Hu[q] * iq;
#pragma unroll
    for (int q = 3; q < NA; ++q) Kh[q] = pin ? ((foot && q - 3 == jf) ? -ip : 0.0) : Hu[q] * iq;
    kff = pin ? -(t + cc0) * ip : -hu * iq;
  }
  // D = Huu·K̂ − Hu (the pinned rows' correction; a free row's rounding residue), formed where
  // it is used so that only Hu and K̂ stay live through the update
#define HD(q) fma(Huu, Kh[q], -Hu[q])
  // s first (hx dies before P's update)
#pragma unroll
  for (int q = 0; q < NA; ++q) s[q] = fma(-kff, HD(q), fma(-hu, Kh[q], hx[q]));
  // V_k: P = H − Hu K̂ᵀ + K̂ Dᵀ with H = ÂᵀPÂ + stage, updated in place block by block (each
  // block reads only its own old entries, so H is never held whole)
  {
    // x-x block: AᵀP_xxA + stage
    const double q00 = P[sidx<NA>(0, 0)], q01 = P[sidx<NA>(0, 1)], q02 = P[sidx<NA>(0, 2)];
    const double q11 = P[sidx<NA>(1, 1)], q12 = P[sidx<NA>(1, 2)], q22 = P[sidx<NA>(2, 2)];
    const double a01 = T * q00 + q01, a02 = T2 * q00 + T * q01 + q02;  // (P A) row 0, cols 1, 2
    const double a11 = T * q01 + q11, a12 = T2 * q01 + T * q11 + q12;  // row 1
    const double a22 = T2 * q02 + T * q12 + q22;                        // row 2
    double Hx[3][3];
    Hx[0][0] = q00;
    Hx[0][1] = a01;
    Hx[0][2] = a02;
    Hx[1][1] = T * a01 + a11;
    Hx[1][2] = T * a02 + a12;
    Hx[2][2] = T2 * a02 + T * a12 + a22;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int cc = r; cc < 3; ++cc) {
        const double v = Hx[r][cc] + be * ev[r] * ev[cc] + ga * c1[r] * c1[cc];
        P[sidx<NA>(r, cc)] = v - Hu[r] * Kh[cc] + Kh[r] * HD(cc);
      }
  }
#pragma unroll
  for (int cc = 3; cc < NA; ++cc) {
    // x-f column cc: (AᵀP)[r][cc] + stage
    const double q0 = P[sidx<NA>(0, cc)], q1 = P[sidx<NA>(1, cc)], q2 = P[sidx<NA>(2, cc)];
    const double cf = (cc - 3 == jf) ? -ga : 0.0;
    const double h0 = q0 + cf * c1[0];
    const double h1 = T * q0 + q1 + cf * c1[1];
    const double h2 = T2 * q0 + T * q1 + q2 + cf * c1[2];
    const double dc = HD(cc);
    P[sidx<NA>(0, cc)] = h0 - Hu[0] * Kh[cc] + Kh[0] * dc;
    P[sidx<NA>(1, cc)] = h1 - Hu[1] * Kh[cc] + Kh[1] * dc;
    P[sidx<NA>(2, cc)] = h2 - Hu[2] * Kh[cc] + Kh[2] * dc;
    // f-f column cc (rows 3..cc)
#pragma unroll
    for (int r = 3; r <= cc; ++r) {
      const double v = P[sidx<NA>(r, cc)] + ((r - 3 == jf && cc - 3 == jf) ? ga : 0.0);
      P[sidx<NA>(r, cc)] = v - Hu[r] * Kh[cc] + Kh[r] * dc;
    }
  }
#undef HD
  pbx[0] = pb[0];
  pbx[1] = pb[1];
  pbx[2] = pb[2];
  sbo = sb;
  Kx[0] = Kh[0];
  Kx[1] = Kh[1];
  Kx[2] = Kh[2];
  kffo = kff;
}

// A free-tail row of sweep 2 (rows past the wave's last pinned row): P, K and 1/Huu are the
// all-free recursion's (ktab: K0, K1, K2, 1/Huu), only s moves — herdt_row<3> of a free row
// without the rounding residue D = Huu·K − Hu.
__device__ __forceinline__ void herdt_tail_row(const RowC& c, double* s, double vr, double ck,
                                               const double* kt, double& kffo) {
  const double T = c.T, T2 = c.T2, p0 = c.p0, bv = c.bv, be = c.be, ga = c.ga;
  const double sb = c.T3 * s[0] + T2 * s[1] + T * s[2];
  const double hu = sb + be * bv * vr + ga * p0 * ck;
  const double hx0 = s[0] + ga * ck;
  const double hx1 = T * s[0] + s[1] + be * vr + ga * T * ck;
  const double hx2 = T2 * s[0] + T * s[1] + s[2] + be * T * vr + ga * c.c12 * ck;
  kffo = -hu * kt[3];
  s[0] = hx0 - hu * kt[0];
  s[1] = hx1 - hu * kt[1];
  s[2] = hx2 - hu * kt[2];
}

template <int MM>
__global__ void __launch_bounds__(64) zmpc_herdt_kernel(HerdtArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char hsm[];
  const int lane = threadIdx.x;
  const int N = a.N;
  unsigned char* segb = hsm;              // [N][64] support segment of row k (0 = current foot)
  unsigned char* kind = hsm + N * 64;     // [N][64] constraint kind
  unsigned char* wset = hsm + 2 * N * 64; // [N][64] working set: 0 free, 1 upper, 2 lower
  PolyLds& pl = *reinterpret_cast<PolyLds*>(hsm + ((3 * N * 64 + 15) & ~15));
  // free-tail feedback [N][3]: K of row k when rows k..N−1 are all free (it depends on the
  // working set only; the bounds, v_ref and the centres enter kff)
  double* ktab = reinterpret_cast<double*>(hsm + ((3 * N * 64 + 15) & ~15) + sizeof(PolyLds));
  // (ktab row k: K0, K1, K2, 1/Huu; the all-free P after row k is in ptab, global, per
  // workgroup: sweep 2 starts its full rows from it)
  // cen [MM+1][64]: the ZMP centre of each support segment after the footstep solve (0: the
  // current foot, j: footstep j) — one LDS read per row instead of a select over MM footsteps
  double* cen = ktab + N * 4;
  {
    // both sides' half-spaces and facet segments, once per workgroup
    const int sd = lane >> 5, i = lane & 31;
    const int nf = sd == 0 ? a.nfl : a.nfr;
    if (i < ZMPC_HERDT_MAX_FACETS) {
      for (int c = 0; c < 3; ++c) pl.h[sd][i][c] = a.poly[sd][i][c];
      // (four scalars, not an array: the array's two stores on the no-segment path made the
      // compiler keep it in scratch, 24 B per lane)
      double e0 = __builtin_nan(""), e1 = 0.0, e2 = 0.0, e3 = 0.0;
      if (i < nf) polytope_segment(a.poly[sd], nf, i, e0, e1, e2, e3);
      pl.seg[sd][i][0] = e0;
      pl.seg[sd][i][1] = e1;
      pl.seg[sd][i][2] = e2;
      pl.seg[sd][i][3] = e3;
    }
    __syncthreads();
  }
  const int64_t w = (int64_t)blockIdx.x * 32 + (lane >> 1);
  const int axis = lane & 1;
  const bool valid = w < a.B;
  const int64_t wc = valid ? w : 0;  // clamped walk for loads (invalid lanes compute garbage)
  double* slab = a.ws + (size_t)blockIdx.x * N * (a.nf * 64 + 6);
  double* ptab = slab + (size_t)N * a.nf * 64;  // [N][6] all-free P (V_k), this workgroup
  auto S = [&](int k, int f) -> double& { return slab[((size_t)k * a.nf + f) * 64 + lane]; };

  const double T = a.T, T2 = a.T2, T3 = a.T3;
  const double c1[3] = {1.0, T, a.c1_2};
  const double ev[3] = {0.0, 1.0, T};
  const double p0 = a.p0, bv = T2, ip0 = 1.0 / a.p0;
  const double al = a.alpha, be = a.beta, ga = a.gamma;
  const double bnd = axis ? a.by : a.bx;
  {
    // the free-tail table: sweep 2's recursion with every row free, from V_N = 0
    const RowC rt{T, T2, T3, bv, p0, ip0, al, be, ga, a.c1_2, 0.0, 0.0, 0.0};
    double Pt[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, st[3] = {0.0, 0.0, 0.0};
    for (int k = N - 1; k >= 0; --k) {
      double pbx[3], sb, Kx[3], kff;
      // 1/Huu of the row as herdt_row computes it: Huu = α + βb_v² + γp0² + B̂ᵀPB̂ (old P)
      const double pb0 = Pt[0] * T3 + Pt[1] * T2 + Pt[2] * T;
      const double pb1 = Pt[1] * T3 + Pt[3] * T2 + Pt[4] * T;
      const double pb2 = Pt[2] * T3 + Pt[4] * T2 + Pt[5] * T;
      const double Huu = al + be * bv * bv + ga * p0 * p0 + (T3 * pb0 + T2 * pb1 + T * pb2);
      double iq = __builtin_amdgcn_rcp(Huu);
      iq = fma(iq, fma(-Huu, iq, 1.0), iq);
      iq = fma(iq, fma(-Huu, iq, 1.0), iq);
      herdt_row<3>(rt, Pt, st, 0.0, 0.0, -1, CK_NONE, 0, pbx, sb, Kx, kff);
      if (lane == 0) {
        ktab[k * 4 + 0] = Kx[0];
        ktab[k * 4 + 1] = Kx[1];
        ktab[k * 4 + 2] = Kx[2];
        ktab[k * 4 + 3] = iq;
        for (int q = 0; q < 6; ++q) ptab[k * 6 + q] = Pt[q];
      }
    }
    __syncthreads();
  }

  double x[3];
  const double* xp = a.x0 + (wc * 2 + axis) * 3;
  x[0] = xp[0];
  x[1] = xp[1];
  x[2] = xp[2];
  int cur, side;
  double fc, air;
  if (a.window_mode) {
    cur = a.cur0[wc];
    side = a.side0[wc];
    fc = a.fc0[wc * 2 + axis];
  } else {
    cur = a.st[wc * a.ss];
    side = 0;  // "left" (:458)
    fc = axis ? a.fspread : 0.0;  // (:456-457)
    if (valid) {
      double* h = a.hist + ((wc * a.n) * 2 + axis) * 3;
      h[0] = x[0];
      h[1] = x[1];
      h[2] = x[2];
      a.foot[(wc * a.n) * 2 + axis] = fc;
    }
  }
  air = fc;
  for (int k = 0; k < N; ++k) wset[k * 64 + lane] = 0;
  int fq = 0;
  unsigned long long n_wave_pass = 0, n_pass = 0, n_m = 0, n_m2 = 0;
  unsigned itmax = 0;  // most passes of one solve (counter [9])
  unsigned long long pr_b = 0, pr_f = 0, pr_w = 0, pr_t0 = (kProf && a.prof) ? clock64() : 0;
  unsigned long long pr_kw = 0, pr_ns = 0, pr_own = 0, pr_fs = 0, pr_lw = 0;
  const int64_t nsteps = a.window_mode ? 1 : a.n - 1;
  const int64_t kstep = (!a.window_mode && axis == 1 && a.kick) ? a.kick_step : -1;
  const double kv = (kstep >= 0 && valid) ? a.kick[wc] : 0.0;

  for (int64_t i = 0; i < nsteps; ++i) {
    // ---- window of this timestep: states, segments, constraint kinds (:561-573, :687-712)
    auto wstate = [&](int k) -> int {
      if (a.window_mode) return a.st[wc * a.ss + k];
      int64_t t = i + 1 + k;
      if (t > a.n - 1) t = a.n - 1;  // padding with the last row (:466-469)
      return a.st[wc * a.ss + t];
    };
    int s_prev = cur, nbreak = 0, nstand = 0, lastbreak = -1;
    // the window's states are loaded WB rows at a time, all in flight together (one row per
    // round trip, at one wave per SIMD)
    constexpr int WB = 16;
    for (int k0 = 0; k0 < N; k0 += WB) {
      int sv[WB];
#pragma unroll
      for (int r = 0; r < WB; ++r) sv[r] = wstate(min(k0 + r, N - 1));
#pragma unroll
      for (int r = 0; r < WB; ++r) {
        const int k = k0 + r;
        if (k < N) {
          const int sk = sv[r];
          segb[k * 64 + lane] = (unsigned char)nbreak;
          const bool cont = (sk == s_prev) || (s_prev == ZMPC_DOUBLE_SUPPORT &&
                                                sk == ZMPC_SINGLE_SUPPORT);
          if (!cont) {
            ++nbreak;
            lastbreak = k;
          }
          s_prev = sk;
          nstand += (sk == ZMPC_STANDING);
          kind[k * 64 + lane] = (sk == ZMPC_STANDING) ? CK_STAND : CK_FOOT;
        }
      }
    }
    const int m = nbreak;                                // footsteps in the horizon
    int mw = valid ? m : 0;  // the wave's largest m (wave-uniform): sweep 1's column count
    for (int o = 32; o > 0; o >>= 1) mw = max(mw, __shfl_xor(mw, o));
    mw = __builtin_amdgcn_readfirstlane(mw);
    const int M = m - ((m > 0 && lastbreak == N - 1) ? 1 : 0);  // with rows in the horizon
    const bool stand_mode = (cur == ZMPC_STANDING || nstand == N) && nstand > 0;
    // host sizes MM from the batch; never expected.  Sweep 1 runs at the wave's largest count,
    // clamped to MM, so a wave holding any such lane solves a truncated problem for every
    // lane: flag them all (mw is wave-uniform), no walk reports success from it
    if (mw > MM) fq |= ZMPC_ST_FACTOR;
    // standing bounds (:721-744)
    double slo = 0.0, shi = 0.0;
    {
      const double fcx = __shfl(fc, lane & ~1, 64), fcy = __shfl(fc, lane | 1, 64);
      if (axis == 0) {
        slo = fcx - 0.5 * a.flen;
        shi = fcx + 0.5 * a.flen;
      } else {
        const double yl = side == 0 ? fcy : fcy + 2 * a.fspread;
        const double yr = side == 0 ? fcy - 2 * a.fspread : fcy;
        slo = fmin(yl, yr) - 0.5 * a.fwid;
        shi = fmax(yl, yr) + 0.5 * a.fwid;
      }
    }
    for (int k = 0; k < N; ++k) {
      unsigned char kd = kind[k * 64 + lane];
      if (kd == CK_STAND && !stand_mode) kd = CK_NONE;
      kind[k * 64 + lane] = kd;
      if (kd == CK_NONE) wset[k * 64 + lane] = 0;
    }
    const int nfac = side == 0 ? a.nfl : a.nfr;
    const RowC rc{T, T2, T3, bv, p0, ip0, al, be, ga, a.c1_2, bnd, shi, slo};
    auto vref = [&](int k) -> double {
      if (a.window_mode) return a.vref[(wc * a.vs / 2 + k) * 2 + axis];
      int64_t t = i + 1 + k;
      if (t > a.n - 1) t = a.n - 1;
      return a.vref[wc * a.vs + t * 2 + axis];
    };

    double u0 = 0.0, f0 = 0.0;
    int fstep = 0;  // this solve's failure bits (pass cap, infeasible swing polytope)
    double fsol[MM > 0 ? MM : 1];
    int it = 0, own = 0;  // own: the passes this lane pair needed (diagnostics, ZMPC_HERDT_PROF)
    bool pair_done = false;
    bool again = true;  // (itmax: the most passes of one solve, counter [9])
    while (again) {
      const unsigned long long tp0 = (kProf && a.prof) ? clock64() : 0;
      // ---- sweep 1: backward Riccati over ξ = [x; f] for V_0(x, f), then the footsteps -----
      // Run at the wave's footstep count (NW = 3 + mw columns, wave-uniform): lanes with fewer
      // footsteps carry zero columns, and no lane pays for the MM − mw columns nobody has.
      double fx0 = 0.0;
      unsigned long long tp1 = 0, tpf = 0;
      int klane = -1;  // this lane's last pinned row (sweep 1 meets it first)
      auto sweep1 = [&](auto na_tag) {
        constexpr int NW = decltype(na_tag)::value;  // 3 + footstep columns
        constexpr int MW = NW - 3;
        constexpr int NPW = NW * (NW + 1) / 2;
        double P[NPW], s[NW];
#pragma unroll
        for (int q = 0; q < NPW; ++q) P[q] = 0.0;
#pragma unroll
        for (int q = 0; q < NW; ++q) s[q] = 0.0;
        // row inputs are loaded one row ahead of their use (at one wave per SIMD nothing else
        // hides their latency)
        double vr_next = vref(N - 1);
        int sg_n = segb[(N - 1) * 64 + lane], kd_n = kind[(N - 1) * 64 + lane],
            wk_n = wset[(N - 1) * 64 + lane];
        for (int k = N - 1; k >= 0; --k) {
          const int sg = sg_n, kd = kd_n, wk = wk_n;
          const double vr = vr_next;
          {
            const int k1 = k > 0 ? k - 1 : 0;
            vr_next = vref(k1);
            sg_n = segb[k1 * 64 + lane];
            kd_n = kind[k1 * 64 + lane];
            wk_n = wset[k1 * 64 + lane];
          }
          double pbx[3], sb, Kx[3], kff;
          herdt_row<NW>(rc, P, s, vr, (sg == 0) ? fc : 0.0, sg - 1, kd, wk, pbx, sb, Kx, kff);
          klane = (wk != 0 && klane < 0) ? k : klane;
        }
        if (kProf && a.prof) tp1 = clock64();
        // ---- footsteps: minimise V_0(x, f) over f, first footstep in the polytope (:771-783)
        double g[MW > 0 ? MW : 1];
#pragma unroll
        for (int q = 0; q < MW; ++q)
          g[q] = s[3 + q] - (P[sidx<NW>(0, 3 + q)] * x[0] + P[sidx<NW>(1, 3 + q)] * x[1] +
                             P[sidx<NW>(2, 3 + q)] * x[2]);
        double sig = 1.0, uu = fc;  // marginal of the first footstep: ½σ(f0 − uu)²
        double gf[MW > 0 ? MW : 1], e0[MW > 0 ? MW : 1];  // F⁻¹g, F⁻¹e₀
        if constexpr (MW > 0) {
          if (M > 0) {
          double L[MW][MW], id[MW];
          if (!small_chol<NW, MW>(P, M, L, id)) fq |= ZMPC_ST_FACTOR;
#pragma unroll
          for (int q = 0; q < MW; ++q) {
            gf[q] = g[q];
            e0[q] = (q == 0) ? 1.0 : 0.0;
          }
          small_chol_solve<MW>(L, id, M, gf);
          small_chol_solve<MW>(L, id, M, e0);
          sig = 1.0 / e0[0];  // 1 / (F⁻¹)₀₀
          uu = gf[0];
          }
        }
        if (m > 0) {
          // pair exchange: x lane = even, y lane = odd
          const double sx = __shfl(sig, lane & ~1, 64), sy = __shfl(sig, lane | 1, 64);
          const double ux = __shfl(uu, lane & ~1, 64), uy = __shfl(uu, lane | 1, 64);
          const double fcx = __shfl(fc, lane & ~1, 64), fcy = __shfl(fc, lane | 1, 64);
          double dx, dy;
          if (!polytope_qp(pl, side, nfac, sx, sy, ux - fcx, uy - fcy, &dx, &dy))
            fstep |= ZMPC_ST_INFEASIBLE;
          fx0 = axis ? fcy + dy : fcx + dx;
        }
        // the other footsteps minimise V_0 with f0 fixed: the KKT point of F f − g = μ e₀ is
        // f = F⁻¹g + μ F⁻¹e₀ with μ from f0 = fx0
#pragma unroll
        for (int q = 0; q < MM; ++q) fsol[q] = 0.0;
        if (MW > 0 && M > 0) {
          const double mu = (fx0 - gf[0]) / e0[0];
#pragma unroll
          for (int q = 1; q < MW; ++q)
            if (q < M) fsol[q] = fma(mu, e0[q], gf[q]);
        }
        if (m > 0) fsol[0] = fx0;  // (M = 0: the only footstep lies past the horizon)
        if (kProf && a.prof) tpf = clock64();
      };
      switch (mw) {
        case 0: sweep1(std::integral_constant<int, 3>{}); break;
        case 1: sweep1(std::integral_constant<int, 3 + (1 <= MM ? 1 : MM)>{}); break;
        case 2: sweep1(std::integral_constant<int, 3 + (2 <= MM ? 2 : MM)>{}); break;
        case 3: sweep1(std::integral_constant<int, 3 + (3 <= MM ? 3 : MM)>{}); break;
        case 4: sweep1(std::integral_constant<int, 3 + (4 <= MM ? 4 : MM)>{}); break;
        case 5: sweep1(std::integral_constant<int, 3 + (5 <= MM ? 5 : MM)>{}); break;
        case 6: sweep1(std::integral_constant<int, 3 + (6 <= MM ? 6 : MM)>{}); break;
        case 7: sweep1(std::integral_constant<int, 3 + (7 <= MM ? 7 : MM)>{}); break;
        default: sweep1(std::integral_constant<int, 3 + MM>{}); break;
      }
      // rows past the wave's last pinned row (the free tail) take K from ktab; the slab keeps
      // only their kff
      int kw = valid ? klane : -1;
      for (int o = 32; o > 0; o >>= 1) kw = max(kw, __shfl_xor(kw, o));
      kw = __builtin_amdgcn_readfirstlane(kw);
      f0 = fx0;
      // ---- sweep 2: the 3-state Riccati with every ZMP centre known (c_k = fc or f_jf), whose
      // control law is the augmented one at f = fsol; slab rows: 4 doubles ---------------------
      cen[lane] = fc;
#pragma unroll
      for (int q = 0; q < MM; ++q) cen[(q + 1) * 64 + lane] = fsol[q];
      // (a segment past MM cannot occur: such a window flags ZMPC_ST_FACTOR above)
      auto centre = [&](int sg) -> double { return cen[(sg <= MM ? sg : 0) * 64 + lane]; };
      {
        double P3[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, s3[3] = {0.0, 0.0, 0.0};
        if (kw >= 0 && kw + 1 < N) {
#pragma unroll
          for (int q = 0; q < 6; ++q) P3[q] = ptab[(kw + 1) * 6 + q];  // V_{kw+1}, all free
        }
        // v_ref rows arrive in blocks of VB, each block's loads issued one block ahead and
        // before the slab stores of the block in hand (vector loads and stores retire through
        // one in-order counter, vmcnt: a load issued after a row's stores is waited for only
        // once those stores are acknowledged)
        constexpr int VB = 8;
        double vb[VB], vn[VB];
#pragma unroll
        for (int r = 0; r < VB; ++r) vb[r] = vref(max(N - 1 - r, 0));
        for (int k0 = N - 1; k0 >= 0; k0 -= VB) {
#pragma unroll
          for (int r = 0; r < VB; ++r) vn[r] = vref(max(k0 - VB - r, 0));
          int sgb[VB], kdb[VB], wkb[VB];  // the block's LDS row bytes, all in flight together
#pragma unroll
          for (int r = 0; r < VB; ++r) {
            const int k = max(k0 - r, 0);
            sgb[r] = segb[k * 64 + lane];
            kdb[r] = kind[k * 64 + lane];
            wkb[r] = wset[k * 64 + lane];
          }
#pragma unroll
          for (int r = 0; r < VB; ++r) {
            const int k = k0 - r;
            if (k >= 0) {
              const double ck = centre(sgb[r]);
              if (k > kw) {
                // free tail (rows past the wave's last pinned row): the s recursion with
                // ktab's K, 1/Huu
                double kff;
                herdt_tail_row(rc, s3, vb[r], ck, ktab + k * 4, kff);
                S(k, 3) = kff;
              } else {
                const int kd = kdb[r], wk = wkb[r];
                double pbx[3], sb, Kx[3], kff;
                herdt_row<3>(rc, P3, s3, vb[r], ck, -1, kd, wk, pbx, sb, Kx, kff);
                // slab row: the control law of a free row, the costate map of a pinned one
                const bool pin = wk != 0;
                S(k, 0) = pin ? pbx[0] : Kx[0];
                S(k, 1) = pin ? pbx[1] : Kx[1];
                S(k, 2) = pin ? pbx[2] : Kx[2];
                S(k, 3) = pin ? sb : kff;
              }
            }
          }
#pragma unroll
          for (int r = 0; r < VB; ++r) vb[r] = vn[r];
        }
      }
      // ---- forward: roll out, primal check of the free rows, dual check of the pinned rows --
      // A pinned row's multiplier comes from the stationarity of its u:
      //   ν_k p0 = −(α u + β b_v (v − vr) + γ p0 (z − c) + B̂ᵀλ_{k+1}),
      //   λ_{k+1} = ∇_x V_{k+1}(x_{k+1}) = P x_{k+1} − s of sweep 2 at row k + 1,
      // so B̂ᵀλ_{k+1} = (PB̂)·x_{k+1} − B̂ᵀs from the slab (the reference's KKT multiplier of
      // that row; the same value a backward costate sweep accumulates).
      // Slab rows are loaded RB at a time: at one wave per SIMD nothing else hides the
      // latency of a row's loads.
      bool changed = false;
      const unsigned long long tp2 = (kProf && a.prof) ? clock64() : 0;
      {
        double xs[3] = {x[0], x[1], x[2]};
        // rows [kb, ke) in blocks of RB; TAIL: K from ktab (rows past the wave's last pinned
        // row), only kff from the slab
        auto fwd = [&](auto tail_tag, int kb, int ke) {
          constexpr bool TAIL = decltype(tail_tag)::value;
          for (int k0 = kb; k0 < ke; k0 += RB) {
            // every load of the block is issued before the first use
            double fk[RB][4], vrb[RB];
            int sgb[RB], kdb[RB], wkb[RB];
#pragma unroll
            for (int r = 0; r < RB; ++r) {
              const int k = min(k0 + r, ke - 1);  // rows past ke: loaded, never used
              if (TAIL) {
                fk[r][0] = ktab[k * 4 + 0];
                fk[r][1] = ktab[k * 4 + 1];
                fk[r][2] = ktab[k * 4 + 2];
              } else {
                fk[r][0] = S(k, 0);
                fk[r][1] = S(k, 1);
                fk[r][2] = S(k, 2);
              }
              fk[r][3] = S(k, 3);
              vrb[r] = vref(k);
              sgb[r] = segb[k * 64 + lane];
              kdb[r] = kind[k * 64 + lane];
              wkb[r] = TAIL ? 0 : wset[k * 64 + lane];
            }
            if (kProf && a.prof) {
              // diagnostics: how long the block's loads keep the wave waiting
              const unsigned long long tw = clock64();
              __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (gfx9 encoding)
              pr_lw += clock64() - tw;
            }
#pragma unroll
            for (int r = 0; r < RB; ++r) {
              const int k = k0 + r;
              if (k < ke) {
                // branch-free: both control laws and both checks, merged by selects (at one
                // wave per SIMD the exec-mask bookkeeping of divergent free/pinned rows cost
                // more than the arithmetic it skipped)
                const int kd = kdb[r], wk = wkb[r];
                const double ccost = centre(sgb[r]);
                const bool pin = wk != 0, foot = kd == CK_FOOT;
                const double hi = foot ? bnd : shi, lo = foot ? -bnd : slo;
                const double ccon = foot ? ccost : 0.0;
                const double cx = c1[0] * xs[0] + c1[1] * xs[1] + c1[2] * xs[2];
                // free: u = −K x − kff; pinned: c1ᵀx + p0 u − ccon = t (ccon: the foot centre)
                const double ufree =
                    -(fk[r][0] * xs[0] + fk[r][1] * xs[1] + fk[r][2] * xs[2]) - fk[r][3];
                const double upin = ((wk == 1 ? hi : lo) + ccon - cx) * ip0;
                const double u = pin ? upin : ufree;
                if (k == 0) u0 = u;
                const double z = cx + p0 * u;
                const double v = ev[1] * xs[1] + ev[2] * xs[2] + bv * u;
                const double y0 = xs[0] + T * xs[1] + T2 * xs[2] + T3 * u;
                const double y1 = xs[1] + T * xs[2] + T2 * u;
                const double y2 = xs[2] + T * u;
                xs[0] = y0;
                xs[1] = y1;
                xs[2] = y2;
                // primal check of a free row with a constraint
                const double tol = 1e-11;
                const double zz = z - ccon;
                const int nf = (zz > hi + tol) ? 1 : ((zz < lo - tol) ? 2 : 0);
                // a pinned row's multiplier (slab: (PB̂)_x, B̂ᵀs of V_{k+1})
                const double bl = fk[r][0] * y0 + fk[r][1] * y1 + fk[r][2] * y2 - fk[r][3];
                const double gu = al * u + be * bv * (v - vrb[r]) + ga * p0 * (z - ccost) + bl;
                const double nu = -gu * ip0;  // ≥ 0 at an upper, ≤ 0 at a lower bound
                const double tn = 1e-10 * (1.0 + fabs(nu));
                const bool drop = (wk == 1 && nu < -tn) || (wk == 2 && nu > tn);
                const int nw = pin ? (drop ? 0 : wk) : (kd != CK_NONE ? nf : 0);
                if (nw != wk) {
                  wset[k * 64 + lane] = (unsigned char)nw;
                  changed = true;
                }
              }
            }
          }
        };
        fwd(std::false_type{}, 0, kw + 1);
        fwd(std::true_type{}, kw + 1, N);
      }
      if (kProf && a.prof) {
        int kl = -1;
        for (int k = 0; k < N; ++k)
          if (wset[k * 64 + lane] != 0) kl = k;
        for (int o = 32; o > 0; o >>= 1) kl = max(kl, __shfl_xor(kl, o));
        pr_kw += (unsigned long long)(kl + 1);
        int nset = 0;
        for (int k = 0; k < N; ++k) nset += wset[k * 64 + lane] != 0;
        pr_ns += (unsigned long long)nset;
        const unsigned long long tp3 = clock64();
        pr_b += tp1 - tp0;
        pr_f += tp2 - tp1;
        pr_fs += tpf - tp1;
        pr_w += tp3 - tp2;
      }
      ++it;
      ++n_wave_pass;
      if (kProf && a.prof) {
        const bool pch = changed || (__shfl_xor(changed ? 1 : 0, 1, 64) != 0);
        if (!pair_done) {
          ++own;
          pair_done = !pch;
        }
      }
      if (valid) {
        ++n_pass;
        n_m += (unsigned)m;
        n_m2 += (unsigned)(m * m);
      }
      if (changed && it >= a.maxit) {
        fstep |= ZMPC_ST_MAXITER;
        changed = false;
      }
      // the pair runs its passes together (the polytope solve reads both lanes)
      again = __any(changed && valid);
    }
    if (valid) itmax = max(itmax, (unsigned)it);
    if (valid) pr_own += (unsigned long long)own;
    // an infeasible joint QP (either lane of the pair) — the analogue of OSQP returning no
    // solution — takes the reference's fallback (zmp_controller.py:796-802): zero jerk on both
    // axes and the first footstep at the air foot's centre.  A solve at the pass cap keeps its
    // last iterate, as OSQP does at its iteration limit.  The walk's status keeps both bits.
    fq |= fstep;
    if (((fstep | __shfl_xor(fstep, 1, 64)) & ZMPC_ST_INFEASIBLE) != 0) {
      u0 = 0.0;
      if (m > 0) f0 = air;
    }
    // ---- advance (reference form x⁺ = A x + B u0, zmp_controller.py:809-810) ----------------
    double xn[3];
    xn[0] = x[0] + T * x[1] + T2 * x[2] + T3 * u0;
    xn[1] = x[1] + T * x[2] + T2 * u0;
    xn[2] = x[2] + T * u0;
    if (!(isfinite(xn[0]) && isfinite(xn[1]) && isfinite(xn[2]))) fq |= ZMPC_ST_NONFINITE;
    if (a.window_mode) {
      if (valid) {
        double* o = a.hist + (wc * 2 + axis) * 3;
        o[0] = xn[0];
        o[1] = xn[1];
        o[2] = xn[2];
        a.foot[wc * 2 + axis] = (m > 0) ? f0 : __builtin_nan("");
      }
      x[0] = xn[0];
      x[1] = xn[1];
      x[2] = xn[2];
      break;
    }
    // foot bookkeeping (:497-529)
    const int nbi = a.nb[wc * a.ns + i];
    if (m > 0) air += (1.0 / (double)nbi) * (f0 - air);
    const int nxt = a.st[wc * a.ss + i + 1];
    if (nxt != cur && cur == ZMPC_SINGLE_SUPPORT) {
      side = 1 - side;
      fc = (m > 0) ? f0 : air;
      air = fc;
    }
    if (i == kstep) xn[1] -= kv;  // F_ext impulse on the y state (:525-526)
    if (nxt != cur) cur = nxt;
    x[0] = xn[0];
    x[1] = xn[1];
    x[2] = xn[2];
    if (valid) {
      double* h = a.hist + ((wc * a.n + i + 1) * 2 + axis) * 3;
      h[0] = x[0];
      h[1] = x[1];
      h[2] = x[2];
      a.foot[(wc * a.n + i + 1) * 2 + axis] = fc;
    }
    // warm start: the converged set shifted one row towards the present
    // (round 3, config 6: row N−1 a copy of the old last row instead of free — 1.316 → 1.157
    // passes per solve, 86.4 → 78.6 ms; the converged set and the solution do not change)
    // (row N−1 keeps its value; freeing row N−2 as the strict kernel does changed nothing here,
    // 1.316 passes either way, and keeping the last 2–3 rows unshifted equals the copy)
    for (int k = 0; k < N - 1; ++k) wset[k * 64 + lane] = wset[(k + 1) * 64 + lane];
  }
  if (valid && a.status != nullptr) {
    const int other = __shfl(fq, lane ^ 1, 64);
    if (axis == 0) a.status[wc] = fq | other;
  }
  if (kProf && a.prof) {
    for (int o = 32; o > 0; o >>= 1) {
      pr_ns += __shfl_xor(pr_ns, o);
      pr_own += __shfl_xor(pr_own, o);
    }
    if (lane == 0) {
      atomicAdd(a.prof + 0, pr_b);
      atomicAdd(a.prof + 1, pr_f);
      atomicAdd(a.prof + 2, pr_w);
      atomicAdd(a.prof + 3, clock64() - pr_t0);
      atomicAdd(a.prof + 4, pr_kw);
      atomicAdd(a.prof + 5, pr_ns);
      atomicAdd(a.prof + 6, n_wave_pass);
      atomicAdd(a.prof + 7, pr_own);
      atomicAdd(a.prof + 8, pr_fs);
      atomicAdd(a.prof + 9, pr_lw);
    }
  }
  if (a.cnt) {
    for (int o = 32; o > 0; o >>= 1) {
      n_pass += __shfl_xor(n_pass, o);
      n_m += __shfl_xor(n_m, o);
      n_m2 += __shfl_xor(n_m2, o);
      itmax = max(itmax, (unsigned)__shfl_xor((int)itmax, o));
    }
    if (lane == 0) {
      atomicAdd(a.cnt + 4, n_wave_pass);
      atomicAdd(a.cnt + 5, n_pass);
      atomicAdd(a.cnt + 6, n_m);
      atomicAdd(a.cnt + 7, n_m2);
      atomicMax(a.cnt + 9, (unsigned long long)itmax);
    }
  }
}

}  // namespace

hipError_t zmpc_launch_herdt(const zmpc_plan* p, const zmpc_herdt_params* prm, int64_t B,
                             int64_t n, int window_mode, const double* vref, int64_t vs,
                             const int8_t* st, int64_t ss, const int32_t* nb, int64_t ns,
                             const double* x0, const double* kick, int64_t kick_step,
                             const int8_t* cur0, const double* fc0, const int8_t* side0,
                             double* hist, double* foot, int32_t* status, hipStream_t s,
                             std::string* why) {
  HerdtArgs a{};
  a.N = p->N;
  a.window_mode = window_mode;
  a.n = n;
  a.B = B;
  a.T = p->T;
  a.T2 = p->T2_2;
  a.T3 = p->T3_6;
  a.c1_2 = p->T2_2 - p->hg;
  a.p0 = p->T3_6 - p->Thg;
  a.alpha = prm->alpha;
  a.beta = prm->beta;
  a.gamma = prm->gamma;
  a.bx = 0.5 * prm->foot_length;
  a.by = 0.5 * prm->foot_width;
  a.flen = prm->foot_length;
  a.fwid = prm->foot_width;
  a.fspread = prm->foot_spread;
  a.nfl = prm->nfacets[0];
  a.nfr = prm->nfacets[1];
  for (int sd = 0; sd < 2; ++sd)
    for (int f = 0; f < ZMPC_HERDT_MAX_FACETS; ++f)
      for (int c = 0; c < 3; ++c) a.poly[sd][f][c] = prm->facets[sd][f][c];
  a.vref = vref;
  a.vs = vs;
  a.st = st;
  a.ss = ss;
  a.nb = nb;
  a.ns = ns;
  a.x0 = x0;
  a.kick = kick;
  a.kick_step = kick_step;
  a.cur0 = cur0;
  a.fc0 = fc0;
  a.side0 = side0;
  a.hist = hist;
  a.foot = foot;
  a.status = status;
  a.cnt = p->lqcnt;
#ifdef ZMPC_DIAG
  static unsigned long long* prof = [] {  // diagnostics build: per-phase clocks to stderr
    unsigned long long* q = nullptr;
    if (getenv("ZMPC_HERDT_PROF") && hipMalloc((void**)&q, 10 * sizeof(unsigned long long)) != hipSuccess)
      q = nullptr;
    return q;
  }();
  if (prof) (void)hipMemsetAsync(prof, 0, 10 * sizeof(unsigned long long), s);
  a.prof = prof;
#else
  a.prof = nullptr;
#endif
  a.maxit = prm->max_passes > 0 ? prm->max_passes : HMAXIT;
  const int mm = prm->max_footsteps;
  const int MM = mm <= 2 ? 2 : mm <= 4 ? 4 : mm <= 6 ? 6 : mm <= 7 ? 7 : mm <= 8 ? 8 : 0;
  if (MM == 0) {
    *why = "more than 8 footsteps inside one horizon window";
    return hipErrorInvalidValue;
  }
  a.nf = SLAB;
  const int64_t blocks = (B + 31) / 32;
  const size_t slab = (size_t)blocks * a.N * (a.nf * 64 + 6) * sizeof(double);
  if (hipMallocAsync((void**)&a.ws, slab, s) != hipSuccess) {
    (void)hipGetLastError();
    return hipErrorOutOfMemory;
  }
  const size_t lds = (((size_t)3 * a.N * 64 + 15) & ~(size_t)15) + sizeof(PolyLds) +
                     (size_t)a.N * 4 * sizeof(double) + (size_t)(8 + 1) * 64 * sizeof(double);
  if (lds > 160 * 1024) {
    (void)hipFreeAsync(a.ws, s);
    *why = "horizon too long for the Herdt solver's LDS flags";
    return hipErrorInvalidValue;
  }
  switch (MM) {
    case 2:
      hipLaunchKernelGGL(zmpc_herdt_kernel<2>, dim3((unsigned)blocks), dim3(64), lds, s, a);
      break;
    case 4:
      hipLaunchKernelGGL(zmpc_herdt_kernel<4>, dim3((unsigned)blocks), dim3(64), lds, s, a);
      break;
    case 6:
      hipLaunchKernelGGL(zmpc_herdt_kernel<6>, dim3((unsigned)blocks), dim3(64), lds, s, a);
      break;
    case 7:
      hipLaunchKernelGGL(zmpc_herdt_kernel<7>, dim3((unsigned)blocks), dim3(64), lds, s, a);
      break;
    default:
      hipLaunchKernelGGL(zmpc_herdt_kernel<8>, dim3((unsigned)blocks), dim3(64), lds, s, a);
      break;
  }
  hipError_t e = hipGetLastError();
  const hipError_t ef = hipFreeAsync(a.ws, s);
  if (a.prof && e == hipSuccess) {
    unsigned long long h[10];
    (void)hipMemcpy(h, a.prof, sizeof(h), hipMemcpyDeviceToHost);
    const double t = (double)(h[3] ? h[3] : 1), wp = (double)(h[6] ? h[6] : 1);
    fprintf(stderr,
            "herdt prof: backward %.3f footsteps+sweep2 %.3f (footsteps alone %.3f) forward %.3f "
            "(its slab-load waits %.3f) (of %llu clocks/wave); "
            "rows to the wave's last pinned row %.1f, pinned rows per lane %.2f (per pass); "
            "lane-pair passes needed %llu vs wave passes x 64 %llu\n",
            h[0] / t, h[1] / t, h[8] / t, h[2] / t, h[9] / t, h[3] / (unsigned long long)blocks,
            h[4] / wp, h[5] / (wp * 64), h[7], h[6] * 64);
  }
  return e != hipSuccess ? e : ef;
}

hipError_t zmpc_herdt_set_attrs() {
  hipError_t e = hipSuccess;
  const void* ks[] = {(const void*)zmpc_herdt_kernel<2>, (const void*)zmpc_herdt_kernel<4>,
                      (const void*)zmpc_herdt_kernel<6>, (const void*)zmpc_herdt_kernel<7>,
                      (const void*)zmpc_herdt_kernel<8>};
  for (const void* k : ks)
    if (e == hipSuccess)
      e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  return e;
}
