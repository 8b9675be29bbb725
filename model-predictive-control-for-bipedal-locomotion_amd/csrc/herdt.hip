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
// Mapping: one lane per (walk, axis), lanes 2w and 2w+1 = axes x, y of walk w; a one-wave
// workgroup holds 32 walks.  Per-row feedback and forward values go through a per-wave global
// slab ([row][field][64]); per-row segment index, constraint kind and working-set flag are LDS
// bytes.
#include <cstdio>

#include "zmpc_internal.h"

namespace {

constexpr int HMAXIT = 64;  // active-set pass cap (ZMPC_ST_MAXITER beyond)

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
};

// Row fields of the slab: K (3), kff, u, ev (= v − vr), ez (= z − c), Kf (MM)
constexpr int F_K = 0, F_KFF = 3, F_U = 4, F_EV = 5, F_EZ = 6, F_KF = 7;

// packed symmetric index (a <= b)
template <int NA>
__device__ __forceinline__ constexpr int sidx(int a, int b) {
  return a <= b ? a * NA - a * (a - 1) / 2 + (b - a) : b * NA - b * (b - 1) / 2 + (a - b);
}

// Exact minimiser of ½σx(dx − ux)² + ½σy(dy − uy)² over {d : a_i·d <= b_i}: the interior
// point, else the best feasible point among the facet-line projections and the vertices.
__device__ void polytope_qp(const double (*P)[3], int nfac, double sx, double sy, double ux,
                            double uy, double* dx, double* dy) {
  const double tol = 1e-12;
  auto feasible = [&](double px, double py) {
    for (int i = 0; i < nfac; ++i)
      if (P[i][0] * px + P[i][1] * py > P[i][2] + tol) return false;
    return true;
  };
  if (feasible(ux, uy)) {
    *dx = ux;
    *dy = uy;
    return;
  }
  double best = 1e300, bx = ux, by = uy;
  auto consider = [&](double px, double py) {
    if (!feasible(px, py)) return;
    const double v = 0.5 * sx * (px - ux) * (px - ux) + 0.5 * sy * (py - uy) * (py - uy);
    if (v < best) {
      best = v;
      bx = px;
      by = py;
    }
  };
  for (int i = 0; i < nfac; ++i) {
    const double ax = P[i][0], ay = P[i][1], b = P[i][2];
    const double den = ax * ax / sx + ay * ay / sy;
    const double t = (ax * ux + ay * uy - b) / den;
    consider(ux - t * ax / sx, uy - t * ay / sy);
    for (int j = i + 1; j < nfac; ++j) {
      const double cx = P[j][0], cy = P[j][1], c = P[j][2];
      const double det = ax * cy - ay * cx;
      if (fabs(det) < 1e-14) continue;
      consider((b * cy - ay * c) / det, (ax * c - b * cx) / det);
    }
  }
  *dx = bx;
  *dy = by;
}

// In-place Cholesky solve of the M×M block F (packed, NA-indexed at offset 3) for rhs g (M).
template <int NA, int MM>
__device__ __forceinline__ bool small_chol_solve(const double* P, int M, double* g) {
  double L[MM][MM];
#pragma unroll
  for (int i = 0; i < MM; ++i)
#pragma unroll
    for (int j = 0; j < MM; ++j) L[i][j] = (i < M && j <= i) ? P[sidx<NA>(3 + i, 3 + j)] : 0.0;
  bool ok = true;
#pragma unroll
  for (int k = 0; k < MM; ++k) {
    if (k < M) {
      double d = L[k][k];
#pragma unroll
      for (int q = 0; q < MM; ++q)
        if (q < k) d -= L[k][q] * L[k][q];
      ok = ok && d > 0.0;
      const double piv = sqrt(fmax(d, 1e-300));
      L[k][k] = piv;
#pragma unroll
      for (int i = 0; i < MM; ++i) {
        if (i > k && i < M) {
          double v = L[i][k];
#pragma unroll
          for (int q = 0; q < MM; ++q)
            if (q < k) v -= L[i][q] * L[k][q];
          L[i][k] = v / piv;
        }
      }
    }
  }
  // forward / backward substitution
#pragma unroll
  for (int i = 0; i < MM; ++i) {
    if (i < M) {
      double v = g[i];
#pragma unroll
      for (int q = 0; q < MM; ++q)
        if (q < i) v -= L[i][q] * g[q];
      g[i] = v / L[i][i];
    }
  }
#pragma unroll
  for (int i = MM - 1; i >= 0; --i) {
    if (i < M) {
      double v = g[i];
#pragma unroll
      for (int q = 0; q < MM; ++q)
        if (q > i && q < M) v -= L[q][i] * g[q];
      g[i] = v / L[i][i];
    }
  }
  return ok;
}

enum : unsigned char { CK_NONE = 0, CK_FOOT = 1, CK_STAND = 2 };

template <int MM>
__global__ void __launch_bounds__(64) zmpc_herdt_kernel(HerdtArgs a) {
  constexpr int NA = 3 + MM;
  constexpr int NP = NA * (NA + 1) / 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char hsm[];
  const int lane = threadIdx.x;
  const int N = a.N;
  unsigned char* segb = hsm;              // [N][64] support segment of row k (0 = current foot)
  unsigned char* kind = hsm + N * 64;     // [N][64] constraint kind
  unsigned char* wset = hsm + 2 * N * 64; // [N][64] working set: 0 free, 1 upper, 2 lower
  const int64_t w = (int64_t)blockIdx.x * 32 + (lane >> 1);
  const int axis = lane & 1;
  const bool valid = w < a.B;
  const int64_t wc = valid ? w : 0;  // clamped walk for loads (invalid lanes compute garbage)
  double* slab = a.ws + (size_t)blockIdx.x * N * a.nf * 64;
  auto S = [&](int k, int f) -> double& { return slab[((size_t)k * a.nf + f) * 64 + lane]; };

  const double T = a.T, T2 = a.T2, T3 = a.T3;
  const double c1[3] = {1.0, T, a.c1_2};
  const double ev[3] = {0.0, 1.0, T};
  const double Bv[3] = {T3, T2, T};
  const double p0 = a.p0, bv = T2;
  const double al = a.alpha, be = a.beta, ga = a.gamma;
  const double bnd = axis ? a.by : a.bx;

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
    for (int k = 0; k < N; ++k) {
      const int sk = wstate(k);
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
    const int m = nbreak;                                // footsteps in the horizon
    const int M = m - ((m > 0 && lastbreak == N - 1) ? 1 : 0);  // with rows in the horizon
    const bool stand_mode = (cur == ZMPC_STANDING || nstand == N) && nstand > 0;
    if (m > MM) fq |= ZMPC_ST_FACTOR;  // host sizes MM from the batch; never expected
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
    const double(*poly)[3] = a.poly[side];
    const int nfac = side == 0 ? a.nfl : a.nfr;
    auto vref = [&](int k) -> double {
      if (a.window_mode) return a.vref[(wc * a.vs / 2 + k) * 2 + axis];
      int64_t t = i + 1 + k;
      if (t > a.n - 1) t = a.n - 1;
      return a.vref[wc * a.vs + t * 2 + axis];
    };

    double u0 = 0.0, f0 = 0.0;
    double fsol[MM > 0 ? MM : 1];
    int it = 0;
    bool again = true;
    while (again) {
      // ---- backward Riccati over ξ = [x; f] --------------------------------------------------
      double P[NP], s[NA];
#pragma unroll
      for (int q = 0; q < NP; ++q) P[q] = 0.0;
#pragma unroll
      for (int q = 0; q < NA; ++q) s[q] = 0.0;
      // global loads are issued one row ahead of their use (at one wave per SIMD nothing else
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
        const int jf = sg - 1;  // footstep column of the ZMP centre (−1: current foot)
        const double fc0 = (sg == 0) ? fc : 0.0;
        // P B̂ (x part of B̂ only)
        double pb[NA];
#pragma unroll
        for (int q = 0; q < NA; ++q)
          pb[q] = P[sidx<NA>(q, 0)] * Bv[0] + P[sidx<NA>(q, 1)] * Bv[1] +
                  P[sidx<NA>(q, 2)] * Bv[2];
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
        // H_ξξ = ÂᵀPÂ + stage
        double H[NP];
        {
          // PA: columns 0..2 transformed by A, f columns unchanged
          double PA[NA][3];
#pragma unroll
          for (int q = 0; q < NA; ++q) {
            const double p0q = P[sidx<NA>(q, 0)], p1q = P[sidx<NA>(q, 1)],
                         p2q = P[sidx<NA>(q, 2)];
            PA[q][0] = p0q;
            PA[q][1] = T * p0q + p1q;
            PA[q][2] = T2 * p0q + T * p1q + p2q;
          }
#pragma unroll
          for (int r = 0; r < NA; ++r)
#pragma unroll
            for (int c = r; c < NA; ++c) {
              double v;
              if (r < 3 && c < 3) {
                // (Aᵀ (P A))[r][c]
                v = (r == 0) ? PA[0][c]
                             : (r == 1) ? T * PA[0][c] + PA[1][c]
                                        : T2 * PA[0][c] + T * PA[1][c] + PA[2][c];
                v += be * ev[r] * ev[c] + ga * c1[r] * c1[c];
              } else if (r < 3) {
                // (Aᵀ P)[r][c] for an f column c
                const double q0 = P[sidx<NA>(0, c)], q1 = P[sidx<NA>(1, c)],
                             q2 = P[sidx<NA>(2, c)];
                v = (r == 0) ? q0 : (r == 1) ? T * q0 + q1 : T2 * q0 + T * q1 + q2;
                if (c - 3 == jf) v += -ga * c1[r];
              } else {
                v = P[sidx<NA>(r, c)];
                if (r - 3 == jf && c - 3 == jf) v += ga;
              }
              H[sidx<NA>(r, c)] = v;
            }
        }
        // control law u = −K̂ ξ − kff
        double Kh[NA], kff;
        if (wk == 0) {
          const double iq = 1.0 / Huu;
#pragma unroll
          for (int q = 0; q < NA; ++q) Kh[q] = Hu[q] * iq;
          kff = -hu * iq;
        } else {
          // pinned: c1ᵀx + p0 u − ccon = t  (ccon: the foot centre on a foot row, 0 standing)
          const bool foot = kd == CK_FOOT;
          const double t = (kd == CK_STAND) ? (wk == 1 ? shi : slo) : (wk == 1 ? bnd : -bnd);
          const double cc0 = foot ? fc0 : 0.0;
          const double ip = 1.0 / p0;
          Kh[0] = c1[0] * ip;
          Kh[1] = c1[1] * ip;
          Kh[2] = c1[2] * ip;
#pragma unroll
          for (int q = 3; q < NA; ++q) Kh[q] = (foot && q - 3 == jf) ? -ip : 0.0;
          kff = -(t + cc0) * ip;
        }
        double D[NA];
#pragma unroll
        for (int q = 0; q < NA; ++q) D[q] = Huu * Kh[q] - Hu[q];
        // V_k: P = H − Hu K̂ᵀ + K̂ Dᵀ (symmetric), s = h − hu K̂ − kff D
#pragma unroll
        for (int r = 0; r < NA; ++r)
#pragma unroll
          for (int c = r; c < NA; ++c)
            P[sidx<NA>(r, c)] = H[sidx<NA>(r, c)] - Hu[r] * Kh[c] + Kh[r] * D[c];
#pragma unroll
        for (int q = 0; q < NA; ++q) s[q] = hx[q] - hu * Kh[q] - kff * D[q];
        S(k, F_K + 0) = Kh[0];
        S(k, F_K + 1) = Kh[1];
        S(k, F_K + 2) = Kh[2];
        S(k, F_KFF) = kff;
#pragma unroll
        for (int q = 0; q < MM; ++q) S(k, F_KF + q) = Kh[3 + q];
      }
      // ---- footsteps: minimise V_0(x, f) over f, first footstep in the polytope (:771-783)
      double g[MM > 0 ? MM : 1];
#pragma unroll
      for (int q = 0; q < MM; ++q)
        g[q] = s[3 + q] -
               (P[sidx<NA>(0, 3 + q)] * x[0] + P[sidx<NA>(1, 3 + q)] * x[1] +
                P[sidx<NA>(2, 3 + q)] * x[2]);
      double sig = 1.0, uu = fc;  // marginal of the first footstep: ½σ(f0 − uu)²
      if (M > 0) {
        double gf[MM > 0 ? MM : 1];
#pragma unroll
        for (int q = 0; q < MM; ++q) gf[q] = g[q];
        if (!small_chol_solve<NA, MM>(P, M, gf)) fq |= ZMPC_ST_FACTOR;
        double e0[MM > 0 ? MM : 1];
#pragma unroll
        for (int q = 0; q < MM; ++q) e0[q] = (q == 0) ? 1.0 : 0.0;
        small_chol_solve<NA, MM>(P, M, e0);
        sig = 1.0 / e0[0];  // 1 / (F⁻¹)₀₀
        uu = gf[0];
      }
      double fx0 = 0.0;
      if (m > 0) {
        // pair exchange: x lane = even, y lane = odd
        const double sx = __shfl(sig, lane & ~1, 64), sy = __shfl(sig, lane | 1, 64);
        const double ux = __shfl(uu, lane & ~1, 64), uy = __shfl(uu, lane | 1, 64);
        const double fcx = __shfl(fc, lane & ~1, 64), fcy = __shfl(fc, lane | 1, 64);
        double dx, dy;
        polytope_qp(poly, nfac, sx, sy, ux - fcx, uy - fcy, &dx, &dy);
        fx0 = axis ? fcy + dy : fcx + dx;
      }
      // remaining footsteps: F_rr f_r = g_r − F_r0 f0
#pragma unroll
      for (int q = 0; q < MM; ++q) fsol[q] = 0.0;
      if (M > 0) {
        fsol[0] = fx0;
        if (M > 1) {
          // solve the (M−1)×(M−1) block by solving the full system with f0 fixed:
          // F [f0; f_r] = [*; g_r]  →  f_r = F_rr⁻¹ (g_r − F_r0 f0), via a shifted copy
          double Pr[NP];
#pragma unroll
          for (int q = 0; q < NP; ++q) Pr[q] = 0.0;
#pragma unroll
          for (int r = 0; r < MM; ++r)
#pragma unroll
            for (int c = r; c < MM; ++c)
              if (r + 1 < MM && c + 1 < MM)
                Pr[sidx<NA>(3 + r, 3 + c)] = P[sidx<NA>(3 + r + 1, 3 + c + 1)];
          double gr[MM > 0 ? MM : 1];
#pragma unroll
          for (int q = 0; q < MM; ++q)
            gr[q] = (q + 1 < MM) ? g[q + 1] - P[sidx<NA>(3, 3 + q + 1)] * fx0 : 0.0;
          small_chol_solve<NA, MM>(Pr, M - 1, gr);
#pragma unroll
          for (int q = 1; q < MM; ++q)
            if (q < M) fsol[q] = gr[q - 1];
        }
      } else if (m > 0) {
        fsol[0] = fx0;  // the only footstep lies past the horizon: nearest polytope point
      }
      f0 = fx0;
      // ---- forward: roll out, primal check ---------------------------------------------------
      bool changed = false;
      {
        double xs[3] = {x[0], x[1], x[2]};
        // row k's feedback (K, kff, Kf·f) and v_ref, loaded one row ahead
        double nK0 = S(0, F_K), nK1 = S(0, F_K + 1), nK2 = S(0, F_K + 2), nkf = S(0, F_KFF);
#pragma unroll
        for (int q = 0; q < MM; ++q) nkf += S(0, F_KF + q) * fsol[q];
        double nvr = vref(0);
        for (int k = 0; k < N; ++k) {
          const int sg = segb[k * 64 + lane];
          const int kd = kind[k * 64 + lane];
          const double K0 = nK0, K1 = nK1, K2 = nK2, fterm = nkf, vrk = nvr;
          {
            const int k1 = k + 1 < N ? k + 1 : k;
            nK0 = S(k1, F_K);
            nK1 = S(k1, F_K + 1);
            nK2 = S(k1, F_K + 2);
            double t = S(k1, F_KFF);
#pragma unroll
            for (int q = 0; q < MM; ++q) t += S(k1, F_KF + q) * fsol[q];
            nkf = t;
            nvr = vref(k1);
          }
          const double u = -(K0 * xs[0] + K1 * xs[1] + K2 * xs[2]) - fterm;
          if (k == 0) u0 = u;
          const double z = c1[0] * xs[0] + c1[1] * xs[1] + c1[2] * xs[2] + p0 * u;
          const double v = ev[1] * xs[1] + ev[2] * xs[2] + bv * u;
          double ccost = fc;
#pragma unroll
          for (int q = 0; q < MM; ++q)
            if (sg - 1 == q) ccost = fsol[q];
          S(k, F_U) = u;
          S(k, F_EV) = v - vrk;
          S(k, F_EZ) = z - ccost;
          const int wk = wset[k * 64 + lane];
          if (kd != CK_NONE && wk == 0) {
            const double tol = 1e-11;
            const double zz = (kd == CK_FOOT) ? z - ccost : z;
            const double hi = (kd == CK_FOOT) ? bnd : shi, lo = (kd == CK_FOOT) ? -bnd : slo;
            const int nf = (zz > hi + tol) ? 1 : ((zz < lo - tol) ? 2 : 0);
            if (nf) {
              wset[k * 64 + lane] = (unsigned char)nf;
              changed = true;
            }
          }
          double y0 = xs[0] + T * xs[1] + T2 * xs[2] + T3 * u;
          double y1 = xs[1] + T * xs[2] + T2 * u;
          double y2 = xs[2] + T * u;
          xs[0] = y0;
          xs[1] = y1;
          xs[2] = y2;
        }
      }
      // ---- costate: multipliers of the pinned rows, dual check --------------------------------
      {
        double lam[3] = {0.0, 0.0, 0.0};
        double nu_ = S(N - 1, F_U), nev = S(N - 1, F_EV), nez = S(N - 1, F_EZ);
        for (int k = N - 1; k >= 0; --k) {
          const double u = nu_, e_v = nev, e_z = nez;
          {
            const int k1 = k > 0 ? k - 1 : 0;
            nu_ = S(k1, F_U);
            nev = S(k1, F_EV);
            nez = S(k1, F_EZ);
          }
          const int wk = wset[k * 64 + lane];
          const double bl = Bv[0] * lam[0] + Bv[1] * lam[1] + Bv[2] * lam[2];
          const double gu = al * u + be * bv * e_v + ga * p0 * e_z + bl;
          double nu = 0.0;
          if (wk != 0) {
            nu = -gu / p0;  // ≥ 0 at an upper, ≤ 0 at a lower bound
            const double tn = 1e-10 * (1.0 + fabs(gu / p0));
            if ((wk == 1 && nu < -tn) || (wk == 2 && nu > tn)) {
              wset[k * 64 + lane] = 0;
              changed = true;
            }
          }
          const double l0 = lam[0], l1 = lam[1], l2 = lam[2];
          const double e = ga * e_z + nu;
          lam[0] = l0 + c1[0] * e;
          lam[1] = T * l0 + l1 + be * ev[1] * e_v + c1[1] * e;
          lam[2] = T2 * l0 + T * l1 + l2 + be * ev[2] * e_v + c1[2] * e;
        }
      }
      ++it;
      if (changed && it >= HMAXIT) {
        fq |= ZMPC_ST_MAXITER;
        changed = false;
      }
      // the pair runs its passes together (the polytope solve reads both lanes)
      again = __any(changed && valid);
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
    for (int k = 0; k < N - 1; ++k) wset[k * 64 + lane] = wset[(k + 1) * 64 + lane];
    wset[(N - 1) * 64 + lane] = 0;
  }
  if (valid && a.status != nullptr) {
    const int other = __shfl(fq, lane ^ 1, 64);
    if (axis == 0) a.status[wc] = fq | other;
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
  const int mm = prm->max_footsteps;
  const int MM = mm <= 2 ? 2 : mm <= 4 ? 4 : mm <= 6 ? 6 : mm <= 7 ? 7 : mm <= 8 ? 8 : 0;
  if (MM == 0) {
    *why = "more than 8 footsteps inside one horizon window";
    return hipErrorInvalidValue;
  }
  a.nf = F_KF + MM;
  const int64_t blocks = (B + 31) / 32;
  const size_t slab = (size_t)blocks * a.N * a.nf * 64 * sizeof(double);
  if (hipMallocAsync((void**)&a.ws, slab, s) != hipSuccess) {
    (void)hipGetLastError();
    return hipErrorOutOfMemory;
  }
  const size_t lds = (size_t)3 * a.N * 64;
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
