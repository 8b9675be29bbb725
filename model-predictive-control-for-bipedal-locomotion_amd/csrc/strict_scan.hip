// Strict (ZMP box-constrained) Wieber QP for small batches: one instance per wavefront, the
// horizon spread over the 64 lanes and the LQ recursions run parallel in time.
//
// Reference (per axis and timestep, cvxpy→OSQP): zmp_controller.py:173-195; the problem, its LQ
// form in η coordinates, the working-set iteration and its tolerances are strict_lq.hip's (same
// step algebra, strict_eta.h).  The lane-per-instance kernel there runs each instance's
// backward and forward sweeps serially over the N slots, so one walk costs 2N dependent steps
// per pass however many lanes are idle.  Here an instance owns a wave; lane l owns the C =
// ⌈N/64⌉ consecutive slots [lC, lC + C):
//
//   backward  each lane composes its slots' one-step elements into one chunk element, a
//             Kogge–Stone suffix scan over the lanes composes the chunks (6 rounds), and the
//             (J, g) part of the lane's right neighbour's suffix is the value function
//             V(η) = ½ηᵀJη − gᵀη at the chunk's end: each lane then runs the ordinary Riccati
//             step (ric_step) back through its own C slots;
//   forward   each lane composes its slots' closed-loop maps (z = −Kη − kff, η⁺ = Fη + e2 z/π,
//             strict_eta.h) into one
//             affine map, a prefix scan over the lanes gives the state at every chunk's start,
//             and each lane rolls through its slots: primal check of the free slots, the pinned
//             slots' multipliers from ∇V_{k+1}(η_{k+1}) (the costate), the new working set.
//
// The element of a span of slots is the conditional value function of Särkkä & García-Fernández
// ("Temporal parallelization of dynamic programming and linear quadratic control", IEEE TAC
// 2023): (A, b, C, g, J) with V_{i→j}(x, y) = max_λ ½xᵀJx − gᵀx + λᵀ(y − Ax − b) − ½λᵀCλ, and
// for e1 then e2 in time, with X = (I + C1 J2)⁻¹:
//   A = A2 X A1,  b = A2 X (b1 + C1 g2) + b2,  C = A2 X C1 A2ᵀ + C2,
//   g = (X A1)ᵀ (g2 − J2 b1) + g1,  J = (X A1)ᵀ J2 A1 + J1.
// A slot's element (the input's cross term with the state eliminated, R = π² + ρ):
//   free      A = Ā − e2 (π/R) c̄ᵀ, b = e2 π r/R, C = e2e2ᵀ/R, J = (ρ/R) c̄c̄ᵀ, g = (ρ r/R) c̄;
//   pinned t  A = Ā − e2 c̄ᵀ/π,     b = e2 t/π,   C = 0,       J = (ρ/π²) c̄c̄ᵀ, g = (ρ t/π²) c̄.
// The value function at the end of the horizon is 0, so the suffix composition's (J, g) at a
// slot is V there.  The working-set iteration, its warm start (the previous timestep's set
// shifted one slot, slot N−2 freed, N−1 kept) and the state advance in the reference form are
// the LQ kernel's, so both kernels converge to the same sets and agree to rounding.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "strict_eta.h"
#include "zmpc_internal.h"

namespace {

using namespace zmpc_eta;

constexpr int SC_MAXIT = 1024;  // active-set pass cap (as strict_lq.hip)
// horizons of the kernel: 32-lane instances to N = 512 (C ≤ 16 slots per lane: 256 VGPRs + 248
// AGPRs), whole-wave ones to 960 (C ≤ 15: 256 + 236; C = 16 of 64 lanes spills 12 B to scratch)
constexpr int kScan32MaxN = 512;
constexpr int kScanMaxN = 960;

struct ScanArgs {
  int N;
  int window_mode;  // 0: rollout of [B, n] walks (both axes); 1: one step of [B, N] windows
  int toff;         // window slot k reads time i + toff + k (1 rollout, 0 step)
  int64_t n, nsteps, ninst;
  const double* zmax;  // rollout [B, n, 2] at b·bstride (bstride 0: one shared walk); step [B, N]
  const double* zmin;
  int64_t bstride;
  const double* x0;  // rollout [B, 2, 3], step [B, 3]
  const double* kick;
  int64_t kick_step;
  const int64_t* kick_steps;
  double* out;  // rollout hist [B, n, 2, 3], step x_next [B, 3]
  int32_t* status;
  unsigned long long* cnt;
  double T, T2, T3, Tsq, Tcu;  // reference-form advance, coordinate scaling
  // z-form step constants (strict_eta.h fill_eta)
  double pi, ipi, ipi2, gp, rho, eps, epsg, epsg2, quz0, epi, tolnu;
  double iR, piR, rhoR, rhoP2;  // slot elements: 1/R, π/R, ρ/R, ρ/π² (R = π² + ρ)
};

// symmetric 3×3 in 6 doubles: 00 01 02 11 12 22
__device__ __forceinline__ constexpr int sy(int i, int j) {
  return i <= j ? (i == 0 ? j : (i == 1 ? 2 + j : 5)) : (j == 0 ? i : (j == 1 ? 2 + i : 5));
}

struct Elem {
  double A[9];  // row-major
  double b[3];
  double C[6];
  double g[3];
  double J[6];
};

__device__ __forceinline__ void elem_identity(Elem& e) {
#pragma unroll
  for (int q = 0; q < 9; ++q) e.A[q] = (q % 4 == 0) ? 1.0 : 0.0;
#pragma unroll
  for (int q = 0; q < 3; ++q) e.b[q] = e.g[q] = 0.0;
#pragma unroll
  for (int q = 0; q < 6; ++q) e.C[q] = e.J[q] = 0.0;
}

// E ← (slot) ∘ E: a slot before the span E.  The slot's element in the parameters
//   A1 = Ā − e2 a2ᵀ, a2 = α c̄ (α = π/R free, 1/π pinned), b1 = b2s e2, C1 = c22 e2e2ᵀ,
//   J1 = κ c̄c̄ᵀ, g1 = γc c̄,
// so that X = (I + C1 J2)⁻¹ differs from I in row 2 only (Sherman–Morrison) and the combine
// reduces to one 3×3 product and rank-1 updates.
template <class Args>
__device__ __forceinline__ void prepend(const Args& a, double al, double b2s, double c22,
                                        double ka, double gc, Elem& E) {
  const double j0 = E.J[sy(0, 2)], j1 = E.J[sy(1, 2)], j2 = E.J[sy(2, 2)];
  const double x2 = recip(fma(c22, j2, 1.0));  // (I + C1 J2)⁻¹ row 2 = (x0, x1, x2)
  const double cx = c22 * x2;
  const double x0 = -cx * j0, x1 = -cx * j1;
  const double g2 = fma(-al, a.gp, 1.0);  // A1[2][2] = 1 − α γ'
  // X A1: rows 0, 1 of Ā; row 2 = x0·[1,1,1] + x1·[0,1,1] + x2·[−α, −α, 1 − αγ']
  const double r20 = fma(-x2, al, x0);
  const double r21 = r20 + x1;
  const double r22 = fma(x2, g2, x0 + x1);
  // A = A2 (X A1)
  double An[9];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double p = E.A[3 * i], q = E.A[3 * i + 1], r = E.A[3 * i + 2];
    An[3 * i + 0] = fma(r, r20, p);
    An[3 * i + 1] = fma(r, r21, p + q);
    An[3 * i + 2] = fma(r, r22, p + q);
  }
  // b = A2 X (b1 + C1 g2) + b2 = A2[:,2] · x2 (b2s + c22 g2_2) + b2
  const double qb = x2 * fma(c22, E.g[2], b2s);
  // C = C2 + c22 x2 (A2 e2)(A2 e2)ᵀ
  const double c0 = E.A[2], c1 = E.A[5], c2 = E.A[8];
#pragma unroll
  for (int i = 0; i < 3; ++i) E.b[i] = fma(E.A[3 * i + 2], qb, E.b[i]);
  E.C[sy(0, 0)] = fma(cx * c0, c0, E.C[sy(0, 0)]);
  E.C[sy(0, 1)] = fma(cx * c0, c1, E.C[sy(0, 1)]);
  E.C[sy(0, 2)] = fma(cx * c0, c2, E.C[sy(0, 2)]);
  E.C[sy(1, 1)] = fma(cx * c1, c1, E.C[sy(1, 1)]);
  E.C[sy(1, 2)] = fma(cx * c1, c2, E.C[sy(1, 2)]);
  E.C[sy(2, 2)] = fma(cx * c2, c2, E.C[sy(2, 2)]);
  // g = A1ᵀ Xᵀ (g2 − J2 b1) + g1
  {
    const double y0 = fma(-b2s, j0, E.g[0]), y1 = fma(-b2s, j1, E.g[1]),
                 y2 = fma(-b2s, j2, E.g[2]);
    const double w0 = fma(x0, y2, y0), w1 = fma(x1, y2, y1), w2 = x2 * y2;
    E.g[0] = fma(-al, w2, w0) + gc;
    E.g[1] = fma(-al, w2, w0 + w1) + gc;
    E.g[2] = fma(g2, w2, w0 + w1) + gc * a.gp;
  }
  // J = A1ᵀ Z A1 + J1, Z = Xᵀ J2 = J2 − c22 x2 j jᵀ (symmetric)
  {
    double Z[6];
    Z[sy(0, 0)] = fma(-cx * j0, j0, E.J[sy(0, 0)]);
    Z[sy(0, 1)] = fma(-cx * j0, j1, E.J[sy(0, 1)]);
    Z[sy(0, 2)] = fma(-cx * j0, j2, E.J[sy(0, 2)]);
    Z[sy(1, 1)] = fma(-cx * j1, j1, E.J[sy(1, 1)]);
    Z[sy(1, 2)] = fma(-cx * j1, j2, E.J[sy(1, 2)]);
    Z[sy(2, 2)] = fma(-cx * j2, j2, E.J[sy(2, 2)]);
    // W = Z A1: columns A1[:,0] = [1,0,−α], A1[:,1] = [1,1,−α], A1[:,2] = [1,1,1−αγ']
    double W[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double z0 = Z[sy(i, 0)], z1 = Z[sy(i, 1)], z2 = Z[sy(i, 2)];
      W[i][0] = fma(-al, z2, z0);
      W[i][1] = W[i][0] + z1;
      W[i][2] = fma(g2, z2, z0 + z1);
    }
    // Jn[p][q] = Σ_i A1[i][p] W[i][q]
    const double ka0 = ka, ka2 = ka * a.gp;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int q = p; q < 3; ++q) {
        const double s01 = W[0][q] + (p >= 1 ? W[1][q] : 0.0);
        const double a2p = (p == 2) ? g2 : -al;
        const double kc = (p == 2 ? ka2 : ka0) * (q == 2 ? a.gp : 1.0);  // κ c̄_p c̄_q
        E.J[sy(p, q)] = fma(a2p, W[2][q], s01) + kc;
      }
  }
#pragma unroll
  for (int q = 0; q < 9; ++q) E.A[q] = An[q];
}

// 3×3 inverse (adjugate / determinant); M = I + C1 J2 has eigenvalues ≥ 1 (C1, J2 ⪰ 0).
__device__ __forceinline__ void inv3(const double* m, double* x) {
  const double c00 = fma(m[4], m[8], -m[5] * m[7]);
  const double c01 = fma(m[5], m[6], -m[3] * m[8]);
  const double c02 = fma(m[3], m[7], -m[4] * m[6]);
  const double id = recip(fma(m[0], c00, fma(m[1], c01, m[2] * c02)));
  x[0] = c00 * id;
  x[3] = c01 * id;
  x[6] = c02 * id;
  x[1] = fma(m[2], m[7], -m[1] * m[8]) * id;
  x[4] = fma(m[0], m[8], -m[2] * m[6]) * id;
  x[7] = fma(m[1], m[6], -m[0] * m[7]) * id;
  x[2] = fma(m[1], m[5], -m[2] * m[4]) * id;
  x[5] = fma(m[2], m[3], -m[0] * m[5]) * id;
  x[8] = fma(m[0], m[4], -m[1] * m[3]) * id;
}

// e1 ← e1 ∘ e2 (e1 first in time), the general combine.
__device__ __forceinline__ void combine(Elem& e1, const Elem& e2) {
  double M[9], X[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      M[3 * i + j] = fma(e1.C[sy(i, 0)], e2.J[sy(0, j)],
                         fma(e1.C[sy(i, 1)], e2.J[sy(1, j)], e1.C[sy(i, 2)] * e2.J[sy(2, j)])) +
                     (i == j ? 1.0 : 0.0);
  inv3(M, X);
  double XA[9];  // X A1
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      XA[3 * i + j] = fma(X[3 * i], e1.A[j], fma(X[3 * i + 1], e1.A[3 + j], X[3 * i + 2] * e1.A[6 + j]));
  // b: A2 X (b1 + C1 g2) + b2
  double t[3], u[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    t[i] = fma(e1.C[sy(i, 0)], e2.g[0], fma(e1.C[sy(i, 1)], e2.g[1], fma(e1.C[sy(i, 2)], e2.g[2], e1.b[i])));
#pragma unroll
  for (int i = 0; i < 3; ++i) u[i] = fma(X[3 * i], t[0], fma(X[3 * i + 1], t[1], X[3 * i + 2] * t[2]));
  double bn[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    bn[i] = fma(e2.A[3 * i], u[0], fma(e2.A[3 * i + 1], u[1], fma(e2.A[3 * i + 2], u[2], e2.b[i])));
  // g: (X A1)ᵀ (g2 − J2 b1) + g1
  double y[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    y[i] = e2.g[i] - fma(e2.J[sy(i, 0)], e1.b[0], fma(e2.J[sy(i, 1)], e1.b[1], e2.J[sy(i, 2)] * e1.b[2]));
#pragma unroll
  for (int j = 0; j < 3; ++j)
    e1.g[j] = fma(XA[j], y[0], fma(XA[3 + j], y[1], fma(XA[6 + j], y[2], e1.g[j])));
  // J: (X A1)ᵀ (J2 A1) + J1
  {
    double JA[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        JA[3 * i + j] = fma(e2.J[sy(i, 0)], e1.A[j],
                            fma(e2.J[sy(i, 1)], e1.A[3 + j], e2.J[sy(i, 2)] * e1.A[6 + j]));
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int q = p; q < 3; ++q)
        e1.J[sy(p, q)] = fma(XA[p], JA[q], fma(XA[3 + p], JA[3 + q], fma(XA[6 + p], JA[6 + q], e1.J[sy(p, q)])));
  }
  // C: A2 (X C1) A2ᵀ + C2
  {
    double XC[9], W[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        XC[3 * i + j] = fma(X[3 * i], e1.C[sy(0, j)], fma(X[3 * i + 1], e1.C[sy(1, j)], X[3 * i + 2] * e1.C[sy(2, j)]));
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        W[3 * i + j] = fma(e2.A[3 * i], XC[j], fma(e2.A[3 * i + 1], XC[3 + j], e2.A[3 * i + 2] * XC[6 + j]));
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int q = p; q < 3; ++q)
        e1.C[sy(p, q)] = fma(W[3 * p], e2.A[3 * q], fma(W[3 * p + 1], e2.A[3 * q + 1], fma(W[3 * p + 2], e2.A[3 * q + 2], e2.C[sy(p, q)])));
  }
  // A: A2 (X A1)
  double An[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      An[3 * i + j] = fma(e2.A[3 * i], XA[j], fma(e2.A[3 * i + 1], XA[3 + j], e2.A[3 * i + 2] * XA[6 + j]));
#pragma unroll
  for (int q = 0; q < 9; ++q) e1.A[q] = An[q];
#pragma unroll
  for (int q = 0; q < 3; ++q) e1.b[q] = bn[q];
}

__device__ __forceinline__ void shfl_elem(const Elem& e, Elem& o, int src) {
#pragma unroll
  for (int q = 0; q < 9; ++q) o.A[q] = __shfl(e.A[q], src, 64);
#pragma unroll
  for (int q = 0; q < 3; ++q) o.b[q] = __shfl(e.b[q], src, 64);
#pragma unroll
  for (int q = 0; q < 6; ++q) o.C[q] = __shfl(e.C[q], src, 64);
#pragma unroll
  for (int q = 0; q < 3; ++q) o.g[q] = __shfl(e.g[q], src, 64);
#pragma unroll
  for (int q = 0; q < 6; ++q) o.J[q] = __shfl(e.J[q], src, 64);
}

// A DPP lane move of a double (two 32-bit moves on the VALU, no LDS pipe) into the rows of
// ROWS (the others read 0); lanes whose source is invalid read 0 (bound_ctrl).
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWS, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWS, 0xF, true);
  return __hiloint2double(hi, lo);
}
// wave_shl:1 / wave_shr:1 — lane i reads lane i + 1 / i − 1 across the whole wave (the instance
// boundaries are the callers' business)
__device__ __forceinline__ double next_lane_f64(double v) { return dpp_f64<0x130>(v); }
__device__ __forceinline__ double prev_lane_f64(double v) { return dpp_f64<0x138>(v); }

// the lane d behind inside the row (row_shr:d, d = 1, 2, 4, 8), or, for d = 16 / 32, the last
// lane of the previous 16 / 32-lane block (row_bcast:15 into rows 1, 3; row_bcast:31 into rows
// 2, 3) — the Kogge-Stone prefix levels of an aligned L-lane instance
__device__ __forceinline__ double prefix_src_f64(double v, int d) {
  switch (d) {
    case 1:
      return dpp_f64<0x111>(v);
    case 2:
      return dpp_f64<0x112>(v);
    case 4:
      return dpp_f64<0x114>(v);
    case 8:
      return dpp_f64<0x118>(v);
    case 16:
      return dpp_f64<0x142, 0xA>(v);
    default:
      return dpp_f64<0x143, 0xC>(v);
  }
}

// row_shl:d — lane i reads lane i + d of its row (d = 1, 2, 4, 8)
__device__ __forceinline__ double row_shl_f64(double v, int d) {
  switch (d) {
    case 1:
      return dpp_f64<0x101>(v);
    case 2:
      return dpp_f64<0x102>(v);
    case 4:
      return dpp_f64<0x104>(v);
    default:
      return dpp_f64<0x108>(v);
  }
}

__device__ __forceinline__ void row_shl_elem(const Elem& e, Elem& o, int d) {
#pragma unroll
  for (int q = 0; q < 9; ++q) o.A[q] = row_shl_f64(e.A[q], d);
#pragma unroll
  for (int q = 0; q < 3; ++q) o.b[q] = row_shl_f64(e.b[q], d);
#pragma unroll
  for (int q = 0; q < 6; ++q) o.C[q] = row_shl_f64(e.C[q], d);
#pragma unroll
  for (int q = 0; q < 3; ++q) o.g[q] = row_shl_f64(e.g[q], d);
#pragma unroll
  for (int q = 0; q < 6; ++q) o.J[q] = row_shl_f64(e.J[q], d);
}

// One wave per workgroup holding 64/L instances of L lanes each; lane l of an instance owns
// slots [lC, lC + C) ∩ [0, N).  The scans stay inside an instance's L lanes; an instance that
// has converged keeps its working set while the others of its wave iterate (a converged set
// reproduces itself, so its extra passes change nothing; they are not counted).
template <int C, int L>
#ifndef ZMPC_SCAN_ONE_WAVE_C  // (chunk widths from which a SIMD holds one wave: A/B builds)
#define ZMPC_SCAN_ONE_WAVE_C 3
#endif
__global__ void __launch_bounds__(64, (C >= ZMPC_SCAN_ONE_WAVE_C ? 1 : 2))
    zmpc_strict_scan_kernel(ScanArgs a) {
  static_assert(L == 64 || L == 32 || L == 16, "lanes per instance");
  const int lane = threadIdx.x;
  const int il = lane & (L - 1);     // lane within the instance
  const int base = lane & ~(L - 1);  // the instance's first lane
  const int N = a.N;
  const int64_t w = (int64_t)blockIdx.x * (64 / L) + lane / L;
  const bool valid = w < a.ninst;
  const int64_t wc = valid ? w : 0;  // (a clamped instance for loads; nothing is written)
  const int64_t b = a.window_mode ? wc : (wc >> 1);
  const int axis = a.window_mode ? 0 : (int)(wc & 1);
  const int k0 = il * C;
  double x[3];
  {
    const double* xp = a.window_mode ? a.x0 + b * 3 : a.x0 + (b * 2 + axis) * 3;
    x[0] = xp[0];
    x[1] = xp[1];
    x[2] = xp[2];
    if (!a.window_mode && il == 0 && valid) {
      double* h = a.out + ((b * a.n) * 2 + axis) * 3;  // hist[b, 0, axis, :] = x0
      h[0] = x[0];
      h[1] = x[1];
      h[2] = x[2];
    }
  }
  const int64_t kstep = (!a.window_mode && axis == 1 && a.kick != nullptr)
                            ? (a.kick_steps ? a.kick_steps[b] : a.kick_step)
                            : -1;
  const double kv = (kstep >= 0) ? a.kick[b] : 0.0;
  int f[C];  // working-set flags of the lane's slots: 0 free, +1 at z_max, −1 at z_min
#pragma unroll
  for (int q = 0; q < C; ++q) f[q] = 0;
  int fq = 0;
  unsigned passes = 0;   // the instance's passes (counters [1], [2])
  unsigned wpasses = 0;  // the wave's passes: per timestep the most of its instances
  unsigned itmax = 0;
  const unsigned long long imask = (L == 64) ? ~0ull : (((1ull << L) - 1) << base);

  // the window's (z_ref, half-width) of the lane's slots at timestep i (padding: the last
  // sample); the next timestep's are loaded while this one's passes run
  auto load_window = [&](int64_t i, double* hi, double* lo) {
#pragma unroll
    for (int q = 0; q < C; ++q) {
      const int k = min(k0 + q, N - 1);
      int64_t e;
      if (a.window_mode) {
        e = b * N + k;
      } else {
        int64_t t = i + a.toff + k;
        if (t > a.n - 1) t = a.n - 1;
        e = b * a.bstride + t * 2 + axis;
      }
      hi[q] = a.zmax[e];
      lo[q] = a.zmin[e];
    }
  };
  double nhi[C], nlo[C];
  load_window(0, nhi, nlo);
  for (int64_t i = 0; i < a.nsteps; ++i) {
    double r[C], h[C];
#pragma unroll
    for (int q = 0; q < C; ++q) {
      r[q] = (nhi[q] + nlo[q]) / 2;  // z_ref (zmp_controller.py:184)
      h[q] = (nhi[q] - nlo[q]) / 2;
    }
    if (i + 1 < a.nsteps) load_window(i + 1, nhi, nlo);
    // η of the state (strict_lq.hip)
    double e0[3];
    {
      const double xi1 = a.T * x[1], xi2 = a.Tsq * x[2];
      e0[0] = fma(-1.0 / 6.0, xi2, x[0]);
      e0[1] = fma(-0.5, xi2, xi1);
      e0[2] = xi2;
    }
    double v0 = 0.0;
    int it = 0;
    bool mine = valid;  // this instance still iterating
    bool again = __any(mine);
    while (again) {
      // ---- backward: chunk element, suffix scan, V at the chunk's end ------------------------
      Ric v;
      {
        Elem E;
        elem_identity(E);
#pragma unroll
        for (int q = C - 1; q >= 0; --q) {
          if (k0 + q < N) {
            const double sg = (double)f[q], ab = fabs(sg);
            const double fr = 1.0 - ab;
            const double t = fma(sg, h[q], r[q]);  // pinned target (r ± h)
            const double al = fr * a.piR + ab * a.ipi;
            const double b2s = fr * (a.piR * r[q]) + ab * (a.ipi * t);
            const double c22 = fr * a.iR;
            const double ka = fr * a.rhoR + ab * a.rhoP2;
            const double gc = fr * (a.rhoR * r[q]) + ab * (a.rhoP2 * t);
            prepend(a, al, b2s, c22, ka, gc, E);
          }
        }
        // suffix scan: inside each 16-lane row on DPP moves (the lane d ahead, d = 1, 2, 4, 8),
        // then across rows, each lane of an aligned block's first half taking the suffix of the
        // second half's first lane (one LDS-pipe shuffle level per doubling of 16)
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
          Elem P;
          row_shl_elem(E, P, d);
          if ((il & 15) + d < 16) combine(E, P);
        }
#pragma unroll
        for (int d = 16; d < L; d <<= 1) {
          Elem P;
          shfl_elem(E, P, base + (il & ~(2 * d - 1)) + d);
          if ((il & d) == 0) combine(E, P);
        }
        // V at the chunk's end = the right neighbour's suffix (0 past the horizon).  Every lane
        // takes part in the shuffles (a source lane outside the exec mask reads as 0); the last
        // lane's result is replaced afterwards.
        {
          double vv[9];
#pragma unroll
          for (int q = 0; q < 6; ++q) vv[q] = next_lane_f64(E.J[q]);
#pragma unroll
          for (int q = 0; q < 3; ++q) vv[6 + q] = next_lane_f64(E.g[q]);
          const bool last = il == L - 1;
          v.p00 = last ? 0.0 : vv[0];
          v.p01 = last ? 0.0 : vv[1];
          v.p02 = last ? 0.0 : vv[2];
          v.p11 = last ? 0.0 : vv[3];
          v.p12 = last ? 0.0 : vv[4];
          v.p22 = last ? 0.0 : vv[5];
          v.s0 = last ? 0.0 : vv[6];
          v.s1 = last ? 0.0 : vv[7];
          v.s2 = last ? 0.0 : vv[8];
        }
      }
      // ---- the lane's slots: Riccati back from V_end, keeping the laws (v ends as V at the
      // chunk's start)
      double K0[C], K1[C], K2[C], kf[C];
#pragma unroll
      for (int q = C - 1; q >= 0; --q) {
        if (k0 + q < N) ric_step(a, v, r[q], h[q], f[q], K0[q], K1[q], K2[q], kf[q]);
        else K0[q] = K1[q] = K2[q] = kf[q] = 0.0;
      }
      // ---- forward: chunk map η ↦ F η + φ, prefix scan, the state at the chunk's start -------
      double F[9], ph[3];
#pragma unroll
      for (int q = 0; q < 9; ++q) F[q] = (q % 4 == 0) ? 1.0 : 0.0;
      ph[0] = ph[1] = ph[2] = 0.0;
#pragma unroll
      for (int q = 0; q < C; ++q) {
        if (k0 + q < N) {
#pragma unroll
          // column c of F through η⁺: η0⁺ = η0 + η1 + η2, η1⁺ = η1 + η2, η2⁺ = (z − η0⁺)/π
          for (int c = 0; c < 3; ++c) {
            const double y0 = F[c], y1 = F[3 + c], y2 = F[6 + c];
            const double kv2 = fma(K0[q], y0, fma(K1[q], y1, K2[q] * y2));
            const double s12 = y1 + y2;
            const double e0 = y0 + s12;
            F[c] = e0;
            F[3 + c] = s12;
            F[6 + c] = -a.ipi * (kv2 + e0);
          }
          const double kv2 = fma(K0[q], ph[0], fma(K1[q], ph[1], K2[q] * ph[2])) + kf[q];
          const double s12 = ph[1] + ph[2];
          const double e0 = ph[0] + s12;
          ph[0] = e0;
          ph[1] = s12;
          ph[2] = -a.ipi * (kv2 + e0);
        }
      }
#pragma unroll
      for (int d = 1; d < L; d <<= 1) {
        double Fp[9], pp[3];
#pragma unroll
        for (int q = 0; q < 9; ++q) Fp[q] = prefix_src_f64(F[q], d);
#pragma unroll
        for (int q = 0; q < 3; ++q) pp[q] = prefix_src_f64(ph[q], d);
        if (d < 16 ? (il & 15) >= d : (il & d) != 0) {  // (F, φ) ← (F, φ) ∘ (Fp, pp): the
                                                        // earlier lanes' map first
          double Fn[9], pn[3];
#pragma unroll
          for (int i2 = 0; i2 < 3; ++i2) {
#pragma unroll
            for (int j = 0; j < 3; ++j)
              Fn[3 * i2 + j] = fma(F[3 * i2], Fp[j], fma(F[3 * i2 + 1], Fp[3 + j], F[3 * i2 + 2] * Fp[6 + j]));
            pn[i2] = fma(F[3 * i2], pp[0], fma(F[3 * i2 + 1], pp[1], fma(F[3 * i2 + 2], pp[2], ph[i2])));
          }
#pragma unroll
          for (int q = 0; q < 9; ++q) F[q] = Fn[q];
#pragma unroll
          for (int q = 0; q < 3; ++q) ph[q] = pn[q];
        }
      }
      double xs[3];
      {
        double xe[3];
#pragma unroll
        for (int i2 = 0; i2 < 3; ++i2)
          xe[i2] = fma(F[3 * i2], e0[0], fma(F[3 * i2 + 1], e0[1], fma(F[3 * i2 + 2], e0[2], ph[i2])));
#pragma unroll
        for (int i2 = 0; i2 < 3; ++i2) {
          const double up = prev_lane_f64(xe[i2]);
          xs[i2] = il == 0 ? e0[i2] : up;
        }
      }
      // ---- the lane's slots forward: roll out, primal check of the free slots --------------
      // costate at the chunk's end: λ = ∇V(η) = P η − s at the right neighbour's chunk start
      // (0 past the horizon: V_N = 0 there, and idle lanes carry it)
      double lam[3];
      {
        double ls[3];
        ls[0] = fma(v.p00, xs[0], fma(v.p01, xs[1], v.p02 * xs[2])) - v.s0;
        ls[1] = fma(v.p01, xs[0], fma(v.p11, xs[1], v.p12 * xs[2])) - v.s1;
        ls[2] = fma(v.p02, xs[0], fma(v.p12, xs[1], v.p22 * xs[2])) - v.s2;
#pragma unroll
        for (int i2 = 0; i2 < 3; ++i2) {
          const double dn = next_lane_f64(ls[i2]);
          lam[i2] = il == L - 1 ? 0.0 : dn;
        }
      }
      double wv[C];  // v (= T³u) at every slot (strict_lq.hip seg_forward)
      int np[C];     // a free slot's primal verdict
      const double tol = 1e-13;  // as strict_lq.hip
#pragma unroll
      for (int q = 0; q < C; ++q) {
        wv[q] = 0.0;
        np[q] = 0;
        if (k0 + q < N) {
          double vq, z;
          fwd_step(a, K0[q], K1[q], K2[q], kf[q], xs, vq, z);
          if (k0 + q == 0 && mine) v0 = vq;
          const double d = z - r[q], ht = h[q] + tol;
          wv[q] = vq;
          np[q] = (d > ht) ? 1 : ((d < -ht) ? -1 : 0);
        }
      }
      // ---- costate back through the chunk (strict_lq.hip seg_costate): the pinned slots'
      // multipliers, dual check, the new working set
      bool changed = false;
#pragma unroll
      for (int q = C - 1; q >= 0; --q) {
        if (k0 + q < N) {
          const int fl = f[q];
          const double sg = (double)fl;
          const double nu = pinned_nu(a, sg, h[q], wv[q], lam);  // ν / Q at pinned slots
          const bool rel = sg * nu < -a.tolnu;
          const int nf = (fl == 0) ? np[q] : (rel ? 0 : fl);
          changed |= nf != fl;
          if (mine) f[q] = nf;
          costate_step(a, wv[q], lam);
        }
      }
      // the instance's verdict (its L lanes of the wave's ballot)
      const bool ich = (__ballot(changed) & imask) != 0;
      if (mine) {
        ++it;
        if (!ich) {
          mine = false;
        } else if (it >= SC_MAXIT) {
          fq |= ZMPC_ST_MAXITER;
          mine = false;
        }
      }
      again = __any(mine);
    }
    passes += (unsigned)it;
    itmax = max(itmax, (unsigned)it);
    {
      int wit = it;  // (lanes of one instance hold the same count)
      for (int o = L; o < 64; o <<= 1) wit = max(wit, __shfl_xor(wit, o, 64));
      wpasses += (unsigned)wit;
    }
    // converged: advance in the reference form x⁺ = A x + B u0 (zmp_controller.py:199)
    const double u0 = __shfl(v0, base, 64) / a.Tcu;
    double xn[3];
    xn[0] = x[0] + a.T * x[1] + a.T2 * x[2] + a.T3 * u0;
    xn[1] = x[1] + a.T * x[2] + a.T2 * u0;
    xn[2] = x[2] + a.T * u0;
    if (i == kstep) xn[1] -= kv;  // force kick (zmp_controller.py:90,105-106)
    if (!(isfinite(xn[0]) && isfinite(xn[1]) && isfinite(xn[2]))) fq |= ZMPC_ST_NONFINITE;
    x[0] = xn[0];
    x[1] = xn[1];
    x[2] = xn[2];
    if (il == 0 && valid) {
      double* o = a.window_mode ? a.out + b * 3 : a.out + ((b * a.n + i + 1) * 2 + axis) * 3;
      o[0] = xn[0];
      o[1] = xn[1];
      o[2] = xn[2];
    }
    // warm start: the set shifted one slot towards the present, slot N−2 freed, N−1 kept
    {
      const int nxt = __builtin_amdgcn_update_dpp(0, f[0], 0x130, 0xF, 0xF, true);  // wave_shl:1
      int g[C];
#pragma unroll
      for (int q = 0; q < C; ++q) {
        const int k = k0 + q;
        const int sh = (q + 1 < C) ? f[q + 1] : nxt;
        g[q] = (k == N - 1) ? f[q] : ((k == N - 2) ? 0 : sh);
      }
#pragma unroll
      for (int q = 0; q < C; ++q) f[q] = (k0 + q < N) ? g[q] : 0;
    }
  }
  if (il == 0 && valid) {
    if (a.status != nullptr) {
      if (a.window_mode)
        a.status[b] = fq;
      else if (fq != 0)
        atomicOr(&a.status[b], fq);
    }
    if (a.cnt) {
      if (lane == 0) atomicAdd(a.cnt + 0, (unsigned long long)wpasses);  // once per wave
      atomicAdd(a.cnt + 1, (unsigned long long)passes);
      atomicAdd(a.cnt + 2, (unsigned long long)passes * (unsigned long long)N);
      atomicMax(a.cnt + 8, (unsigned long long)itmax);
    }
  }
}

// The kernel's constants from (T, the reference-form advance's T²/2 and T³/6, h/g, Q, R); also
// called by tests/emu's host build of this kernel.
void fill_consts(ScanArgs& a, double T, double T2_2, double T3_6, double hg, double Q, double R) {
  a.T = T;
  a.T2 = T2_2;
  a.T3 = T3_6;
  fill_eta(a, T, hg, Q, R);
  const double quu = a.pi * a.pi + a.rho;  // the slot elements' R (v-input form, header)
  a.iR = 1.0 / quu;
  a.piR = a.pi / quu;
  a.rhoR = a.rho / quu;
  a.rhoP2 = a.rho * a.ipi2;
}

void fill(const zmpc_plan* p, ScanArgs& a) {
  a.N = p->N;
  fill_consts(a, p->T, p->T2_2, p->T3_6, p->hg, p->Q, p->R);
  a.cnt = p->lqcnt;
}

// Lanes per instance: a whole wave while the instances fit one wave per SIMD (the latency of
// one pass is what counts), 32 beyond (two instances per wave; chunks of up to 16 slots,
// N ≤ 512; whole-wave instances beyond, to N = 960: N = 330–510 at 1024 walks 8.3e7–9.1e7 → 1.26e8–1.40e8 solves/s, profiles/r5aa/).  Chunks of C ≥ 3 slots per lane hold 1 wave per SIMD (their state spills past 256
// VGPRs into AGPRs instead of scratch: __launch_bounds__ above), shorter ones 2.  (C = 3 at 2
// waves per SIMD spilled 12 B to scratch; 1024 walks at N = 150, 32 lanes at one wave per
// SIMD: 10.2 → 6.2 ms, profiles/r5q/.)
int lanes_per_instance(const zmpc_plan* p, int64_t ninst) {
  const int64_t cus = p->cus > 0 ? p->cus : 256;
  // (one instance per SIMD: at N ≤ 128 the whole-wave instances would fit two waves per SIMD,
  // but two instances per wave already run 1.6–1.8× faster there, profiles/r5t/)
  return (ninst > cus * 4 && p->N <= kScan32MaxN) ? 32 : 64;
}

hipError_t launch(const zmpc_plan* p, const ScanArgs& a, hipStream_t s, int L) {
  const dim3 blk(64);
  int cmin = 1;
#ifdef ZMPC_DIAG
  if (const char* e = getenv("ZMPC_SCAN_CMIN")) cmin = atoi(e);  // (diagnostics: wider chunks)
#endif
  if (L == 32) {
    const dim3 grid((unsigned)((a.ninst + 1) / 2));
    switch (std::max((p->N + 31) / 32, std::min(cmin, 16))) {
#define ZMPC_SCASE(CC)                                                        \
  case CC:                                                                    \
    hipLaunchKernelGGL((zmpc_strict_scan_kernel<CC, 32>), grid, blk, 0, s, a); \
    break;
      ZMPC_SCASE(1) ZMPC_SCASE(2) ZMPC_SCASE(3) ZMPC_SCASE(4) ZMPC_SCASE(5) ZMPC_SCASE(6)
      ZMPC_SCASE(7) ZMPC_SCASE(8) ZMPC_SCASE(9) ZMPC_SCASE(10) ZMPC_SCASE(11) ZMPC_SCASE(12)
      ZMPC_SCASE(13) ZMPC_SCASE(14) ZMPC_SCASE(15) ZMPC_SCASE(16)
#undef ZMPC_SCASE
      default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  const dim3 grid((unsigned)a.ninst);
  switch ((p->N + 63) / 64) {
#define ZMPC_SCASE(CC)                                                        \
  case CC:                                                                    \
    hipLaunchKernelGGL((zmpc_strict_scan_kernel<CC, 64>), grid, blk, 0, s, a); \
    break;
    ZMPC_SCASE(1) ZMPC_SCASE(2) ZMPC_SCASE(3) ZMPC_SCASE(4) ZMPC_SCASE(5) ZMPC_SCASE(6)
    ZMPC_SCASE(7) ZMPC_SCASE(8) ZMPC_SCASE(9) ZMPC_SCASE(10) ZMPC_SCASE(11) ZMPC_SCASE(12)
    ZMPC_SCASE(13) ZMPC_SCASE(14) ZMPC_SCASE(15)
#undef ZMPC_SCASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

bool zmpc_strict_scan_supported(const zmpc_plan* p) { return p->N >= 1 && p->N <= kScanMaxN; }

hipError_t zmpc_launch_rollout_strict_scan(const zmpc_plan* p, int64_t B, int64_t n,
                                           const double* zmax, const double* zmin,
                                           int64_t bstride, const double* x0, const double* kick,
                                           int64_t kick_step, const int64_t* kick_steps,
                                           double* hist, int32_t* status, hipStream_t s,
                                           std::string* why) {
  if (!zmpc_strict_scan_supported(p)) {
    *why = "the small-batch strict kernel supports horizons N <= 960";
    return hipErrorInvalidValue;
  }
  if (status) {
    hipError_t e = hipMemsetAsync(status, 0, sizeof(int32_t) * B, s);
    if (e != hipSuccess) return e;
  }
  if (B == 0) return hipSuccess;
  ScanArgs a{};
  fill(p, a);
  a.window_mode = 0;
  a.toff = 1;
  a.n = n;
  a.nsteps = n - 1;
  a.ninst = 2 * B;
  a.zmax = zmax;
  a.zmin = zmin;
  a.bstride = bstride;
  a.x0 = x0;
  a.kick = kick;
  a.kick_step = kick_step;
  a.kick_steps = kick_steps;
  a.out = hist;
  a.status = status;
  return launch(p, a, s, lanes_per_instance(p, a.ninst));
}

hipError_t zmpc_launch_step_strict_scan(const zmpc_plan* p, int64_t B, const double* x,
                                        const double* zmax_win, const double* zmin_win,
                                        double* x_next, int32_t* status, hipStream_t s,
                                        std::string* why) {
  if (!zmpc_strict_scan_supported(p)) {
    *why = "the small-batch strict kernel supports horizons N <= 960";
    return hipErrorInvalidValue;
  }
  if (B == 0) return hipSuccess;
  ScanArgs a{};
  fill(p, a);
  a.window_mode = 1;
  a.toff = 0;
  a.n = 0;
  a.nsteps = 1;
  a.ninst = B;
  a.zmax = zmax_win;
  a.zmin = zmin_win;
  a.bstride = 0;
  a.x0 = x;
  a.out = x_next;
  a.status = status;
  a.kick_step = -1;
  return launch(p, a, s, lanes_per_instance(p, a.ninst));
}
