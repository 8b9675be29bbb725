// The strict QP's LQ step in η coordinates, shared by the lane-per-instance kernel
// (strict_lq.hip) and the parallel-in-time small-batch kernel (strict_scan.hip).  Coordinates:
// strict_lq.hip's header; the step's algebra (z-control form): below.
#pragma once

#include <hip/hip_runtime.h>

// every fused multiply-add is an explicit fma() (also for the including file from here on)
#pragma clang fp contract(off)

namespace zmpc_eta {

struct Ric {  // value function V(η) = ½ηᵀPη − sᵀη
  double p00, p01, p02, p11, p12, p22, s0, s1, s2;
};

// 1/Quu: hardware reciprocal + two Newton steps (Quu ≥ 1 > 0, no special cases)
__device__ __forceinline__ double recip(double q) {
  double iq = __builtin_amdgcn_rcp(q);
  iq = fma(iq, fma(-q, iq, 1.0), iq);
  return fma(iq, fma(-q, iq, 1.0), iq);
}

// The Riccati step takes the slot's ZMP z as its input (z-control form): with a = 1/π,
// v = a(z − c̄ᵀη) and F = Ā − a e2 c̄ᵀ (= rows [1,1,1], [0,1,1], −a[1,1,1]):
//   η⁺ = F η + a e2 z,   stage ½(z − r)² + ½ε(z − c̄ᵀη)²,   ε = ρ/π²,
//   Qux = a FᵀP e2 − ε c̄,  Quu = 1 + ε + a² P22,  qu = −(r + a s2),  Qxx = ε c̄c̄ᵀ + FᵀPF,
//   P ← Qxx − Qux Kᵀ,  s ← Fᵀs + Qux kff;  free: K = Qux/Quu, kff = qu/Quu; pinned at t: K = 0,
//   kff = −t (z = t exactly).
// The v-control form (v the input, P ← c̄c̄ᵀ + ĀᵀPĀ − Qux Kᵀ) subtracts two terms of size γ'² ≈
// (h/g)²/T⁴ that cancel to P's size when the jerk is cheap (ρ ≪ π²): at R/Q = 1e-9, N = 64 it
// lost three digits (the input 7e-12 relative, 2.3e-9 m CoM RMSE over the default walk); this
// form has no such cancellation at any weight (≤ 4e-15 relative, ρ/π² from 1e-6 to 4e4;
// tests/golden/strict_weights_ref.npz).  Args carries ipi (a), ipi2 (a²), eps, epsg (εγ'), epsg2
// (εγ'²), quz0 (1 + ε), epi (επ = ρ/π) and gp (γ').
struct ZCore {
  double u0, u1, u2;  // Qux
  double Quu;
  double t00, t01, t11;  // FᵀPF without the a²P22 term: Qxx = t + c + ε c̄c̄ᵀ
  double c, ce, cg;      // a²P22, c + ε, c + εγ'
  double wz;             // −qu
};

template <class Args>
__device__ __forceinline__ ZCore zcore(const Args& a, const Ric& v, double r) {
  ZCore c;
  const double q1 = v.p02 + v.p12;
  const double n01 = v.p00 + v.p01;
  const double n11 = n01 + (v.p01 + v.p11);
  const double w0 = a.ipi * v.p02, w1 = a.ipi * q1;  // a Ā'ᵀP e2
  c.c = a.ipi2 * v.p22;
  c.ce = c.c + a.eps;
  c.cg = c.c + a.epsg;
  c.u0 = w0 - c.ce;
  c.u1 = w1 - c.ce;
  c.u2 = w1 - c.cg;
  c.Quu = a.quz0 + c.c;
  c.t00 = fma(-2.0, w0, v.p00);
  c.t01 = (n01 - w0) - w1;
  c.t11 = fma(-2.0, w1, n11);
  c.wz = fma(a.ipi, v.s2, r);
  return c;
}

// V_k from V_{k+1} and the law (K, kff): P ← Qxx − Qux Kᵀ, s ← Fᵀs + Qux kff.
template <class Args>
__device__ __forceinline__ void zupdate(const Args& a, Ric& v, const ZCore& c, double K0,
                                        double K1, double K2, double kf) {
  v.p00 = fma(-c.u0, K0, c.t00 + c.ce);
  v.p01 = fma(-c.u0, K1, c.t01 + c.ce);
  v.p02 = fma(-c.u0, K2, c.t01 + c.cg);
  v.p11 = fma(-c.u1, K1, c.t11 + c.ce);
  v.p12 = fma(-c.u1, K2, c.t11 + c.cg);
  v.p22 = fma(-c.u2, K2, c.t11 + (c.c + a.epsg2));
  const double as2 = a.ipi * v.s2;
  const double f0 = v.s0 - as2, f1 = (v.s0 + v.s1) - as2;  // Fᵀs
  v.s0 = fma(c.u0, kf, f0);
  v.s1 = fma(c.u1, kf, f1);
  v.s2 = fma(c.u2, kf, f1);
}

// One backward Riccati step, per-lane signed slot flag f (0 free, +1 at z_max, −1 at z_min):
// V_{k+1} in v → V_k; outputs the step's law z = −K η − kff.  Branch-free with σ = f as a double:
// iqa = 1/Quu at free slots and exactly 0 at pinned ones, so K = Qux·iqa and kff = −wz·iqa − t.
template <class Args>
__device__ __forceinline__ void ric_step(const Args& a, Ric& v, double r, double h, int f,
                                         double& K0, double& K1, double& K2, double& kf) {
  const ZCore c = zcore(a, v, r);
  const double iq = recip(c.Quu);
  const double sg = (double)f, ab = fabs(sg);
  const double iqa = fma(-ab, iq, iq);
  K0 = c.u0 * iqa;
  K1 = c.u1 * iqa;
  K2 = c.u2 * iqa;
  kf = fma(-c.wz, iqa, -fma(sg, h, ab * r));  // −wz/Quu free, −t = −(r + σh) pinned
  zupdate(a, v, c, K0, K1, K2, kf);
}

// The same step at a free slot; also returns 1/Quu and Qux (the free-tail table).
template <class Args>
__device__ __forceinline__ void ric_free(const Args& a, Ric& v, double r, double& K0, double& K1,
                                         double& K2, double& kf, double& iqo, double& u0,
                                         double& u1, double& u2) {
  const ZCore c = zcore(a, v, r);
  const double iq = recip(c.Quu);
  K0 = c.u0 * iq;
  K1 = c.u1 * iq;
  K2 = c.u2 * iq;
  kf = -c.wz * iq;
  iqo = iq;
  u0 = c.u0;
  u1 = c.u1;
  u2 = c.u2;
  zupdate(a, v, c, K0, K1, K2, kf);
}

// One forward step of the closed loop z = −K η − kff: η advances; returns v (= T³u) and z.
// η⁺ = Āη + e2 v with v = a(z − c̄ᵀη), and c̄ᵀη = η0⁺ + π η2 (γ' − 1 = π): η2⁺ = a(z − η0⁺).
template <class Args>
__device__ __forceinline__ void fwd_step(const Args& a, double K0, double K1, double K2,
                                         double kf, double* x, double& v, double& z) {
  z = -fma(K0, x[0], fma(K1, x[1], K2 * x[2])) - kf;
  const double s12 = x[1] + x[2];
  const double e0 = x[0] + s12;
  const double e2 = a.ipi * (z - e0);
  v = e2 - x[2];
  x[0] = e0;
  x[1] = s12;
  x[2] = e2;
}

// A pinned slot's bound multiplier from stationarity in z_k (objective / Q, in metres):
// ν = −((z − r) + επ v + λ2_{k+1}/π), z − r = σh at the pinned slot; valid when σν ≥ 0.
template <class Args>
__device__ __forceinline__ double pinned_nu(const Args& a, double sg, double h, double v,
                                            const double* lam) {
  return -fma(sg, h, fma(a.ipi, lam[2], a.epi * v));
}

// The costate one slot back: λ_k = Fᵀλ_{k+1} − επ v_k c̄.
template <class Args>
__device__ __forceinline__ void costate_step(const Args& a, double v, double* lam) {
  const double ev = a.epi * v;
  const double al2 = a.ipi * lam[2];
  const double m0 = lam[0] - al2, m1 = (lam[0] + lam[1]) - al2;
  lam[0] = m0 - ev;
  lam[1] = m1 - ev;
  lam[2] = fma(-a.gp, ev, m1);
}

// The z-form constants from the plan's (T, h/g, Q, R) (host side, every strict kernel).
template <class Args>
inline void fill_eta(Args& a, double T, double hg, double Q, double R) {
  a.Tsq = T * T;
  a.Tcu = a.Tsq * T;
  const double hgt = hg / a.Tsq;
  a.pi = 1.0 / 6.0 - hgt;  // p(0)/T³ (zmp_controller.py:171, i = j)
  a.ipi = 1.0 / a.pi;
  a.ipi2 = a.ipi * a.ipi;
  a.gp = 7.0 / 6.0 - hgt;
  a.rho = R / (Q * a.Tcu * a.Tcu);
  a.eps = a.rho * a.ipi2;
  a.epsg = a.eps * a.gp;
  a.epsg2 = a.epsg * a.gp;
  a.quz0 = 1.0 + a.eps;
  a.epi = a.rho * a.ipi;
  // multiplier tolerance: the scaled objective's ν is in metres of ZMP, as the primal check's
  // 1e-13 — the same for every Q (it was 1e-13/Q before round 5)
  a.tolnu = 1e-13;
}

}  // namespace zmpc_eta
