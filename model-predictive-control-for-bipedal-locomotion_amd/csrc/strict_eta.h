// The strict QP's LQ step in η coordinates, shared by the lane-per-instance kernel
// (strict_lq.hip) and the parallel-in-time small-batch kernel (strict_scan.hip).  Coordinates and
// the step's algebra: strict_lq.hip's header.  Args carries pi, ipi, gipi, pig, gp, gp2 and
// quu0 (= π² + ρ) as doubles.
#pragma once

#include <hip/hip_runtime.h>

// every fused multiply-add is an explicit fma() (also for the including file from here on)
#pragma clang fp contract(off)

namespace zmpc_eta {

struct Ric {  // value function V(η) = ½ηᵀPη − sᵀη
  double p00, p01, p02, p11, p12, p22, s0, s1, s2;
};

// 1/Quu: hardware reciprocal + two Newton steps (Quu ≥ ρ + π² > 0, no special cases)
__device__ __forceinline__ double recip(double q) {
  double iq = __builtin_amdgcn_rcp(q);
  iq = fma(iq, fma(-q, iq, 1.0), iq);
  return fma(iq, fma(-q, iq, 1.0), iq);
}

// The parts of a Riccati step every form shares: ĀᵀPĀ (m..), Qux, Quu, −qu (w), −qx (nqx).
struct StepCore {
  double m01, m02, m11, m12, m22;  // ĀᵀPĀ except M00 = p00
  double ux0, ux1, ux2, Quu, w, nqx0, nqx1, nqx2;
};

template <class Args>
__device__ __forceinline__ StepCore step_core(const Args& a, const Ric& v, double r) {
  StepCore c;
  const double q1 = v.p02 + v.p12, q2 = q1 + v.p22;  // prefix of P's last column
  c.m01 = v.p00 + v.p01;
  c.m11 = c.m01 + (v.p01 + v.p11);
  c.m02 = c.m01 + v.p02;
  c.m12 = c.m11 + q1;
  c.m22 = c.m12 + q2;
  c.ux0 = a.pi + v.p02;
  c.ux1 = a.pi + q1;
  c.ux2 = a.pig + q2;
  c.Quu = a.quu0 + v.p22;
  c.w = fma(a.pi, r, v.s2);
  const double t1 = v.s0 + v.s1, t2 = t1 + v.s2;
  c.nqx0 = r + v.s0;
  c.nqx1 = r + t1;
  c.nqx2 = fma(a.gp, r, t2);
  return c;
}

// One backward Riccati step, per-lane signed slot flag f (0 free, +1 at z_max, −1 at z_min):
// V_{k+1} in v → V_k; outputs the step's law.  Branch-free with σ = f as a double and |σ|: the
// free part (iqa) and the pinned part (ka, kfa, zero at free slots) of the law,
// K = Qux·iqa + ka and kff = qu·iqa + kfa — exactly Qux/Quu, qu/Quu at a free slot and c̄/π,
// −t/π at a pinned one (t = r + σh).  D = Quu K − Qux is formed unconditionally and enters only
// through ka and kfa, which vanish at free slots.
template <class Args>
__device__ __forceinline__ void ric_step(const Args& a, Ric& v, double r, double h, int f,
                                         double& K0, double& K1, double& K2, double& kf) {
  const StepCore c = step_core(a, v, r);
  const double iq = recip(c.Quu);
  const double sg = (double)f, ab = fabs(sg);
  const double iqa = fma(-ab, iq, iq);  // iq at free slots, exactly 0 at pinned ones
  const double ka01 = ab * a.ipi;
  const double ka2 = ab * a.gipi;
  const double kfa = -fma(sg, h, ab * r) * a.ipi;  // −t/π at pinned slots, 0 at free ones
  K0 = fma(c.ux0, iqa, ka01);
  K1 = fma(c.ux1, iqa, ka01);
  K2 = fma(c.ux2, iqa, ka2);
  kf = fma(-c.w, iqa, kfa);
  const double D0 = fma(c.Quu, K0, -c.ux0);
  const double D1 = fma(c.Quu, K1, -c.ux1);
  const double D2 = fma(c.Quu, K2, -c.ux2);
  const double P00 = fma(ka01, D0, fma(-c.ux0, K0, 1.0 + v.p00));
  const double P01 = fma(ka01, D1, fma(-c.ux0, K1, 1.0 + c.m01));
  const double P02 = fma(ka01, D2, fma(-c.ux0, K2, a.gp + c.m02));
  const double P11 = fma(ka01, D1, fma(-c.ux1, K1, 1.0 + c.m11));
  const double P12 = fma(ka01, D2, fma(-c.ux1, K2, a.gp + c.m12));
  const double P22 = fma(ka2, D2, fma(-c.ux2, K2, a.gp2 + c.m22));
  v.s0 = fma(-kfa, D0, fma(-K0, c.w, c.nqx0));
  v.s1 = fma(-kfa, D1, fma(-K1, c.w, c.nqx1));
  v.s2 = fma(-kfa, D2, fma(-K2, c.w, c.nqx2));
  v.p00 = P00;
  v.p01 = P01;
  v.p02 = P02;
  v.p11 = P11;
  v.p12 = P12;
  v.p22 = P22;
}

// One forward step of the closed loop v = −K η − kff: η advances, returns v and z.
template <class Args>
__device__ __forceinline__ void fwd_step(const Args& a, double K0, double K1, double K2,
                                         double kf, double* x, double& v, double& z) {
  v = -fma(K0, x[0], fma(K1, x[1], K2 * x[2])) - kf;
  z = fma(a.pi, v, fma(a.gp, x[2], x[0] + x[1]));
  const double s12 = x[1] + x[2];
  x[0] = x[0] + s12;
  x[1] = s12;
  x[2] = x[2] + v;
}

}  // namespace zmpc_eta
