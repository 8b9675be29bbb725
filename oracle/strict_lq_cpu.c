// CPU restatement of the strict (ZMP box-constrained) Wieber rollout in LQ form — TEST
// INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load it (oracle/strict_cpu.py, ctypes): as the checker of the device kernel's algorithm and as
// the optimized multi-core strict CPU baseline.  The product never links it.
//
// Reference: zmp_controller.py:173-195 (per axis and timestep, cvxpy -> OSQP there)
//   min_J ½Q‖Px x + Pu J − z_ref‖² + ½R‖J‖²  s.t.  z_min ≤ Px x + Pu J ≤ z_max,  u0 = J[0],
// z_ref = (z_max + z_min)/2 (:184), the rollout of :59-108 (window rows past n − 1 repeat the last
// sample, :81-88; the y-velocity kick at i == kick_step, :90,105-106), x⁺ = A x + B u0 (:199).
// Pu[k,j] = C A^(k−j) B and Px[k] = C A^(k+1) (:162-171): the predicted ZMP is the LIPM output,
// so the QP is an LQ tracking problem with one output bound per horizon slot, solved per working
// set by a backward Riccati recursion, a forward rollout (primal check of the free slots) and a
// costate sweep (bound multipliers of the pinned slots), the working set from the primal-dual
// active-set iteration (warm start: the previous timestep's converged set shifted one slot, the
// shifted terminal slot N−2 free, slot N−1 kept).
//
// Coordinates (the device kernel's): ξ = [x0, T x1, T² x2], v = T³ u, objective / Q, then
// η = [ξ0 − ξ2/6, ξ1 − ξ2/2, ξ2], in which the jerk integrator is
//   η⁺ = Ā η + e2 v,   Ā = [[1,1,1],[0,1,1],[0,0,1]],   z = c̄ᵀη + π v,  c̄ = [1, 1, γ'],
// γ' = 7/6 − (h/g)/T², π = 1/6 − (h/g)/T² (= p(0)/T³), stage cost ½(z − r)² + ½ρv², ρ = R/(Q T⁶).
// B̄ = e2 makes B̄ᵀPB̄ = P22, PB̄ = P[:,2] and B̄ᵀs = s2 free, and ĀᵀPĀ is the 2-D prefix sum of P.
// Value function V(η) = ½ηᵀPη − sᵀη.
//
// Build: gcc -O2 -fopenmp -ffp-contract=off -shared -fPIC (oracle/Makefile).
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define LQ_MAXIT 1024  // (as strict_lq.hip)
#define ST_MAXITER 1
#define ST_NONFINITE 2

typedef struct {
  int N;
  double T, T2_2, T3_6;  // reference-form state advance (zmp_controller.py:18-20,199)
  double Tsq, Tcu;       // T², T³
  double pi, ipi, ipi2;  // π, a = 1/π, a²
  double gp;             // γ'
  double rho, eps;       // ρ, ε = ρ/π²
  double epsg, epsg2;    // εγ', εγ'²
  double quz0;           // 1 + ε
  double epi;            // επ = ρ/π
  double tolnu;          // multiplier tolerance (metres of ZMP in the objective / Q)
} Consts;

typedef struct {
  double p00, p01, p02, p11, p12, p22, s0, s1, s2;
} Ric;

static void consts_init(Consts* c, int N, double T, double T2_2, double T3_6, double hg,
                        double Q, double R) {
  c->N = N;
  c->T = T;
  c->T2_2 = T2_2;
  c->T3_6 = T3_6;
  c->Tsq = T * T;
  c->Tcu = c->Tsq * T;
  const double hgt = hg / c->Tsq;
  c->pi = 1.0 / 6.0 - hgt;
  c->ipi = 1.0 / c->pi;
  c->ipi2 = c->ipi * c->ipi;
  c->gp = 7.0 / 6.0 - hgt;
  c->rho = R / (Q * c->Tcu * c->Tcu);
  c->eps = c->rho * c->ipi2;
  c->epsg = c->eps * c->gp;
  c->epsg2 = c->epsg * c->gp;
  c->quz0 = 1.0 + c->eps;
  c->epi = c->rho * c->ipi;
  c->tolnu = 1e-13;
}

// One backward Riccati step at a slot with flag f (0 free, 1 at z_max, 2 at z_min): V_{k+1} in v
// -> V_k; the step's law z = −K η − kf, the slot's ZMP z as the input (z-control form: η⁺ = F η +
// a e2 z, F = Ā − a e2 c̄ᵀ, stage ½(z − r)² + ½ε(z − c̄ᵀη)²; pinned: K = 0, kf = −t).
static void ric_step(const Consts* c, Ric* v, double hi, double lo, int f, double K[3],
                     double* kf) {
  const double r = (hi + lo) / 2;  // z_ref (zmp_controller.py:184)
  const double q1 = v->p02 + v->p12;
  const double n01 = v->p00 + v->p01;
  const double n11 = n01 + (v->p01 + v->p11);
  const double w0 = c->ipi * v->p02, w1 = c->ipi * q1;
  const double cc = c->ipi2 * v->p22;
  const double ce = cc + c->eps, cg = cc + c->epsg;
  const double u0 = w0 - ce, u1 = w1 - ce, u2 = w1 - cg;  // Qux
  const double wz = fma(c->ipi, v->s2, r);                // −qu
  if (f == 0) {
    const double iq = 1.0 / (c->quz0 + cc);
    K[0] = u0 * iq;
    K[1] = u1 * iq;
    K[2] = u2 * iq;
    *kf = -wz * iq;
  } else {
    K[0] = K[1] = K[2] = 0.0;
    *kf = -((f == 1) ? hi : lo);
  }
  const double t00 = fma(-2.0, w0, v->p00);
  const double t01 = (n01 - w0) - w1;
  const double t11 = fma(-2.0, w1, n11);
  // P = Qxx − Qux Kᵀ,  s = Fᵀs + Qux kf
  v->p00 = fma(-u0, K[0], t00 + ce);
  v->p01 = fma(-u0, K[1], t01 + ce);
  v->p02 = fma(-u0, K[2], t01 + cg);
  v->p11 = fma(-u1, K[1], t11 + ce);
  v->p12 = fma(-u1, K[2], t11 + cg);
  v->p22 = fma(-u2, K[2], t11 + (cc + c->epsg2));
  const double as2 = c->ipi * v->s2;
  const double f0 = v->s0 - as2, f1 = (v->s0 + v->s1) - as2;
  v->s0 = fma(u0, *kf, f0);
  v->s1 = fma(u1, *kf, f1);
  v->s2 = fma(u2, *kf, f1);
}

typedef struct {
  double *K, *kf, *w, *hi, *lo;
  unsigned char *f, *nf;
} Work;

// One (walk, axis) instance over the whole rollout.  b: walk bounds [n][2] (stride 2 per row),
// axis column a.  x: initial state (3), hist out (row stride 6).  Returns status bits, adds the
// active-set passes to *passes.
static int instance(const Consts* c, int64_t n, const double* zmax, const double* zmin, int a,
                    const double* x0, double kick, int64_t kick_step, double* hist, Work* wk,
                    uint64_t* passes) {
  const int N = c->N;
  int st = 0;
  double x[3] = {x0[0], x0[1], x0[2]};
  hist[0] = x[0];
  hist[1] = x[1];
  hist[2] = x[2];
  memset(wk->f, 0, (size_t)N);
  const double tol = 1e-13;
  for (int64_t i = 0; i + 1 < n; ++i) {
    for (int k = 0; k < N; ++k) {
      int64_t t = i + 1 + k;
      if (t > n - 1) t = n - 1;  // window padding (zmp_controller.py:81-88)
      wk->hi[k] = zmax[t * 2 + a];
      wk->lo[k] = zmin[t * 2 + a];
    }
    double v0 = 0.0;
    for (int it = 1;; ++it) {
      ++*passes;
      Ric v = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      for (int k = N - 1; k >= 0; --k)
        ric_step(c, &v, wk->hi[k], wk->lo[k], wk->f[k], wk->K + 3 * k, wk->kf + k);
      double e[3] = {x[0], c->T * x[1], c->Tsq * x[2]};  // ξ
      e[0] = fma(-1.0 / 6.0, e[2], e[0]);                 // η
      e[1] = fma(-0.5, e[2], e[1]);
      for (int k = 0; k < N; ++k) {
        const double* K = wk->K + 3 * k;
        // z = −Kη − kf; η⁺ = Āη + e2 v, v = (z − c̄ᵀη)/π, and c̄ᵀη = η0⁺ + π η2 (γ' − 1 = π)
        const double z = -fma(K[0], e[0], fma(K[1], e[1], K[2] * e[2])) - wk->kf[k];
        const double s12 = e[1] + e[2];
        const double e0 = e[0] + s12;
        const double e2n = c->ipi * (z - e0);
        const double u = e2n - e[2];
        if (k == 0) v0 = u;
        e[0] = e0;
        e[1] = s12;
        e[2] = e2n;
        wk->w[k] = u;
        wk->nf[k] = (z > wk->hi[k] + tol) ? 1 : ((z < wk->lo[k] - tol) ? 2 : 0);
      }
      // costate from λ_N = ∇V_N = 0: λ_k = Fᵀλ_{k+1} − επ v_k c̄; a pinned slot's multiplier
      // from stationarity in z_k: ν = −((z − r) + επ v + λ2_{k+1}/π), z − r = ±half-width
      double l0 = 0, l1 = 0, l2 = 0;
      int changed = 0;
      for (int k = N - 1; k >= 0; --k) {
        const int f = wk->f[k];
        const double hi = wk->hi[k], lo = wk->lo[k];
        const double ev = c->epi * wk->w[k];
        int nf;
        if (f == 0) {
          nf = wk->nf[k];
        } else {
          const double zr = (f == 1) ? (hi - lo) / 2 : -((hi - lo) / 2);
          const double nu = -(zr + fma(c->ipi, l2, ev));
          const int rel = (f == 1 && nu < -c->tolnu) || (f == 2 && nu > c->tolnu);
          nf = rel ? 0 : f;
        }
        changed |= nf != f;
        wk->nf[k] = (unsigned char)nf;
        const double al2 = c->ipi * l2;
        const double m0 = l0 - al2, m1 = (l0 + l1) - al2;
        l0 = m0 - ev;
        l1 = m1 - ev;
        l2 = fma(-c->gp, ev, m1);
      }
      memcpy(wk->f, wk->nf, (size_t)N);
      if (changed && it >= LQ_MAXIT) {
        st |= ST_MAXITER;
        changed = 0;
      }
      if (!changed) break;
    }
    // converged: x⁺ = A x + B u0 in the reference form (zmp_controller.py:199)
    const double u0 = v0 / c->Tcu;
    double xn[3];
    xn[0] = x[0] + c->T * x[1] + c->T2_2 * x[2] + c->T3_6 * u0;
    xn[1] = x[1] + c->T * x[2] + c->T2_2 * u0;
    xn[2] = x[2] + c->T * u0;
    if (i == kick_step) xn[1] -= kick;  // force kick (zmp_controller.py:90,105-106)
    if (!(isfinite(xn[0]) && isfinite(xn[1]) && isfinite(xn[2]))) st |= ST_NONFINITE;
    x[0] = xn[0];
    x[1] = xn[1];
    x[2] = xn[2];
    double* h = hist + (i + 1) * 6;
    h[0] = x[0];
    h[1] = x[1];
    h[2] = x[2];
    // warm start: shifted one slot towards the present, slot N−1 kept, slot N−2 free
    memmove(wk->f, wk->f + 1, (size_t)(N - 1));
    if (N >= 2) wk->f[N - 2] = 0;
  }
  return st;
}

// Batched strict rollout: zmax/zmin [B][n][2] (bstride = 2n) or one shared [n][2] (bstride 0),
// x0 [B][2][3], kick [B] (NULL: none) subtracted from the y velocity at i == kick_step,
// hist [B][n][2][3], status [B], passes [B] (may be NULL).  threads <= 0: OpenMP default.
int zmpc_cpu_strict_rollout(int64_t B, int64_t n, int N, double T, double T2_2, double T3_6,
                            double hg, double Q, double R, const double* zmax,
                            const double* zmin, int64_t bstride, const double* x0,
                            const double* kick, int64_t kick_step, double* hist,
                            int32_t* status, uint64_t* passes, int threads) {
  if (B < 0 || n < 1 || N < 1 || !zmax || !zmin || !x0 || !hist) return -1;
  Consts c;
  consts_init(&c, N, T, T2_2, T3_6, hg, Q, R);
  if (status) memset(status, 0, sizeof(int32_t) * (size_t)B);
  if (passes) memset(passes, 0, sizeof(uint64_t) * (size_t)B);
  int bad = 0;
#pragma omp parallel num_threads(threads > 0 ? threads : omp_get_max_threads())
  {
    Work wk;
    double* dbuf = (double*)malloc(sizeof(double) * 7 * (size_t)N);
    unsigned char* fbuf = (unsigned char*)malloc(2 * (size_t)N);
    if (!dbuf || !fbuf) {
#pragma omp atomic write
      bad = 1;
    } else {
      wk.K = dbuf;
      wk.kf = dbuf + 3 * N;
      wk.w = dbuf + 4 * N;
      wk.hi = dbuf + 5 * N;
      wk.lo = dbuf + 6 * N;
      wk.f = fbuf;
      wk.nf = fbuf + N;
#pragma omp for schedule(dynamic, 1)
      for (int64_t q = 0; q < 2 * B; ++q) {
        const int64_t b = q >> 1;
        const int a = (int)(q & 1);
        uint64_t np = 0;
        double tmp[3];
        const double* xb = x0 + (b * 2 + a) * 3;
        tmp[0] = xb[0];
        tmp[1] = xb[1];
        tmp[2] = xb[2];
        // the instance writes its column of the history through a strided view
        double* h = hist + (b * n * 2 + a) * 3;
        double kv = (a == 1 && kick) ? kick[b] : 0.0;
        int64_t ks = (a == 1 && kick) ? kick_step : -1;
        // history rows of one axis are 6 doubles apart: instance() writes (i·6 + 0..2)
        const int s = instance(&c, n, zmax + b * bstride, zmin + b * bstride, a, tmp, kv, ks, h,
                               &wk, &np);
        if (status) {
#pragma omp atomic
          status[b] |= s;
        }
        if (passes) {
#pragma omp atomic
          passes[b] += np;
        }
      }
    }
    free(dbuf);
    free(fbuf);
  }
  return bad ? -3 : 0;
}
