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
// Mapping: one 64-lane wavefront per walk (both axes).  Per wave:
//   1. stage z_ref = (z_max + z_min)/2 (:197) for both axes in LDS, padded with the last row
//      (:81-88), from coalesced loads of the walk's contiguous [n,2] bound rows;
//   2. correlation with an 8-wide register sliding window; k streams from scalar loads
//      (wave-uniform index) so each j costs one LDS read per axis for 8 FMAs;
//   3. chunked affine scan over the 64 lanes with P = Ā^C (Ā = A - B kxᵀ), Kogge-Stone;
//   4. each lane replays its chunk in the reference form x⁺ = A x + B u, applies the
//      F_ext kick (:105-106) and stores the states.
#include <cstdlib>

#include "zmpc_internal.h"

namespace {

constexpr int kCW = 8;  // outputs per lane in the correlation register tile

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

}  // namespace

size_t zmpc_rollout_unc_lds_bytes(int Kpad, int64_t n) {
  const int64_t nsteps = n - 1;
  const int64_t passes = (nsteps + 64 * kCW - 1) / (64 * kCW);
  const int64_t Lz = passes * 64 * kCW + Kpad + 1;
  const int64_t nf = ((nsteps + 1) + 1) & ~1LL;
  return (size_t)(2 * Lz + 2 * nf) * sizeof(double);
}

__global__ void __launch_bounds__(64) zmpc_rollout_unc_kernel(
    int Kpad, int n, LipmConsts lc, const double* __restrict__ k, const double* __restrict__ kxp,
    const double* __restrict__ zmax, const double* __restrict__ zmin, int64_t bstride,
    const double* __restrict__ x0, const double* __restrict__ kick, int64_t kick_step,
    double* __restrict__ hist, int32_t* __restrict__ status, int dbg) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const int nsteps = n - 1;
  const int passes = (nsteps + 64 * kCW - 1) / (64 * kCW);
  const int Lz = passes * 64 * kCW + Kpad + 1;
  const int nf = (nsteps + 2) & ~1;
  double* zr0 = smem;
  double* zr1 = smem + Lz;
  double* f0 = smem + 2 * Lz;
  double* f1 = f0 + nf;

  // ---- 1. z_ref for both axes, padded with the last row -------------------------------
  const double* zmx = zmax + b * bstride;
  const double* zmn = zmin + b * bstride;
  for (int e = lane; e < ((dbg & 8) ? 0 : 2 * n); e += 64) {
    const double zr = (zmx[e] + zmn[e]) / 2;  // z_ref = (z_max + z_min) / 2
    if (e & 1)
      zr1[e >> 1] = zr;
    else
      zr0[e >> 1] = zr;
  }
  {
    const double last0 = (zmx[2 * n - 2] + zmn[2 * n - 2]) / 2;
    const double last1 = (zmx[2 * n - 1] + zmn[2 * n - 1]) / 2;
    for (int t = n + lane; t < Lz; t += 64) {
      zr0[t] = last0;
      zr1[t] = last1;
    }
  }
  __syncthreads();

  // ---- 2. f_i = Σ_j k_j z_ref[i+1+j], 8 outputs per lane, sliding register window -----
  for (int pass = 0; pass < ((dbg & 1) ? 0 : passes); ++pass) {
    const int i0 = pass * 64 * kCW + lane * kCW;
    double a0[kCW], a1[kCW], w0[kCW], w1[kCW];
#pragma unroll
    for (int m = 0; m < kCW; ++m) {
      a0[m] = 0.0;
      a1[m] = 0.0;
      w0[m] = zr0[i0 + 1 + m];
      w1[m] = zr1[i0 + 1 + m];
    }
    for (int j = 0; j < Kpad; j += kCW) {
#pragma unroll
      for (int jj = 0; jj < kCW; ++jj) {
        const double kj = k[j + jj];
#pragma unroll
        for (int m = 0; m < kCW; ++m) {
          a0[m] = fma(kj, w0[(jj + m) % kCW], a0[m]);
          a1[m] = fma(kj, w1[(jj + m) % kCW], a1[m]);
        }
        w0[jj] = zr0[i0 + 1 + j + jj + kCW];
        w1[jj] = zr1[i0 + 1 + j + jj + kCW];
      }
    }
#pragma unroll
    for (int m = 0; m < kCW; ++m) {
      if (i0 + m < nsteps) {
        f0[i0 + m] = a0[m];
        f1[i0 + m] = a1[m];
      }
    }
  }
  __syncthreads();

  // ---- 3. affine scan of x_{i+1} = Ā x_i + B f_i (+ kick) over 64 lane chunks ----------
  const double kx0 = kxp[0], kx1 = kxp[1], kx2 = kxp[2];
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
  const int C = (nsteps + 63) / 64;  // steps per lane chunk
  const int mbeg = lane * C;
  const int mend = min(mbeg + C, nsteps);
  const double kk = (kick != nullptr) ? kick[b] : 0.0;

  double s0[3] = {0.0, 0.0, 0.0}, s1[3] = {0.0, 0.0, 0.0};
  for (int m = mbeg; m < mend; ++m) {
    double t[3];
    matvec3(Ab, s0, t);
    s0[0] = fma(Bv[0], f0[m], t[0]);
    s0[1] = fma(Bv[1], f0[m], t[1]);
    s0[2] = fma(Bv[2], f0[m], t[2]);
    matvec3(Ab, s1, t);
    s1[0] = fma(Bv[0], f1[m], t[0]);
    s1[1] = fma(Bv[1], f1[m], t[1]);
    s1[2] = fma(Bv[2], f1[m], t[2]);
    if (m == kick_step) s1[1] -= kk;
  }
  Mat3 P = Ab;  // P = Ā^C
  for (int q = 1; q < C; ++q) P = matmul3(P, Ab);
  const double* xb = x0 + b * 6;
  const double xi0[3] = {xb[0], xb[1], xb[2]};
  const double xi1[3] = {xb[3], xb[4], xb[5]};
  if (lane == 0) {
    double t[3];
    matvec3(P, xi0, t);
    for (int i = 0; i < 3; ++i) s0[i] += t[i];
    matvec3(P, xi1, t);
    for (int i = 0; i < 3; ++i) s1[i] += t[i];
  }
  // inclusive Kogge-Stone: T_l += P^d T_{l-d}
  Mat3 Pd = P;
  for (int d = 1; d < ((dbg & 2) ? 1 : 64); d <<= 1) {
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
  double x[3], y[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double p0 = __shfl_up(s0[i], 1, 64);
    const double p1 = __shfl_up(s1[i], 1, 64);
    x[i] = (lane == 0) ? xi0[i] : p0;
    y[i] = (lane == 0) ? xi1[i] : p1;
  }

  // ---- 4. replay in the reference form and store ------------------------------------
  double* hb = hist + b * (int64_t)n * 6;
  if (lane == 0) {
    hb[0] = xi0[0]; hb[1] = xi0[1]; hb[2] = xi0[2];
    hb[3] = xi1[0]; hb[4] = xi1[1]; hb[5] = xi1[2];
  }
  bool finite = true;
  for (int m = mbeg; m < mend; ++m) {
    const double ux = f0[m] - (kx0 * x[0] + kx1 * x[1] + kx2 * x[2]);
    const double uy = f1[m] - (kx0 * y[0] + kx1 * y[1] + kx2 * y[2]);
    double xn[3], yn[3];
    lipm_step(lc, x, ux, xn);
    lipm_step(lc, y, uy, yn);
    if (m == kick_step) yn[1] -= kk;
    double* o = hb + (int64_t)(m + 1) * 6;
    if (dbg & 4) continue;
    reinterpret_cast<double2*>(o)[0] = make_double2(xn[0], xn[1]);
    reinterpret_cast<double2*>(o)[1] = make_double2(xn[2], yn[0]);
    reinterpret_cast<double2*>(o)[2] = make_double2(yn[1], yn[2]);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      x[i] = xn[i];
      y[i] = yn[i];
    }
  }
  if (status != nullptr) {
    finite = isfinite(x[0]) && isfinite(x[1]) && isfinite(x[2]) && isfinite(y[0]) &&
             isfinite(y[1]) && isfinite(y[2]);
    const unsigned long long bad = __ballot(!finite);
    if (lane == 0) status[b] = bad ? ZMPC_ST_NONFINITE : 0;
  }
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

hipError_t zmpc_launch_rollout_unc(const zmpc_plan* p, int64_t B, int64_t n, const double* zmax,
                                   const double* zmin, int64_t bstride, const double* x0,
                                   const double* kick,
                                   int64_t kick_step, double* hist, int32_t* status,
                                   hipStream_t s, std::string* why) {
  const size_t lds = zmpc_rollout_unc_lds_bytes(p->Kpad, n);
  if (lds > 160 * 1024) {
    *why = "walk too long for the LDS-resident rollout (n=" + std::to_string(n) + ")";
    return hipErrorInvalidValue;
  }
  if (n == 1) {
    // no QP solve: the history is the initial state only
    hipError_t e = hipMemcpyAsync(hist, x0, 6 * sizeof(double) * (size_t)B,
                                  hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
    if (status) return hipMemsetAsync(status, 0, sizeof(int32_t) * B, s);
    return hipSuccess;
  }
  static const int dbg = [] {
    const char* e = getenv("ZMPC_DEBUG_ROLLOUT");  // diagnostic ablation bits (0 in production)
    return e ? atoi(e) : 0;
  }();
  hipLaunchKernelGGL(zmpc_rollout_unc_kernel, dim3((unsigned)B), dim3(64), lds, s, p->Kpad,
                     (int)n, p->lc, p->k, p->kx, zmax, zmin, bstride, x0, kick, kick_step, hist,
                     status, dbg);
  return hipGetLastError();
}

hipError_t zmpc_launch_step_unc(const zmpc_plan* p, int64_t B, const double* x,
                                const double* zmax_win, const double* zmin_win, double* x_next,
                                int32_t* status, hipStream_t s) {
  hipLaunchKernelGGL(zmpc_step_unc_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, B,
                     p->N, p->lc, p->k, p->kx, x, zmax_win, zmin_win, x_next, status);
  return hipGetLastError();
}

// The dynamic-LDS ceiling must be raised once per device for > 64 KiB requests.
hipError_t zmpc_rollout_unc_set_attrs() {
  return hipFuncSetAttribute((const void*)zmpc_rollout_unc_kernel,
                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}
