// Plan precompute for the Wieber LIPM-ZMP QP (batch- and timestep-invariant work).
//
// The reference rebuilds all of this inside every predict_wieber_axis call
// (zmp_controller.py:162-171 interpreted O(N²) loop, :198 PuᵀPu and np.linalg.inv); it depends
// only on (N, dt, h, g, Q, R), so it is built once per plan here, on the device:
//   1. p (Toeplitz column of Pu) and Px               zmp_controller.py:166-171
//   2. M = PuᵀPu + (R/Q)·I  — FP64 MFMA at N >= 64     zmp_controller.py:198
//   3. M = L Lᵀ (Cholesky)
//   4. y = M⁻¹ e0, gain row k = Pu y (= row 0 of inv(M) Puᵀ), kx = k·Px
//   5. strict plans: X = L⁻¹ Puᵀ, G = XᵀX / Q = Pu (R·I + Q·PuᵀPu)⁻¹ Puᵀ,
//      the inverse z-space Hessian of the strict QP (zmp_controller.py:173-195).
#include "zmpc_internal.h"

typedef double dbl4 __attribute__((ext_vector_type(4)));

// 1. Toeplitz column and Px, with FP contraction off so the arithmetic is the reference's
//    operation for operation: p(d) = (T**3)/6 * (1+3d+3d²) - T*h/g (zmp_controller.py:171),
//    Px[i] = [1, T*(i+1), (T**2)/2*(i+1)**2 - h/g] (:167-169).
__global__ void zmpc_build_prediction(int N, double T, double T2_2, double T3_6, double hg,
                                      double Thg, double* __restrict__ p,
                                      double* __restrict__ Px) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const long long d = i;
  const double poly = (double)(1 + 3 * d + 3 * d * d);
  p[i] = T3_6 * poly - Thg;
  const long long ip1 = i + 1;
  Px[3 * i + 0] = 1.0;
  Px[3 * i + 1] = T * (double)ip1;
  Px[3 * i + 2] = T2_2 * (double)(ip1 * ip1) - hg;
}

// Operand fetchers for the Gram kernels: value of the (k, a) element of the matrix whose
// columns are contracted, C[a][b] = Σ_k Op(k,a)·Op(k,b).
struct PuOp {  // Pu[k][a] = p(k-a) for k >= a
  const double* p;
  int N;
  __device__ double operator()(int k, int a) const {
    return (k < N && a < N && k >= a) ? p[k - a] : 0.0;
  }
  __device__ int kbegin(int a0, int b0) const { return (a0 > b0 ? a0 : b0) & ~3; }
};
struct ToeplitzOp {  // lower-triangular Toeplitz T[k][a] = c(k-a) for k >= a (Pu, or Pu⁻¹)
  const double* c;
  int N;
  __device__ double operator()(int k, int a) const {
    return (k < N && a < N && k >= a) ? c[k - a] : 0.0;
  }
  __device__ int kbegin(int a0, int b0) const { return (a0 > b0 ? a0 : b0) & ~3; }
};
struct DenseOp {  // X[k][a], row-major N×N
  const double* X;
  int N;
  __device__ double operator()(int k, int a) const {
    return (k < N && a < N) ? X[(size_t)k * N + a] : 0.0;
  }
  __device__ int kbegin(int, int) const { return 0; }
};

// 2/5. C = alpha·OpᵀOp + diag·I with v_mfma_f64_16x16x4_f64: one wave per 16×16 tile.
// Operand lane map (gfx950): A[i = lane&15][k = lane>>4], B[k = lane>>4][j = lane&15];
// result D: col = lane&15, row = (lane>>4) + 4·r.
template <class Op>
__global__ void __launch_bounds__(64) zmpc_gram_mfma(int N, Op op, double alpha, double diag,
                                                     double* __restrict__ C) {
  const int tiles = (N + 15) >> 4;
  const int ta = blockIdx.x / tiles, tb = blockIdx.x % tiles;
  const int a0 = ta << 4, b0 = tb << 4;
  const int lane = threadIdx.x;
  const int r = lane & 15, kq = lane >> 4;
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  for (int k0 = op.kbegin(a0, b0); k0 < N; k0 += 4) {
    const int k = k0 + kq;
    const double av = op(k, a0 + r);
    const double bv = op(k, b0 + r);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int a = a0 + kq + 4 * q, b = b0 + r;
    if (a < N && b < N) C[(size_t)a * N + b] = alpha * acc[q] + (a == b ? diag : 0.0);
  }
}

// Same contraction with scalar FMAs (small N, where a 16×16 tile would be mostly padding).
template <class Op>
__global__ void zmpc_gram_fma(int N, Op op, double alpha, double diag, double* __restrict__ C) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * N) return;
  const int a = idx / N, b = idx % N;
  double s = 0.0;
  for (int k = op.kbegin(a, b); k < N; ++k) s = fma(op(k, a), op(k, b), s);
  C[idx] = alpha * s + (a == b ? diag : 0.0);
}

// 3. Right-looking Cholesky of the N×N matrix in L (in place), one workgroup; the pivot
// column is staged in LDS.  info = 0 on success, k+1 if the k-th pivot is not positive.
__global__ void __launch_bounds__(1024) zmpc_cholesky(int N, double* __restrict__ L,
                                                      int* __restrict__ info) {
  extern __shared__ double col[];  // [N]
  __shared__ int bad;
  const int tid = threadIdx.x, nt = blockDim.x;
  if (tid == 0) bad = 0;
  __syncthreads();
  for (int k = 0; k < N; ++k) {
    const double d = L[(size_t)k * N + k];
    if (!(d > 0.0)) {
      if (tid == 0) { bad = k + 1; }
      break;
    }
    const double piv = sqrt(d);
    for (int i = k + tid; i < N; i += nt) {
      const double v = (i == k) ? piv : L[(size_t)i * N + k] / piv;
      col[i] = v;
    }
    __syncthreads();
    for (int i = k + tid; i < N; i += nt) L[(size_t)i * N + k] = col[i];
    const int m = N - k - 1;
    for (int idx = tid; idx < m * m; idx += nt) {
      const int i = k + 1 + idx / m, j = k + 1 + idx % m;
      if (j <= i) L[(size_t)i * N + j] -= col[i] * col[j];
    }
    __syncthreads();
  }
  __syncthreads();
  for (int idx = tid; idx < N * N; idx += nt) {
    const int i = idx / N, j = idx % N;
    if (j > i) L[idx] = 0.0;
  }
  if (tid == 0) *info = bad;
}

// 4. y = M⁻¹ e0 by two triangular solves in LDS, k = Pu y, kx = k·Px.  One workgroup.
__global__ void __launch_bounds__(1024) zmpc_gain(int N, int Kpad, const double* __restrict__ L,
                                                  const double* __restrict__ p,
                                                  const double* __restrict__ Px,
                                                  double* __restrict__ k,
                                                  double* __restrict__ kx) {
  extern __shared__ double w[];  // [N]
  __shared__ double red[3][1024 / 64];
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int i = tid; i < N; i += nt) w[i] = (i == 0) ? 1.0 : 0.0;
  __syncthreads();
  // forward: L w = e0 (column-oriented)
  for (int j = 0; j < N; ++j) {
    const double wj = w[j] / L[(size_t)j * N + j];
    __syncthreads();
    for (int i = j + 1 + tid; i < N; i += nt) w[i] -= L[(size_t)i * N + j] * wj;
    if (tid == 0) w[j] = wj;
    __syncthreads();
  }
  // backward: Lᵀ y = w  (Lᵀ[i][j] = L[j][i])
  for (int j = N - 1; j >= 0; --j) {
    const double yj = w[j] / L[(size_t)j * N + j];
    __syncthreads();
    for (int i = tid; i < j; i += nt) w[i] -= L[(size_t)j * N + i] * yj;
    if (tid == 0) w[j] = yj;
    __syncthreads();
  }
  // k_j = Σ_{i<=j} p(j-i) y_i ; kx = Σ_j k_j Px[j,:]
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  for (int j = tid; j < Kpad; j += nt) {
    double kj = 0.0;
    if (j < N) {
      for (int i = 0; i <= j; ++i) kj = fma(p[j - i], w[i], kj);
      s0 = fma(kj, Px[3 * j + 0], s0);
      s1 = fma(kj, Px[3 * j + 1], s1);
      s2 = fma(kj, Px[3 * j + 2], s2);
    }
    k[j] = kj;
  }
  for (int off = 32; off > 0; off >>= 1) {
    s0 += __shfl_xor(s0, off);
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
  }
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = s0;
    red[1][tid >> 6] = s1;
    red[2][tid >> 6] = s2;
  }
  __syncthreads();
  if (tid < 3) {
    double s = 0.0;
    for (int q = 0; q < nt / 64; ++q) s += red[tid][q];
    kx[tid] = s;
  }
}

// 4b. Scan matrices of the unconstrained rollout: Ā = A − B kxᵀ and, for C = 1..8,
// (Ā^C)^(2^r), r = 0..5 (the lane-chunk propagators of the Kogge-Stone scan).  One thread.
__global__ void zmpc_scan_matrices(double T, double T2_2, double T3_6,
                                   const double* __restrict__ kx, double* __restrict__ out) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  const double A[9] = {1.0, T, T2_2, 0.0, 1.0, T, 0.0, 0.0, 1.0};
  const double Bv[3] = {T3_6, T2_2, T};
  double Ab[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Ab[3 * i + j] = A[3 * i + j] - Bv[i] * kx[j];
  auto mul = [](const double* x, const double* y, double* z) {
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        z[3 * i + j] = fma(x[3 * i + 0], y[0 + j], fma(x[3 * i + 1], y[3 + j], x[3 * i + 2] * y[6 + j]));
  };
  double P[9];
  for (int q = 0; q < 9; ++q) P[q] = Ab[q];
  for (int C = 1; C <= 8; ++C) {
    if (C > 1) {
      double t[9];
      mul(P, Ab, t);
      for (int q = 0; q < 9; ++q) P[q] = t[q];
    }
    double Q[9];
    for (int q = 0; q < 9; ++q) Q[q] = P[q];
    for (int r = 0; r < kScanLevels; ++r) {
      for (int q = 0; q < 9; ++q) out[(C - 1) * kScanStride + r * 9 + q] = Q[q];
      double t[9];
      mul(Q, Q, t);
      for (int q = 0; q < 9; ++q) Q[q] = t[q];
    }
  }
}

// 5a. X = L⁻¹ Puᵀ: one thread per column c, forward substitution with L broadcast across the
// wave (every lane reads the same L element).  Puᵀ[i][c] = p(c-i) for i <= c.
__global__ void zmpc_solve_LPuT(int N, const double* __restrict__ L, const double* __restrict__ p,
                                double* __restrict__ X) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N) return;
  for (int i = 0; i < N; ++i) {
    double s = (i <= c) ? p[c - i] : 0.0;
    for (int j = 0; j < i; ++j) s = fma(-L[(size_t)i * N + j], X[(size_t)j * N + c], s);
    X[(size_t)i * N + c] = s / L[(size_t)i * N + i];
  }
}

// 5b. v = first column of Pu⁻¹ (lower-triangular Toeplitz again): p * v = e0, one thread.
__global__ void zmpc_toeplitz_inverse(int N, const double* __restrict__ p,
                                      double* __restrict__ v) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  const double p0 = p[0];
  v[0] = 1.0 / p0;
  for (int k = 1; k < N; ++k) {
    double s = 0.0;
    for (int j = 1; j <= k; ++j) s = fma(p[j], v[k - j], s);
    v[k] = -s / p0;
  }
}

template <class Op>
static void launch_gram(int N, Op op, double alpha, double diag, double* C, hipStream_t s) {
  if (N >= 64) {
    const int tiles = (N + 15) / 16;
    hipLaunchKernelGGL(zmpc_gram_mfma<Op>, dim3(tiles * tiles), dim3(64), 0, s, N, op, alpha,
                       diag, C);
  } else {
    hipLaunchKernelGGL(zmpc_gram_fma<Op>, dim3((N * N + 255) / 256), dim3(256), 0, s, N, op,
                       alpha, diag, C);
  }
}

static hipError_t launch_gram_pu(const zmpc_plan* P, double diag, hipStream_t s) {
  PuOp op{P->p, P->N};
  const int N = P->N;
  if (N >= 64) {
    const int tiles = (N + 15) / 16;
    hipLaunchKernelGGL(zmpc_gram_mfma<PuOp>, dim3(tiles * tiles), dim3(64), 0, s, N, op, 1.0,
                       diag, P->M);
  } else {
    hipLaunchKernelGGL(zmpc_gram_fma<PuOp>, dim3((N * N + 255) / 256), dim3(256), 0, s, N, op,
                       1.0, diag, P->M);
  }
  return hipGetLastError();
}

// FFT tables (rollout.hip, long walks): twiddles e^{−2πi m/PT}, m < PT (sincospi: the
// argument −2m/PT is exact), and for every P = 2^p in [kFftPmin, PT] the gain spectrum
// DFT(g)[q]/P, g[d] = k_{d−1} for d = 1..N (the correlation f_i = Σ_d g[d] z_{i+d}), summed
// directly with exact table angles ((q·d) mod P).
__global__ void zmpc_fft_twiddles(double* tw) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= kFftPT) return;
  double sn, cs;
  sincospi(-2.0 * (double)m / (double)kFftPT, &sn, &cs);
  tw[2 * m] = cs;
  tw[2 * m + 1] = sn;
}

__global__ void zmpc_fft_gain(int N, const double* __restrict__ k, const double* __restrict__ tw,
                              double* g) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= kFftGComplex) return;
  int P = kFftPmin;
  while (idx >= 2 * P - kFftPmin) P *= 2;
  const int q = idx - (P - kFftPmin);
  const int sh = kFftPT / P;
  double re = 0.0, im = 0.0;
  int m = 0;  // (q·d) mod P
  for (int d = 1; d <= N; ++d) {
    m = (m + q) & (P - 1);
    const double kd = k[d - 1];
    re = fma(kd, tw[2 * (m * sh)], re);
    im = fma(kd, tw[2 * (m * sh) + 1], im);
  }
  g[2 * idx] = re / P;
  g[2 * idx + 1] = im / P;
}

hipError_t zmpc_launch_plan(zmpc_plan* P, hipStream_t s) {
  const int N = P->N;
  hipError_t e;
  hipLaunchKernelGGL(zmpc_build_prediction, dim3((N + 255) / 256), dim3(256), 0, s, N, P->T,
                     P->T2_2, P->T3_6, P->hg, P->Thg, P->p, P->Px);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // M = PuᵀPu + (R/Q) I   (zmp_controller.py:198: Pu.T @ Pu + self.config.R/self.config.Q * eye)
  if ((e = launch_gram_pu(P, P->R / P->Q, s)) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(P->L, P->M, sizeof(double) * N * N, hipMemcpyDeviceToDevice, s)) !=
      hipSuccess)
    return e;
  hipLaunchKernelGGL(zmpc_cholesky, dim3(1), dim3(1024), sizeof(double) * N, s, N, P->L,
                     P->info);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(zmpc_gain, dim3(1), dim3(1024), sizeof(double) * N, s, N, P->Kpad, P->L,
                     P->p, P->Px, P->k, P->kx);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(zmpc_scan_matrices, dim3(1), dim3(64), 0, s, P->T, P->T2_2, P->T3_6, P->kx,
                     P->scanP);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (P->fft_tw && P->fft_g) {
    hipLaunchKernelGGL(zmpc_fft_twiddles, dim3(kFftPT / 256), dim3(256), 0, s, P->fft_tw);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(zmpc_fft_gain, dim3((kFftGComplex + 255) / 256), dim3(256), 0, s, N, P->k,
                       P->fft_tw, P->fft_g);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (P->strict) {
    hipLaunchKernelGGL(zmpc_solve_LPuT, dim3((N + 63) / 64), dim3(64), 0, s, N, P->L, P->p,
                       P->X);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    DenseOp op{P->X, N};
    if (N >= 64) {
      const int tiles = (N + 15) / 16;
      hipLaunchKernelGGL(zmpc_gram_mfma<DenseOp>, dim3(tiles * tiles), dim3(64), 0, s, N, op,
                         1.0 / P->Q, 0.0, P->G);
    } else {
      hipLaunchKernelGGL(zmpc_gram_fma<DenseOp>, dim3((N * N + 255) / 256), dim3(256), 0, s, N,
                         op, 1.0 / P->Q, 0.0, P->G);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // z-space Hessian H = Q·I + R·Pu⁻ᵀPu⁻¹ for the primal side of the strict active set
    hipLaunchKernelGGL(zmpc_toeplitz_inverse, dim3(1), dim3(64), 0, s, N, P->p, P->v);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    launch_gram(N, ToeplitzOp{P->v, N}, P->R, P->Q, P->Hz, s);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  return hipSuccess;
}
