// Plan precompute for the Wieber LIPM-ZMP QP (batch- and timestep-invariant work).
//
// The reference rebuilds all of this inside every predict_wieber_axis call
// (zmp_controller.py:162-171 interpreted O(N²) loop, :198 PuᵀPu and np.linalg.inv); it depends
// only on (N, dt, h, g, Q, R), so it is built once per plan here, on the device:
//   1. p (Toeplitz column of Pu) and Px               zmp_controller.py:166-171
//   2. M = PuᵀPu + (R/Q)·I  — FP64 MFMA at N >= 64     zmp_controller.py:198
//   3. M = L Lᵀ (blocked Cholesky, 16-column panels, FP64 MFMA panel updates)
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
// columns are contracted, C[a][b] = Σ_k Op(k,a)·Op(k,b).  `stage` copies what the operand reads
// into LDS once per workgroup (the Toeplitz column: N doubles) so the K loop reads LDS.
struct ToeplitzOp {  // lower-triangular Toeplitz T[k][a] = c(k-a) for k >= a (Pu, or Pu⁻¹)
  const double* c;
  int N;
  static constexpr bool kStaged = true;
  __device__ double at(const double* sc, int k, int a) const {
    return (k < N && a < N && k >= a) ? sc[k - a] : 0.0;
  }
  __device__ int kbegin(int a0, int b0) const { return (a0 > b0 ? a0 : b0) & ~3; }
};
using PuOp = ToeplitzOp;  // Pu[k][a] = p(k-a)
struct DenseOp {  // X[k][a], row-major N×N
  const double* X;
  int N;
  static constexpr bool kStaged = false;
  __device__ double at(const double*, int k, int a) const {
    return (k < N && a < N) ? X[(size_t)k * N + a] : 0.0;
  }
  __device__ int kbegin(int, int) const { return 0; }
};

// 2/5. C = alpha·OpᵀOp + diag·I with v_mfma_f64_16x16x4_f64: one wave per 16×16 tile of the
// lower triangle (ta >= tb; C is symmetric, the tile is written to both halves), two
// accumulators alternating so consecutive MFMAs do not wait on each other's result.
// Operand lane map (gfx950): A[i = lane&15][k = lane>>4], B[k = lane>>4][j = lane&15];
// result D: col = lane&15, row = (lane>>4) + 4·r.
template <class Op>
__global__ void __launch_bounds__(64) zmpc_gram_mfma(int N, Op op, double alpha, double diag,
                                                     double* __restrict__ C) {
  extern __shared__ double sc[];  // staged operand (Toeplitz column), N doubles
  const int t = blockIdx.x;
  int ta = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((ta + 1) * (ta + 2) / 2 <= t) ++ta;
  while (ta * (ta + 1) / 2 > t) --ta;
  const int tb = t - ta * (ta + 1) / 2;
  const int a0 = ta << 4, b0 = tb << 4;
  const int lane = threadIdx.x;
  const int r = lane & 15, kq = lane >> 4;
  if constexpr (Op::kStaged) {
    for (int j = lane; j < N; j += 64) sc[j] = op.c[j];
    __syncthreads();
  }
  dbl4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
  int k0 = op.kbegin(a0, b0);
  for (; k0 + 4 < N; k0 += 8) {
    const double av0 = op.at(sc, k0 + kq, a0 + r), bv0 = op.at(sc, k0 + kq, b0 + r);
    const double av1 = op.at(sc, k0 + 4 + kq, a0 + r), bv1 = op.at(sc, k0 + 4 + kq, b0 + r);
    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av0, bv0, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av1, bv1, acc1, 0, 0, 0);
  }
  if (k0 < N) {
    const double av = op.at(sc, k0 + kq, a0 + r), bv = op.at(sc, k0 + kq, b0 + r);
    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc0, 0, 0, 0);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int a = a0 + kq + 4 * q, b = b0 + r;
    const double v = alpha * (acc0[q] + acc1[q]) + (a == b ? diag : 0.0);
    if (a < N && b < N) {
      C[(size_t)a * N + b] = v;
      if (ta != tb) C[(size_t)b * N + a] = v;
    }
  }
}

// Same contraction with scalar FMAs (small N, where a 16×16 tile would be mostly padding).
template <class Op>
__global__ void zmpc_gram_fma(int N, Op op, double alpha, double diag, double* __restrict__ C) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * N) return;
  const int a = idx / N, b = idx % N;
  double s = 0.0;
  const double* src = nullptr;
  if constexpr (Op::kStaged) src = op.c;
  for (int k = op.kbegin(a, b); k < N; ++k) s = fma(op.at(src, k, a), op.at(src, k, b), s);
  C[idx] = alpha * s + (a == b ? diag : 0.0);
}

// 3. Blocked left-looking Cholesky M = L Lᵀ (L written from M), 16-column panels, one launch per
// panel p0 (p0 = 0, 16, 32, ...), one wave per 16-row tile of rows [p0, N).  Every wave
//  (a) forms the panel's diagonal tile D = M[p0.., p0..] − L[p0.., :p0]·L[p0.., :p0]ᵀ and its own
//      tile T = M[r0.., p0..] − L[r0.., :p0]·L[p0.., :p0]ᵀ with v_mfma_f64_16x16x4_f64 (K = p0,
//      the L rows streamed 16 columns per batch, loads issued ahead of the MFMAs),
//  (b) factors D = Lpp·Lppᵀ in registers (lane i holds row i; columns broadcast by shuffles),
//  (c) solves its tile, L[r0.., p0..] = T·Lpp⁻ᵀ (lane i owns row i),
// and wave 0 writes Lpp and zeroes the upper triangle of its 16 rows.  The M entries come from
// M itself, never from L: wave 0 overwrites the diagonal block in L while the other waves of the
// launch may still be reading it.  Every entry of L is written by some panel (lower part as
// Lpp / T, upper part zeroed), so L needs no initial copy of M.
// info = 0 on success, else the first non-positive pivot's index + 1.
__global__ void __launch_bounds__(64) zmpc_chol_panel(int N, int p0, const double* __restrict__ M,
                                                      double* __restrict__ L,
                                                      int* __restrict__ info) {
  __shared__ double sD[16][17];
  __shared__ double sT[16][17];
  const int lane = threadIdx.x, r = lane & 15, kq = lane >> 4;
  const int r0 = p0 + 16 * blockIdx.x;
  const bool diag = blockIdx.x == 0;
  const int pr = p0 + r, tr = r0 + r;
  const bool pok = pr < N, tok = tr < N;
  const double* Lp = L + (size_t)(pok ? pr : 0) * N;
  const double* Lt = L + (size_t)(tok ? tr : 0) * N;
  dbl4 accD = {0.0, 0.0, 0.0, 0.0}, accT = {0.0, 0.0, 0.0, 0.0};
  // k = k0 + 4·kq + u: each lane reads 4 consecutive doubles of its row per batch; A and B of
  // one MFMA step come from the same (kq, u), so the contraction runs over every k < p0 once
  for (int k0 = 0; k0 < p0; k0 += 16) {
    double a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + 4 * kq + u;
      a[u] = pok ? Lp[k] : 0.0;
      b[u] = (!diag && tok) ? Lt[k] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      accD = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], a[u], accD, 0, 0, 0);
      if (!diag) accT = __builtin_amdgcn_mfma_f64_16x16x4f64(b[u], a[u], accT, 0, 0, 0);
    }
  }
  // acc[q] = (row kq + 4q, column r) of the product; subtract from M (identity padding past N)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = kq + 4 * q;
    const bool inD = (p0 + i < N) && pok;
    sD[i][r] = inD ? M[(size_t)(p0 + i) * N + pr] - accD[q] : (i == r ? 1.0 : 0.0);
    if (!diag) {
      const bool inT = (r0 + i < N) && pok;
      sT[i][r] = inT ? M[(size_t)(r0 + i) * N + pr] - accT[q] : 0.0;
    }
  }
  __syncthreads();
  // (b) 16×16 Cholesky, lane r holds row r of D (every lane group of 16 computes the same)
  double d[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) d[c] = sD[r][c];
  int bad = 0;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const double dc = __shfl(d[c], c, 64);
    if (!(dc > 0.0) && bad == 0) bad = c + 1;
    const double piv = sqrt(dc);
    const double l = (r == c) ? piv : d[c] / piv;  // L[r][c] for r >= c
    d[c] = (r >= c) ? l : 0.0;
#pragma unroll
    for (int j = c + 1; j < 16; ++j) {
      const double ljc = __shfl(l, j, 64);
      if (r >= j) d[j] = fma(-l, ljc, d[j]);
    }
  }
  if (diag) {
    if (kq == 0 && pok) {
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if (p0 + c < N) L[(size_t)pr * N + p0 + c] = d[c];
    }
    if (pok)
      for (int j = p0 + 16 + kq; j < N; j += 4) L[(size_t)pr * N + j] = 0.0;
    if (lane == 0 && bad != 0 && *info == 0) *info = p0 + bad;
    return;
  }
  // (c) X·Lppᵀ = T row by row: X[r][c] = (T[r][c] − Σ_{m<c} X[r][m]·Lpp[c][m]) / Lpp[c][c]
  double t[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) t[c] = sT[r][c];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    double acc = t[c];
#pragma unroll
    for (int m = 0; m < c; ++m) acc = fma(-t[m], __shfl(d[m], c, 64), acc);
    t[c] = acc / __shfl(d[c], c, 64);
  }
  if (kq == 0 && tok) {
#pragma unroll
    for (int c = 0; c < 16; ++c)
      if (p0 + c < N) L[(size_t)tr * N + p0 + c] = t[c];
  }
}

// 4b. the rollout's two-parallel fast-FIR taps (rollout.hip, axis_correlate_ffa): row m holds
// (E_m, O_m, E_m + O_{m−1}, 0) with E_m = k_{2m}, O_m = k_{2m+1}, zero outside [0, N)
__global__ void zmpc_ffa_taps(int N, const double* __restrict__ k, double* __restrict__ t) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= kffa_rows(N)) return;
  const double e = (2 * m < N) ? k[2 * m] : 0.0;
  const double o = (2 * m + 1 < N) ? k[2 * m + 1] : 0.0;
  const double op = (m >= 1 && 2 * m - 1 < N) ? k[2 * m - 1] : 0.0;
  t[4 * m + 0] = e;
  t[4 * m + 1] = o;
  t[4 * m + 2] = e + op;
  t[4 * m + 3] = 0.0;
}

// 4c. suffix sums of the gain row for the rollout's sparse-difference correlation (rollout.hip,
// axis_correlate_sparse): S_j = k_j + S_{j+1} from j = N − 1 down, laid out as ksum_rows says.
// One wave; the sum is sequential in one lane (N ≤ 4096 additions, once per plan).
__global__ void __launch_bounds__(64) zmpc_ksum(int N, const double* __restrict__ k,
                                                double* __restrict__ t) {
  const int lane = threadIdx.x;
  for (int i = lane; i < ksum_rows(N); i += 64)
    if ((i < 9 || i >= N + 8) && i != ksum_s0(N)) t[i] = 0.0;
  if (lane == 0) {
    double acc = 0.0;
    for (int j = N - 1; j >= 1; --j) {
      acc += k[j];
      t[j + 8] = acc;
    }
    t[ksum_s0(N)] = acc + k[0];
  }
}

// 4. y = M⁻¹ e0 by two blocked triangular solves (64-row blocks), then k = Pu y, kx = k·Px.
// One 1024-thread workgroup.  Per block: the off-block part of every row's dot product is a
// wave reduction over coalesced row (forward) / column-block (backward) reads, the 64×64
// diagonal block is staged in LDS and solved by wave 0 with shuffles — two barriers per block
// instead of two per column.
__global__ void __launch_bounds__(1024) zmpc_gain(int N, int Kpad, const double* __restrict__ L,
                                                  const double* __restrict__ p,
                                                  const double* __restrict__ Px,
                                                  double* __restrict__ k,
                                                  double* __restrict__ kx) {
  extern __shared__ double w[];             // [N]
  __shared__ double blk[64][65];            // diagonal block
  __shared__ double part[16][64];           // partial sums
  __shared__ double red[3][1024 / 64];
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wv = tid >> 6;
  // forward: L w = e0
  for (int b0 = 0; b0 < N; b0 += 64) {
    const int nb = min(64, N - b0);
    for (int idx = tid; idx < 64 * 64; idx += nt) {
      const int i = idx >> 6, c = idx & 63;
      blk[i][c] = (i < nb && c < nb) ? L[(size_t)(b0 + i) * N + b0 + c] : 0.0;
    }
    // t_i = Σ_{c<b0} L[b0+i][c] w[c]: wave wv takes rows wv, wv+16, ...; lanes over c
    for (int i = wv; i < nb; i += 16) {
      double s = 0.0;
      const double* row = L + (size_t)(b0 + i) * N;
      for (int c = lane; c < b0; c += 64) s = fma(row[c], w[c], s);
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
      if (lane == 0) part[0][i] = s;
    }
    __syncthreads();
    if (wv == 0) {
      double v = ((b0 + lane == 0) ? 1.0 : 0.0) - (lane < nb ? part[0][lane] : 0.0);
      for (int c = 0; c < nb; ++c) {
        const double wc = __shfl(v, c, 64) / blk[c][c];
        if (lane == c) v = wc;
        else if (lane > c) v = fma(-blk[lane][c], wc, v);
      }
      if (lane < nb) w[b0 + lane] = v;
    }
    __syncthreads();
  }
  // backward: Lᵀ y = w (y overwrites w), blocks from the end
  for (int b0 = ((N - 1) / 64) * 64; b0 >= 0; b0 -= 64) {
    const int nb = min(64, N - b0);
    for (int idx = tid; idx < 64 * 64; idx += nt) {
      const int i = idx >> 6, c = idx & 63;
      blk[i][c] = (i < nb && c < nb) ? L[(size_t)(b0 + i) * N + b0 + c] : 0.0;
    }
    // t_c = Σ_{i >= b0+64} L[i][b0+c] y_i: thread (wv, lane = c), rows i = b0+64+wv, += 16
    {
      double s = 0.0;
      if (lane < nb)
        for (int i = b0 + 64 + wv; i < N; i += 16) s = fma(L[(size_t)i * N + b0 + lane], w[i], s);
      part[wv][lane] = s;
    }
    __syncthreads();
    if (wv == 0) {
      double t = 0.0;
      for (int g = 0; g < 16; ++g) t += part[g][lane];
      double v = lane < nb ? w[b0 + lane] - t : 0.0;
      for (int c = nb - 1; c >= 0; --c) {
        const double yc = __shfl(v, c, 64) / blk[c][c];
        if (lane == c) v = yc;
        else if (lane < c) v = fma(-blk[c][lane], yc, v);
      }
      if (lane < nb) w[b0 + lane] = v;
    }
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
  {  // chunk-sum columns: V_p = Ā^p B, E_p = Ā^p e1
    double V[3] = {Bv[0], Bv[1], Bv[2]}, E[3] = {0.0, 1.0, 0.0};
    for (int p = 0; p < 8; ++p) {
      for (int i = 0; i < 3; ++i) {
        out[kScanGOff + p * 6 + i] = V[i];
        out[kScanGOff + p * 6 + 3 + i] = E[i];
      }
      double v2[3], e2[3];
      for (int i = 0; i < 3; ++i) {
        v2[i] = fma(Ab[3 * i], V[0], fma(Ab[3 * i + 1], V[1], Ab[3 * i + 2] * V[2]));
        e2[i] = fma(Ab[3 * i], E[0], fma(Ab[3 * i + 1], E[1], Ab[3 * i + 2] * E[2]));
      }
      for (int i = 0; i < 3; ++i) {
        V[i] = v2[i];
        E[i] = e2[i];
      }
    }
  }
  double P[9];
  for (int q = 0; q < 9; ++q) P[q] = Ab[q];
  for (int C = 1; C <= 8; ++C) {
    if (C > 1) {
      double t[9];
      mul(P, Ab, t);
      for (int q = 0; q < 9; ++q) P[q] = t[q];
    }
    // per-lane powers (Ā^C)^k, k = 0..32
    {
      double W[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
      for (int k = 0; k <= 32; ++k) {
        for (int q = 0; q < 9; ++q) out[kScanPowOff + ((C - 1) * 33 + k) * 9 + q] = W[q];
        double t[9];
        mul(W, P, t);
        for (int q = 0; q < 9; ++q) W[q] = t[q];
      }
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

// 5a. X = L⁻¹ Puᵀ (N×N, X starts as Puᵀ: X[i][c] = p(c−i), i <= c): blocked forward
// substitution, one launch per 16-row block r0, one wave per 16-column tile c0.  The wave forms
// T = X[r0.., c0..] − L[r0.., :r0]·X[:r0, c0..] with v_mfma_f64_16x16x4_f64, then solves
// Lbb·Y = T column by column (lane r owns column r; Lbb staged in LDS).
__global__ void zmpc_init_PuT(int N, const double* __restrict__ p, double* __restrict__ X) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * N) return;
  const int i = idx / N, c = idx % N;
  X[idx] = (i <= c) ? p[c - i] : 0.0;
}

__global__ void __launch_bounds__(64) zmpc_trsm_panel(int N, int r0, const double* __restrict__ L,
                                                      double* __restrict__ X) {
  __shared__ double sT[16][17];
  __shared__ double sL[16][17];
  const int lane = threadIdx.x, r = lane & 15, kq = lane >> 4;
  const int c0 = 16 * blockIdx.x;
  const int ar = r0 + r, xc = c0 + r;
  const bool aok = ar < N, cok = xc < N;
  const double* La = L + (size_t)(aok ? ar : 0) * N;
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  for (int k0 = 0; k0 < r0; k0 += 16) {
    double a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int kk = k0 + 4 * kq + u;
      a[u] = aok ? La[kk] : 0.0;                         // A[i = r][k] = L[r0+r][kk]
      b[u] = cok ? X[(size_t)kk * N + xc] : 0.0;         // B[k][j = r] = X[kk][c0+r]
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[u], acc, 0, 0, 0);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = kq + 4 * q;  // row of the tile, column r
    sT[i][r] = (r0 + i < N && cok) ? X[(size_t)(r0 + i) * N + xc] - acc[q] : 0.0;
    sL[i][r] = (r0 + i < N && r0 + r < N) ? L[(size_t)(r0 + i) * N + r0 + r]
                                          : (i == r ? 1.0 : 0.0);
  }
  __syncthreads();
  double y[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    double v = sT[i][r];
#pragma unroll
    for (int m = 0; m < i; ++m) v = fma(-sL[i][m], y[m], v);
    y[i] = v / sL[i][i];
  }
  if (kq == 0 && cok) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (r0 + i < N) X[(size_t)(r0 + i) * N + xc] = y[i];
  }
}

// 5b. v = first column of Pu⁻¹ (lower-triangular Toeplitz again): p * v = e0, i.e.
// v_k = −(Σ_{j=1..k} p_j v_{k−j}) / p0 — sequential in k, each sum a wave reduction; p and v in
// LDS.  One wave.
__global__ void __launch_bounds__(64) zmpc_toeplitz_inverse(int N, const double* __restrict__ p,
                                                            double* __restrict__ v) {
  extern __shared__ double sm[];  // p [N], v [N]
  double* sp = sm;
  double* sv = sm + N;
  const int lane = threadIdx.x;
  for (int j = lane; j < N; j += 64) sp[j] = p[j];
  __syncthreads();
  const double p0 = sp[0];
  if (lane == 0) sv[0] = 1.0 / p0;
  __syncthreads();
  for (int kk = 1; kk < N; ++kk) {
    double s = 0.0;
    for (int j = 1 + lane; j <= kk; j += 64) s = fma(sp[j], sv[kk - j], s);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) sv[kk] = -s / p0;
    __syncthreads();
  }
  for (int j = lane; j < N; j += 64) v[j] = sv[j];
}

template <class Op>
static void launch_gram(int N, Op op, double alpha, double diag, double* C, hipStream_t s) {
  if (N >= 64) {
    const int tiles = (N + 15) / 16;
    const size_t lds = Op::kStaged ? sizeof(double) * N : 0;
    hipLaunchKernelGGL(zmpc_gram_mfma<Op>, dim3(tiles * (tiles + 1) / 2), dim3(64), lds, s, N,
                       op, alpha, diag, C);
  } else {
    hipLaunchKernelGGL(zmpc_gram_fma<Op>, dim3((N * N + 255) / 256), dim3(256), 0, s, N, op,
                       alpha, diag, C);
  }
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

hipError_t zmpc_launch_plan(zmpc_plan* P, hipStream_t s, hipEvent_t* ev) {
  const int N = P->N;
  hipError_t e;
  // stage boundary i: ev[i] (recorded at most once, in order)
  int stage = 0;
  auto mark = [&](int upto) -> hipError_t {
    if (!ev) return hipSuccess;
    for (; stage <= upto; ++stage) {
      hipError_t r = hipEventRecord(ev[stage], s);
      if (r != hipSuccess) return r;
    }
    return hipSuccess;
  };
  if ((e = mark(0)) != hipSuccess) return e;
  hipLaunchKernelGGL(zmpc_build_prediction, dim3((N + 255) / 256), dim3(256), 0, s, N, P->T,
                     P->T2_2, P->T3_6, P->hg, P->Thg, P->p, P->Px);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = mark(1)) != hipSuccess) return e;
  // M = PuᵀPu + (R/Q) I   (zmp_controller.py:198: Pu.T @ Pu + self.config.R/self.config.Q * eye)
  launch_gram(N, PuOp{P->p, N}, 1.0, P->R / P->Q, P->M, s);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = mark(2)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(P->info, 0, sizeof(int), s)) != hipSuccess) return e;
  for (int p0 = 0; p0 < N; p0 += 16) {
    hipLaunchKernelGGL(zmpc_chol_panel, dim3((N - p0 + 15) / 16), dim3(64), 0, s, N, p0, P->M,
                       P->L, P->info);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if ((e = mark(3)) != hipSuccess) return e;
  // w[N] (up to 32 KiB at N = 4096) on top of ≈42 KiB of static LDS
  if ((e = hipFuncSetAttribute((const void*)zmpc_gain, hipFuncAttributeMaxDynamicSharedMemorySize,
                               96 * 1024)) != hipSuccess)
    return e;
  hipLaunchKernelGGL(zmpc_gain, dim3(1), dim3(1024), sizeof(double) * N, s, N, P->Kpad, P->L,
                     P->p, P->Px, P->k, P->kx);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(zmpc_ffa_taps, dim3((kffa_rows(N) + 63) / 64), dim3(64), 0, s, N, P->k,
                     P->kffa);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(zmpc_ksum, dim3(1), dim3(64), 0, s, N, P->k, P->ksum);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = mark(4)) != hipSuccess) return e;
  hipLaunchKernelGGL(zmpc_scan_matrices, dim3(1), dim3(64), 0, s, P->T, P->T2_2, P->T3_6, P->kx,
                     P->scanP);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = mark(5)) != hipSuccess) return e;
  if (P->fft_tw && P->fft_g) {
    hipLaunchKernelGGL(zmpc_fft_twiddles, dim3(kFftPT / 256), dim3(256), 0, s, P->fft_tw);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(zmpc_fft_gain, dim3((kFftGComplex + 255) / 256), dim3(256), 0, s, N, P->k,
                       P->fft_tw, P->fft_g);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if ((e = mark(6)) != hipSuccess) return e;
  if (P->strict) {
    hipLaunchKernelGGL(zmpc_init_PuT, dim3((N * N + 255) / 256), dim3(256), 0, s, N, P->p, P->X);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    for (int r0 = 0; r0 < N; r0 += 16) {
      hipLaunchKernelGGL(zmpc_trsm_panel, dim3((N + 15) / 16), dim3(64), 0, s, N, r0, P->L, P->X);
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if ((e = mark(7)) != hipSuccess) return e;
    launch_gram(N, DenseOp{P->X, N}, 1.0 / P->Q, 0.0, P->G, s);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = mark(8)) != hipSuccess) return e;
    // z-space Hessian H = Q·I + R·Pu⁻ᵀPu⁻¹ for the primal side of the strict active set
    hipLaunchKernelGGL(zmpc_toeplitz_inverse, dim3(1), dim3(64), 2 * sizeof(double) * N, s, N,
                       P->p, P->v);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = mark(9)) != hipSuccess) return e;
    launch_gram(N, ToeplitzOp{P->v, N}, P->R, P->Q, P->Hz, s);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  // stage 10 (the strict LQ table) and the total are recorded by the caller
  return mark(10);
}
