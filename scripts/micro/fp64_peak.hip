// Diagnostic micro-benchmark: sustained FP64 FMA rate of the VALU (register-only chains) and
// of an LDS-fed correlation loop shaped like the rollout's (CW outputs per lane, k from SMEM).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int CH>
__global__ void __launch_bounds__(256) fma_chains(double* out, int iters, double a, double b) {
  double acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x * 1e-3 + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = fma(acc[c], a, b);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef double dbl4 __attribute__((ext_vector_type(4)));
template <int CH>
__global__ void __launch_bounds__(256) mfma_chains(double* out, int iters, double a0) {
  dbl4 acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = dbl4{0.0, 0.0, 0.0, 0.0};
  double a = a0 + threadIdx.x * 1e-6, b = 1.0 - threadIdx.x * 1e-7;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CW>
__global__ void __launch_bounds__(128) corr_lds(const double* __restrict__ k, int kc, double* out, int reps) {
  __shared__ double z[64 * CW + 1024];
  for (int t = threadIdx.x; t < 64 * CW + 1024; t += blockDim.x) z[t] = 1e-3 * t;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  double f[CW];
#pragma unroll
  for (int m = 0; m < CW; ++m) f[m] = 0;
  for (int r = 0; r < reps; ++r) {
    const double* zp = z + lane * CW;
    double w[CW];
#pragma unroll
    for (int m = 0; m < CW; ++m) w[m] = zp[1 + m];
    for (int j = 0; j < kc; j += CW) {
#pragma unroll
      for (int jj = 0; jj < CW; ++jj) {
        const double kj = k[j + jj];
#pragma unroll
        for (int m = 0; m < CW; ++m) f[m] = fma(kj, w[(jj + m) % CW], f[m]);
        w[jj] = zp[1 + jj + CW];
      }
      zp += CW;
    }
  }
  double s = 0;
#pragma unroll
  for (int m = 0; m < CW; ++m) s += f[m];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int clk = 0;
  CHECK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
  printf("CUs %d, max clock %.0f MHz\n", cus, clk / 1e3);
  double* out;
  CHECK(hipMalloc(&out, sizeof(double) * 4096 * 1024));
  double* k;
  CHECK(hipMalloc(&k, sizeof(double) * 2048));
  CHECK(hipMemset(k, 0, sizeof(double) * 2048));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int iters = 4000;
  for (int wpsimd : {1, 2, 4, 8}) {
    const int blocks = cus * wpsimd;  // 256 threads = 4 waves: one per SIMD per block
    for (int rep = 0; rep < 2; ++rep) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(fma_chains<8>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001, 1e-9);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
    }
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double flops = 2.0 * 8 * iters * (double)blocks * 256;
    printf("fma_chains<8> waves/SIMD=%d: %.3f ms, %.1f TFLOP/s FP64\n", wpsimd, ms, flops / ms / 1e9);
  }
  for (int wpsimd : {1, 2, 4}) {
    const int blocks = cus * wpsimd;
    for (int rep = 0; rep < 2; ++rep) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(mfma_chains<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-3);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
    }
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double flops = 2.0 * 1024 * 4 * iters * (double)blocks * 4;  // 4 waves per block
    printf("mfma_f64_16x16x4 chains<4> waves/SIMD=%d: %.3f ms, %.1f TFLOP/s FP64, %.1f cycles/MFMA at 2.4 GHz\n",
           wpsimd, ms, flops / ms / 1e9, ms * 1e-3 * 2.4e9 / (4.0 * iters * wpsimd));
  }
  const int kc = 154, reps = 200;
  for (int wpsimd : {2, 4, 8}) {
    const int blocks = cus * wpsimd * 2;  // 128 threads = 2 waves
    for (int rep = 0; rep < 2; ++rep) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(corr_lds<7>, dim3(blocks), dim3(128), 0, 0, k, kc, out, reps);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
    }
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double flops = 2.0 * 7 * kc * reps * (double)blocks * 128;
    printf("corr_lds<7> waves/SIMD=%d: %.3f ms, %.1f TFLOP/s FP64\n", wpsimd, ms, flops / ms / 1e9);
  }
  return 0;
}
