// Diagnostic micro-benchmark: do FP64 MFMA (v_mfma_f64_16x16x4_f64) and FP64 VALU FMA run
// concurrently on one SIMD?  512-thread workgroups, one per CU: waves w and w+4 share a SIMD.
// mode 0: all 8 waves VALU; 1: all 8 MFMA; 2: waves 0-3 VALU, 4-7 MFMA; 3: only waves 0-3 VALU
// (4-7 exit); 4: only waves 4-7 MFMA.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef double dbl4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double valu_work(int iters, double a, double b) {
  double acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = threadIdx.x * 1e-3 + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = fma(acc[c], a, b);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) s += acc[c];
  return s;
}

__device__ __forceinline__ double mfma_work(int iters, double a0) {
  dbl4 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = dbl4{0.0, 0.0, 0.0, 0.0};
  double a = a0 + threadIdx.x * 1e-6, b = 1.0 - threadIdx.x * 1e-7;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < 4; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  return s;
}

__global__ void __launch_bounds__(512) mix(double* out, int mode, int vit, int mit) {
  const int w = threadIdx.x >> 6;
  double s = 0;
  const bool valu = (mode == 0) || ((mode == 2 || mode == 3) && w < 4);
  const bool mfma = (mode == 1) || ((mode == 2 || mode == 4) && w >= 4);
  if (valu) s = valu_work(vit, 1.0000001, 1e-9);
  if (mfma) s = mfma_work(mit, 1e-3);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  double* out;
  CHECK(hipMalloc(&out, sizeof(double) * 512 * cus * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // per wave: VALU 8 chains x vit FMA instr; MFMA 4 chains x mit MFMAs (2048 FLOP each)
  const int vit = 4000, mit = 1000;
  const char* names[] = {"8 VALU waves", "8 MFMA waves", "4 VALU + 4 MFMA", "4 VALU only", "4 MFMA only"};
  for (int mode = 0; mode < 5; ++mode) {
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(mix, dim3(cus), dim3(512), 0, 0, out, mode, vit, mit);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
    }
    const double vw = (mode == 0) ? 8 : (mode == 2 || mode == 3) ? 4 : 0;
    const double mw = (mode == 1) ? 8 : (mode == 2 || mode == 4) ? 4 : 0;
    const double vflop = vw * 64.0 * 8 * vit * 2 * cus;
    const double mflop = mw * 4.0 * mit * 2048 * cus;
    printf("%-18s %.3f ms  VALU %.1f TF  MFMA %.1f TF  total %.1f TF\n", names[mode], ms,
           vflop / ms / 1e9, mflop / ms / 1e9, (vflop + mflop) / ms / 1e9);
  }
  return 0;
}
