// Probe: the largest dynamic LDS a 1024- / 512- / 256-thread workgroup can launch with on this
// device once hipFuncAttributeMaxDynamicSharedMemorySize is raised (diagnostics only).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(1024) k1024(double* o) {
  extern __shared__ double sm[];
  sm[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) o[blockIdx.x] = sm[5];
}
__global__ void __launch_bounds__(512) k512(double* o) {
  extern __shared__ double sm[];
  sm[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) o[blockIdx.x] = sm[5];
}
int main() {
  double* o;
  (void)hipMalloc(&o, 1024 * 8);
  hipDeviceProp_t pr;
  (void)hipGetDeviceProperties(&pr, 0);
  printf("sharedMemPerBlock %zu maxSharedMemoryPerMultiProcessor %zu\n", pr.sharedMemPerBlock,
         pr.maxSharedMemoryPerMultiProcessor);
  hipError_t e1 = hipFuncSetAttribute((const void*)k1024, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipError_t e2 = hipFuncSetAttribute((const void*)k512, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  printf("set attr: %d %d\n", (int)e1, (int)e2);
  for (int kb : {64, 65, 80, 96, 128, 160}) {
    hipLaunchKernelGGL(k1024, dim3(4), dim3(1024), kb * 1024, 0, o);
    hipError_t a = hipGetLastError();
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(k512, dim3(4), dim3(512), kb * 1024, 0, o);
    hipError_t b = hipGetLastError();
    (void)hipDeviceSynchronize();
    printf("%3d KiB: 1024 threads %s, 512 threads %s\n", kb, hipGetErrorString(a), hipGetErrorString(b));
  }
  return 0;
}
