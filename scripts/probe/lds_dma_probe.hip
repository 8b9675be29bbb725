// Probe of the LDS-DMA idiom strict_lq.hip uses for its checkpoint prefetch: a [9][64]-double
// block copied global → LDS by four dwordx4 and two dword DMAs at a given LDS byte offset, read
// back per lane.  Usage: lds_dma_probe  (prints one line per tested offset; exit 1 on mismatch)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int SIZE>
__device__ __forceinline__ void lds_dma(void* dst, const void* src) {
  static_assert(SIZE == 16 || SIZE == 4, "dwordx4 or dword");
  const unsigned d = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)dst);
  const uintptr_t g = (uintptr_t)src;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(g & 0xffffffffu));
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(g >> 32));
  const unsigned long long base = ((unsigned long long)hi << 32) | lo;
  unsigned long long ex;
  unsigned keep, t;
  if constexpr (SIZE == 16)
    asm volatile(
        "s_mov_b64 %0, exec\n\ts_mov_b64 exec, -1\n\t"
        "v_mbcnt_lo_u32_b32 %2, -1, 0\n\tv_mbcnt_hi_u32_b32 %2, -1, %2\n\t"
        "v_lshlrev_b32 %2, 4, %2\n\t"
        "s_mov_b32 %1, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %2, %4\n\t"
        "s_mov_b32 m0, %1\n\ts_mov_b64 exec, %0"
        : "=&s"(ex), "=&s"(keep), "=&v"(t)
        : "s"(d), "s"(base)
        : "memory");
  else
    asm volatile(
        "s_mov_b64 %0, exec\n\ts_mov_b64 exec, -1\n\t"
        "v_mbcnt_lo_u32_b32 %2, -1, 0\n\tv_mbcnt_hi_u32_b32 %2, -1, %2\n\t"
        "v_lshlrev_b32 %2, 2, %2\n\t"
        "s_mov_b32 %1, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "global_load_lds_dword %2, %4\n\t"
        "s_mov_b32 m0, %1\n\ts_mov_b64 exec, %0"
        : "=&s"(ex), "=&s"(keep), "=&v"(t)
        : "s"(d), "s"(base)
        : "memory");
}
__device__ __forceinline__ void lds_dma16(void* dst, const void* src) { lds_dma<16>(dst, src); }
__device__ __forceinline__ void lds_dma4(void* dst, const void* src) { lds_dma<4>(dst, src); }

// store → DMA visibility: the wave stores a [9][64] block lane-wise (lane l: field f at
// f·64 + l), DMAs it, then stores a second pattern to the same bytes and DMAs again.
__global__ void probe_st(double* buf, double* out, int off) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  double* slot = reinterpret_cast<double*>(smem + off);
  for (int round = 0; round < 2; ++round) {
    for (int f = 0; f < 9; ++f) buf[f * 64 + lane] = round * 10000.0 + f * 64 + lane;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const char* s = reinterpret_cast<const char*>(buf);
    char* d = reinterpret_cast<char*>(slot);
    for (int c = 0; c < 4; ++c) lds_dma16(d + c * 1024, s + c * 1024);
    lds_dma4(d + 4096, s + 4096);
    lds_dma4(d + 4352, s + 4352);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int f = 0; f < 9; ++f) out[round * 576 + f * 64 + lane] = slot[f * 64 + lane];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

__global__ void probe(const double* src, double* out, int off) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  double* slot = reinterpret_cast<double*>(smem + off);
  for (int f = 0; f < 9; ++f) slot[f * 64 + lane] = -1.0;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const char* s = reinterpret_cast<const char*>(src);
  char* d = reinterpret_cast<char*>(slot);
  if (lane % 3 == 1) {  // (a third of the lanes enabled: the DMA must still move all 64 parts)
    for (int c = 0; c < 4; ++c) lds_dma16(d + c * 1024, s + c * 1024);
    lds_dma4(d + 4096, s + 4096);
    lds_dma4(d + 4352, s + 4352);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int f = 0; f < 9; ++f) out[f * 64 + lane] = slot[f * 64 + lane];
  out[9 * 64 + lane] = (double)(unsigned)(uintptr_t)slot;
}

int main() {
  const int offs[] = {0, 4096, 60000 & ~15, 65536, 70000 & ~15, 126976, 155648};
  std::vector<double> h(576);
  for (int i = 0; i < 576; ++i) h[i] = 1000.0 + i;
  double *src, *out;
  if (hipMalloc(&src, 576 * 8) || hipMalloc(&out, 640 * 8)) return 2;
  hipMemcpy(src, h.data(), 576 * 8, hipMemcpyHostToDevice);
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  int bad_total = 0;
  for (int off : offs) {
    hipMemset(out, 0, 640 * 8);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 160 * 1024, 0, src, out, off);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
    std::vector<double> o(640);
    hipMemcpy(o.data(), out, 640 * 8, hipMemcpyDeviceToHost);
    int bad = 0, first = -1;
    for (int i = 0; i < 576; ++i)
      if (o[i] != h[i]) { ++bad; if (first < 0) first = i; }
    printf("offset %6d (slot address low bits %.0f): %d of 576 wrong%s", off, o[576], bad,
           bad ? "" : "\n");
    if (bad) printf(", first [%d] = %.1f (want %.1f)\n", first, o[first], h[first]);
    bad_total += bad;
  }
  {
    double* buf;
    double* o2;
    if (hipMalloc(&buf, 576 * 8) || hipMalloc(&o2, 1152 * 8)) return 2;
    (void)hipFuncSetAttribute((const void*)probe_st, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    hipLaunchKernelGGL(probe_st, dim3(1), dim3(64), 160 * 1024, 0, buf, o2, 126976);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
    std::vector<double> o(1152);
    (void)hipMemcpy(o.data(), o2, 1152 * 8, hipMemcpyDeviceToHost);
    for (int r = 0; r < 2; ++r) {
      int bad = 0, first = -1;
      for (int i = 0; i < 576; ++i)
        if (o[r * 576 + i] != r * 10000.0 + i) { ++bad; if (first < 0) first = i; }
      printf("store->DMA round %d: %d of 576 wrong", r, bad);
      if (bad) printf(", first [%d] = %.1f (want %.1f)", first, o[r * 576 + first], r * 10000.0 + first);
      printf("\n");
      bad_total += bad;
    }
  }
  return bad_total ? 1 : 0;
}
