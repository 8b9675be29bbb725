// Host emulation of the few HIP device facilities the strict kernels use (strict_scan.hip,
// strict_lq.hip), for the CPU tests of their wave-level logic (tests/test_scan_emulation.py,
// tests/test_lq_emulation.py).  Test infrastructure only.
// One wave = 64 lanes run as stackful coroutines (ucontext) in one thread; every cross-lane
// operation (shuffles, __any) is a lockstep point: each lane publishes its value and yields,
// and reads once every lane has published.  Correct for kernels whose cross-lane operations
// sit in wave-uniform control flow, as the kernel's do.
#pragma once
#include <ucontext.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <cstdlib>
using std::fabs;
using std::fma;
using std::isfinite;
using std::max;
using std::min;
#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __launch_bounds__(...)
typedef int hipError_t;
typedef void* hipStream_t;
typedef void* hipEvent_t;
enum { hipSuccess = 0, hipErrorInvalidValue = 1, hipErrorOutOfMemory = 2 };
struct EmuDim3 {
  unsigned x = 0, y = 0, z = 0;
};
extern EmuDim3 threadIdx, blockIdx;
extern uint64_t emu_buf[64];
void emu_yield();
inline double __builtin_amdgcn_rcp(double x) { return 1.0 / x; }
template <class T>
inline T emu_xchg(T v, int src) {
  uint64_t u = 0;
  std::memcpy(&u, &v, sizeof(T));
  emu_buf[threadIdx.x] = u;
  emu_yield();
  const uint64_t r = emu_buf[src];
  emu_yield();
  T o;
  std::memcpy(&o, &r, sizeof(T));
  return o;
}
template <class T>
inline T __shfl_down(T v, int d, int = 64) {
  const int l = (int)threadIdx.x;
  return emu_xchg(v, l + d < 64 ? l + d : l);
}
template <class T>
inline T __shfl_up(T v, int d, int = 64) {
  const int l = (int)threadIdx.x;
  return emu_xchg(v, l >= d ? l - d : l);
}
template <class T>
inline T __shfl_xor(T v, int m, int = 64) {
  return emu_xchg(v, (int)threadIdx.x ^ m);
}
template <class T>
inline T __shfl(T v, int s, int = 64) {
  return emu_xchg(v, s);
}
inline int __double2loint(double v) {
  uint64_t u;
  std::memcpy(&u, &v, 8);
  return (int)(uint32_t)u;
}
inline int __double2hiint(double v) {
  uint64_t u;
  std::memcpy(&u, &v, 8);
  return (int)(uint32_t)(u >> 32);
}
inline double __hiloint2double(int hi, int lo) {
  const uint64_t u = ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
  double v;
  std::memcpy(&v, &u, 8);
  return v;
}
// DPP lane moves: row_shl:n (0x101-0x10F) and row_shr:n (0x111-0x11F) inside 16-lane rows,
// wave_shl:1 (0x130), wave_shr:1 (0x138), row_bcast:15 (0x142: row r reads lane 16r − 1) and
// row_bcast:31 (0x143: rows 2, 3 read lane 31).  Rows outside row_mask keep `old`; an invalid
// source reads 0 under bound_ctrl, else `old`.
inline int __builtin_amdgcn_update_dpp(int old, int src, int ctrl, int row_mask, int bank_mask,
                                       bool bound_ctrl) {
  const int l = (int)threadIdx.x;
  int from = -1;
  if (ctrl > 0x100 && ctrl < 0x110) {
    const int n = ctrl - 0x100;
    if ((l & 15) + n < 16) from = l + n;
  } else if (ctrl > 0x110 && ctrl < 0x120) {
    const int n = ctrl - 0x110;
    if ((l & 15) >= n) from = l - n;
  } else if (ctrl == 0x130) {
    if (l < 63) from = l + 1;
  } else if (ctrl == 0x138) {
    if (l > 0) from = l - 1;
  } else if (ctrl == 0x142) {
    if (l >= 16) from = (l & ~15) - 1;
  } else if (ctrl == 0x143) {
    if (l >= 32) from = 31;
  } else {
    std::abort();  // (a DPP control the emulation does not model)
  }
  if (bank_mask != 0xF) std::abort();
  const int v = emu_xchg(src, from >= 0 ? from : l);
  if (!((row_mask >> (l >> 4)) & 1)) return old;
  return from >= 0 ? v : (bound_ctrl ? 0 : old);
}
inline bool __any(bool b) {
  emu_buf[threadIdx.x] = b;
  emu_yield();
  bool r = false;
  for (int i = 0; i < 64; ++i) r |= emu_buf[i] != 0;
  emu_yield();
  return r;
}
inline unsigned long long __ballot(bool b) {
  emu_buf[threadIdx.x] = b;
  emu_yield();
  unsigned long long m = 0;
  for (int i = 0; i < 64; ++i) m |= (unsigned long long)(emu_buf[i] != 0) << i;
  emu_yield();
  return m;
}
inline int __popcll(unsigned long long m) { return __builtin_popcountll(m); }
inline int atomicOr(int32_t* p, int v) {
  const int o = *p;
  *p |= v;
  return o;
}
inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) {
  const auto o = *p;
  *p += v;
  return o;
}
inline unsigned long long atomicMax(unsigned long long* p, unsigned long long v) {
  const auto o = *p;
  *p = std::max(*p, v);
  return o;
}
inline int atomicAdd(int* p, int v) {
  const int o = *p;
  *p += v;
  return o;
}
// (strict_lq.hip) wave-uniform values, scheduling hints, cache policy: no-ops on the host
inline int __builtin_amdgcn_readfirstlane(int v) { return v; }
inline void __builtin_amdgcn_sched_barrier(int) {}
inline void __builtin_amdgcn_s_waitcnt(int) {}
inline void __builtin_amdgcn_s_setprio(int) {}
#define __builtin_nontemporal_store(v, p) (*(p) = (v))
#define __builtin_nontemporal_load(p) (*(p))
inline unsigned long long clock64() { return 0; }
#define __shared__
inline void __syncthreads() {}  // (the row-staging kernel, which the emulation does not run)
struct dim3 {
  unsigned x, y, z;
  dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};
struct double2 {
  double x, y;
};
inline double2 make_double2(double x, double y) { return double2{x, y}; }
#define hipLaunchKernelGGL(...) (void)0
inline hipError_t hipGetLastError() { return 0; }
inline hipError_t hipMemsetAsync(void*, int, size_t, hipStream_t) { return 0; }
