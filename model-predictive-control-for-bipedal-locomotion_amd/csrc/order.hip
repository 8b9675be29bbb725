// Walk order for the lane-per-instance active-set kernels (strict_lq.hip).
//
// A wave runs its 64 lanes in lockstep: every active-set pass runs until the wave's slowest lane
// has converged, and the working-set part of a pass extends to the wave's last active slot.
// How much of the horizon is active, and for how long, follows mostly from the disturbance a walk
// takes — the force kick of zmp_controller.py:90,105-106 (the F_ext sweep of
// run_compare_resistance.py:87-169).  Walks handed over in arbitrary order mix light and heavy
// kicks in every wave, so every wave pays for its heaviest lane.  Sorting the walks by
// (kick step, kick) before they are mapped to lanes puts walks with similar disturbances into the
// same wave: the results are unchanged (each lane's arithmetic depends on its own walk only),
// only the schedule is.  Config 4 (125 000 shared-CoP scenarios, F uniform in [0, 800] N):
// 141.9 → 108.4 ms (profiles/r3s2/).
#include <hipcub/hipcub.hpp>

#include "zmpc_internal.h"

namespace {

// Sort key: kick step (−1: none) in the high word, the kick as an order-preserving 32-bit image
// of its float value in the low word (a scheduling key, so float precision is plenty).
__global__ void __launch_bounds__(256) zmpc_kick_key_kernel(const double* __restrict__ kick,
                                                            const int64_t* __restrict__ ksteps,
                                                            int64_t kstep, int64_t B,
                                                            unsigned long long* keys,
                                                            int32_t* idx) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const int64_t ks = ksteps ? ksteps[b] : kstep;
  const unsigned hi = (unsigned)(ks < 0 ? 0 : (ks >= 0x7fffffff ? 0x7fffffff : ks + 1));
  const float kf = (float)kick[b];
  unsigned u = __float_as_uint(kf == 0.0f ? 0.0f : kf);  // −0 → +0
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);       // IEEE order → unsigned order
  keys[b] = ((unsigned long long)hi << 32) | u;
  idx[b] = (int32_t)b;
}

}  // namespace

size_t zmpc_kick_order_bytes(int64_t B) {
  size_t tmp = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const unsigned long long*)nullptr,
                                           (unsigned long long*)nullptr, (const int32_t*)nullptr,
                                           (int32_t*)nullptr, (int)B);
  // keys in/out [B] u64, values in [B] i32 (perm is the caller's), sort temporaries
  return (size_t)B * 16 + (size_t)B * 4 + tmp + 256;
}

hipError_t zmpc_kick_order(const double* kick, const int64_t* kick_steps, int64_t kick_step,
                           int64_t B, int32_t* perm, void* ws, hipStream_t s) {
  size_t tmp = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(
      nullptr, tmp, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
      (const int32_t*)nullptr, (int32_t*)nullptr, (int)B);
  if (e != hipSuccess) return e;
  unsigned char* p = static_cast<unsigned char*>(ws);
  auto* kin = reinterpret_cast<unsigned long long*>(p);
  auto* kout = kin + B;
  auto* iin = reinterpret_cast<int32_t*>(kout + B);
  void* t = reinterpret_cast<void*>(((uintptr_t)(iin + B) + 255) & ~(uintptr_t)255);
  hipLaunchKernelGGL(zmpc_kick_key_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s,
                     kick, kick_steps, kick_step, B, kin, iin);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return hipcub::DeviceRadixSort::SortPairs(t, tmp, kin, kout, iin, perm, (int)B, 0, 64, s);
}
