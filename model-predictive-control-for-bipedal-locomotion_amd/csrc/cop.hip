// Batched CoP-bound producer: the footstep plan and the walking phase
// machine of generators/footstep_generator.py:19-49 and generators/cop_generator.py:34-115,
// one walk per thread, for B walks with their own (distance, step_length, foot_spread, ssp,
// dsp, standing, dt).  The float clock `t += dt` decides the sample count and the transition
// samples, so every comparison and accumulation is evaluated as the reference evaluates it
// in double precision (no contraction).  Walks are ragged: the output rows [n_b, n_cap) repeat
// the walk's last sample — exactly the window padding the rollout applies (zmp_controller.py
// :81-88), so a padded walk rolls out like the unpadded one over its first n_b samples.
#include "zmpc_internal.h"

namespace {

#pragma clang fp contract(off)

constexpr double kFootHalfL = 0.11 / 2;  // footstep_generator.py:34 shape (0.11, 0.05)
constexpr double kFootHalfW = 0.05 / 2;

struct CopParams {
  double distance, step_length, foot_spread, ssp, dsp, standing, dt;
};

// x of the next step (footstep_generator.py:40-47): full steps, the last at most half a step.
__device__ __forceinline__ double advance(double x, double distance, double step) {
  const double remaining = distance - x;
  if (remaining <= step) return x + fmin(remaining, 0.5 * step);
  return x + step;
}

// Footsteps in order: (0, −s), (0, +s), the alternating steps, then the trailing foot.
struct FootIter {
  double distance, step, spread;
  double x, side;
  int k;  // index of the next foot
  bool done_loop;
  __device__ void init(const CopParams& p) {
    distance = p.distance;
    step = p.step_length;
    spread = p.foot_spread;
    x = 0.0;
    side = p.foot_spread;
    k = 0;
    done_loop = false;
  }
  __device__ void next(double* fx, double* fy) {
    if (k == 0) {
      *fx = 0.0;
      *fy = -spread;
    } else if (k == 1) {
      *fx = 0.0;
      *fy = spread;
    } else if (!done_loop && x < distance) {
      x = advance(x, distance, step);
      side = -side;
      *fx = x;
      *fy = side;
    } else {
      done_loop = true;
      *fx = x;
      *fy = -side;  // the trailing foot joins the leading one
    }
    ++k;
  }
};

__device__ int count_feet(const CopParams& p) {
  double x = 0.0;
  int n = 2;
  while (x < p.distance) {
    x = advance(x, p.distance, p.step_length);
    ++n;
  }
  return n + 1;
}

enum { ST_STANDING = 0, ST_DOUBLE = 1, ST_SINGLE = 2 };

// Runs the phase machine of cop_generator.py:71-113 for one walk; writes rows when zmax is
// not null (row stride 2, n_cap rows, padded with the last row).  Returns the sample count.
__device__ int64_t cop_walk(const CopParams& p, int64_t n_cap, double* zmax, double* zmin,
                            int8_t* states) {
  const int last = count_feet(p) - 1;
  FootIter it;
  it.init(p);
  double ax, ay, bx, by;  // feet[foot - 1], feet[foot]
  it.next(&ax, &ay);
  it.next(&bx, &by);
  int foot = 1, state = ST_STANDING;
  double t = 0.0, t_switch = p.standing;
  int64_t n = 0;
  double ux = 0, uy = 0, lx = 0, ly = 0;
  while (foot <= last) {
    if (t > t_switch) {
      double dur = 0.0;
      if (state == ST_STANDING) {
        if (foot == last) {
          foot += 1;
        } else {
          state = ST_DOUBLE;
          dur = p.dsp;
        }
      } else if (state == ST_SINGLE) {
        state = ST_DOUBLE;
        foot += 1;
        ax = bx;
        ay = by;
        it.next(&bx, &by);
        dur = p.dsp;
      } else {  // double support
        if (foot == last) {
          state = ST_STANDING;
          dur = p.standing;
        } else {
          state = ST_SINGLE;
          dur = p.ssp;
        }
      }
      t_switch += dur;
    }
    if (foot <= last) {
      if (state == ST_SINGLE) {
        ux = bx + kFootHalfL;
        uy = by + kFootHalfW;
        lx = bx - kFootHalfL;
        ly = by - kFootHalfW;
      } else {
        ux = fmax(ax + kFootHalfL, bx + kFootHalfL);
        uy = fmax(ay + kFootHalfW, by + kFootHalfW);
        lx = fmin(ax - kFootHalfL, bx - kFootHalfL);
        ly = fmin(ay - kFootHalfW, by - kFootHalfW);
      }
      if (zmax != nullptr && n < n_cap) {
        zmax[2 * n] = ux;
        zmax[2 * n + 1] = uy;
        zmin[2 * n] = lx;
        zmin[2 * n + 1] = ly;
        if (states) states[n] = (int8_t)state;
      }
      ++n;
    }
    t += p.dt;
  }
  if (zmax != nullptr)
    for (int64_t r = n; r < n_cap; ++r) {
      zmax[2 * r] = ux;
      zmax[2 * r + 1] = uy;
      zmin[2 * r] = lx;
      zmin[2 * r + 1] = ly;
      if (states) states[r] = -1;
    }
  return n;
}

__global__ void zmpc_cop_kernel(int64_t B, const double* __restrict__ params, int64_t n_cap,
                                double* __restrict__ zmax, double* __restrict__ zmin,
                                int8_t* __restrict__ states, int64_t* __restrict__ n_out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double* q = params + b * 7;
  const CopParams p{q[0], q[1], q[2], q[3], q[4], q[5], q[6]};
  const int64_t n = cop_walk(p, n_cap, zmax ? zmax + b * n_cap * 2 : nullptr,
                             zmin ? zmin + b * n_cap * 2 : nullptr,
                             states ? states + b * n_cap : nullptr);
  if (n_out) n_out[b] = n;
}

}  // namespace

hipError_t zmpc_launch_cop(int64_t B, const double* params, int64_t n_cap, double* zmax,
                           double* zmin, int8_t* states, int64_t* n_out, hipStream_t s) {
  if (B == 0) return hipSuccess;
  hipLaunchKernelGGL(zmpc_cop_kernel, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, s, B,
                     params, n_cap, zmax, zmin, states, n_out);
  return hipGetLastError();
}
