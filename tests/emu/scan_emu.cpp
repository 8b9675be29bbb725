// Driver of the host emulation of zmpc_strict_scan_kernel (tests/test_scan_emulation.py): one
// strict rollout of one walk (both axes) from a binary input file, the history to stdout.
// argv[2]: lanes per instance (64, default, or 32).  Input: int32 N, int64 n, f64 T, h/g, Q, R, zmax[n][2], zmin[n][2], x0[2][3], kick, int64
// kick step (−1: none).  Test infrastructure only.
#include "hip/hip_runtime.h"

#ifndef EMU_STACK_SHIFT  // log2 of each lane's coroutine stack (the sanitizer build: smaller)
#define EMU_STACK_SHIFT 20
#endif

EmuDim3 threadIdx, blockIdx;
uint64_t emu_buf[64];
static ucontext_t g_main, g_lane[64];
static int g_cur;
static bool g_done[64];
void emu_yield() { swapcontext(&g_lane[g_cur], &g_main); }

#include "scan_kernel_emu.h"  // generated from csrc/strict_scan.hip (kernel part)

#include <cstdio>
#include <cstdlib>
#include <vector>

static emu::ScanArgs g_args;
static int g_L = 64;  // lanes per instance
static void lane_main() {
  if (g_L == 64) {
    switch ((g_args.N + 63) / 64) {
#define EMU_CASE(CC)                                  \
  case CC:                                            \
    emu::zmpc_strict_scan_kernel<CC, 64>(g_args); \
    break;
      EMU_CASE(1) EMU_CASE(2) EMU_CASE(3) EMU_CASE(4) EMU_CASE(5) EMU_CASE(6) EMU_CASE(7) EMU_CASE(8)
#undef EMU_CASE
      default:
        break;
    }
  } else {
    switch ((g_args.N + 31) / 32) {
#define EMU_CASE(CC)                                  \
  case CC:                                            \
    emu::zmpc_strict_scan_kernel<CC, 32>(g_args); \
    break;
      EMU_CASE(1) EMU_CASE(2) EMU_CASE(3) EMU_CASE(4) EMU_CASE(5) EMU_CASE(6) EMU_CASE(7) EMU_CASE(8)
#undef EMU_CASE
      default:
        break;
    }
  }
  g_done[g_cur] = true;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  if (argc > 2) g_L = atoi(argv[2]);
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int N = 0;
  long n = 0;
  double T, hg, Q, R, kickv = 0;
  long kstep = -1;
  bool ok = fread(&N, 4, 1, f) == 1 && fread(&n, 8, 1, f) == 1 && fread(&T, 8, 1, f) == 1 &&
            fread(&hg, 8, 1, f) == 1 && fread(&Q, 8, 1, f) == 1 && fread(&R, 8, 1, f) == 1;
  std::vector<double> zx(n * 2), zn(n * 2), x0(6), hist(n * 6);
  ok = ok && fread(zx.data(), 8, n * 2, f) == (size_t)n * 2 &&
       fread(zn.data(), 8, n * 2, f) == (size_t)n * 2 && fread(x0.data(), 8, 6, f) == 6 &&
       fread(&kickv, 8, 1, f) == 1 && fread(&kstep, 8, 1, f) == 1;
  fclose(f);
  if (!ok || N < 1 || N > 512) return 2;
  emu::ScanArgs& a = g_args;
  // the constants as strict_scan.hip's fill() forms them from a plan
  a.N = N;
  emu::fill_consts(a, T, T * T / 2, T * T * T / 6, hg, Q, R);
  a.window_mode = 0;
  a.toff = 1;
  a.n = n;
  a.nsteps = n - 1;
  a.ninst = 2;
  a.zmax = zx.data();
  a.zmin = zn.data();
  a.bstride = 0;
  a.x0 = x0.data();
  a.kick = kstep >= 0 ? &kickv : nullptr;
  a.kick_step = kstep;
  a.out = hist.data();
  int32_t status = 0;
  a.status = &status;
  a.cnt = nullptr;
  std::vector<char> stacks((size_t)64 << EMU_STACK_SHIFT);
  const unsigned waves = g_L == 64 ? 2 : 1;  // the walk's two (walk, axis) instances
  for (unsigned w = 0; w < waves; ++w) {
    blockIdx.x = w;
    for (int l = 0; l < 64; ++l) {
      getcontext(&g_lane[l]);
      g_lane[l].uc_stack.ss_sp = stacks.data() + ((size_t)l << EMU_STACK_SHIFT);
      g_lane[l].uc_stack.ss_size = (size_t)1 << EMU_STACK_SHIFT;
      g_lane[l].uc_link = &g_main;
      g_done[l] = false;
      makecontext(&g_lane[l], lane_main, 0);
    }
    for (bool any = true; any;) {
      any = false;
      for (int l = 0; l < 64; ++l) {
        if (g_done[l]) continue;
        g_cur = l;
        threadIdx.x = l;
        swapcontext(&g_main, &g_lane[l]);
        any = true;
      }
    }
  }
  fwrite(hist.data(), 8, n * 6, stdout);
  fprintf(stderr, "status %d\n", status);
  return 0;
}
