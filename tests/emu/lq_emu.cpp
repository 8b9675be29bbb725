// Driver of the host emulation of zmpc_strict_lq_kernel (tests/test_lq_emulation.py): one strict
// rollout of one walk (both axes: the one-wave-per-workgroup instance, one wave per axis) from a
// binary input file through the kernel's own run-length staging, free-tail table and LQ
// kernel source; the history to stdout.  argv[2]: "runs" (run-length bounds, default) or "rows".
// Every lane of the wave runs a copy of the walk: the emulation's lockstep shuffles need
// wave-uniform control flow, and lanes that diverge (a lane outside `part`, one that has
// finished) are what only the hardware's exec masks model (the -m gpu tests).
// Input: int32 N, int64 n, f64 T, h/g, Q, R, zmax[n][2], zmin[n][2], x0[2][3], kick, int64 kick
// step (−1: none).  Test infrastructure only.
#include "hip/hip_runtime.h"

#ifndef EMU_STACK_SHIFT  // log2 of each lane's coroutine stack
#define EMU_STACK_SHIFT 20
#endif

EmuDim3 threadIdx, blockIdx;
uint64_t emu_buf[64];
static ucontext_t g_main, g_lane[64];
static int g_cur;
static bool g_done[64];
void emu_yield() { swapcontext(&g_lane[g_cur], &g_main); }

#include "lq_kernel_emu.h"  // generated from csrc/strict_lq.hip (device part)

namespace emu {
alignas(16) unsigned char lq_smem[160 * 1024];
}

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static emu::LqArgs g_args;
static const double* g_tab;
static bool g_runs = true;
static void lane_main() {
  if (g_runs)
    emu::zmpc_strict_lq_kernel<8, 1, false, true, false>(g_args, g_tab);
  else
    emu::zmpc_strict_lq_kernel<8, 1, false, false, false>(g_args, g_tab);
  g_done[g_cur] = true;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  if (argc > 2) g_runs = strcmp(argv[2], "rows") != 0;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int N = 0;
  long n = 0;
  double T, hg, Q, R, kickv = 0;
  long kstep = -1;
  bool ok = fread(&N, 4, 1, f) == 1 && fread(&n, 8, 1, f) == 1 && fread(&T, 8, 1, f) == 1 &&
            fread(&hg, 8, 1, f) == 1 && fread(&Q, 8, 1, f) == 1 && fread(&R, 8, 1, f) == 1;
  std::vector<double> zx(n * 2), zn(n * 2), x0(6), hist(64 * n * 6);
  ok = ok && fread(zx.data(), 8, n * 2, f) == (size_t)n * 2 &&
       fread(zn.data(), 8, n * 2, f) == (size_t)n * 2 && fread(x0.data(), 8, 6, f) == 6 &&
       fread(&kickv, 8, 1, f) == 1 && fread(&kstep, 8, 1, f) == 1;
  fclose(f);
  if (!ok || N < 1 || N > 2560 || n < 2) return 2;
  zmpc_plan p;
  p.N = N;
  p.T = T;
  p.T2_2 = T * T / 2;
  p.T3_6 = T * T * T / 6;
  p.hg = hg;
  p.Q = Q;
  p.R = R;
  emu::LqArgs& a = g_args;
  emu::fill_consts(&p, a);
  a.cnt = nullptr;
  // LDS checkpoints per wave (the kernel's default at N = 150: 2); LQ_EMU_NLCK overrides
  a.nlck = getenv("LQ_EMU_NLCK") ? atoi(getenv("LQ_EMU_NLCK")) : emu::kLdsCk;
  if (emu::lq_lds_bytes(1, N, a.nlck) > sizeof(emu::lq_smem)) return 3;
  // the plan's free-tail table (one thread)
  std::vector<double> tab((size_t)N * 16);
  threadIdx.x = 0;
  blockIdx.x = blockIdx.y = 0;
  emu::zmpc_strict_lq_table_kernel(a, tab.data());
  g_tab = tab.data();
  // 64 copies of the walk (one 64-walk group), bounds staged for both axes
  constexpr int kB = 64;
  std::vector<double> zx64((size_t)kB * n * 2), zn64((size_t)kB * n * 2), x064(kB * 6),
      kick64(kB, kickv);
  for (int b = 0; b < kB; ++b) {
    std::memcpy(&zx64[(size_t)b * n * 2], zx.data(), sizeof(double) * n * 2);
    std::memcpy(&zn64[(size_t)b * n * 2], zn.data(), sizeof(double) * n * 2);
    std::memcpy(&x064[b * 6], x0.data(), sizeof(double) * 6);
  }
  a.window_mode = 0;
  a.toff = 1;
  a.n = n;
  a.nsteps = n - 1;
  a.B = kB;
  a.shared = 0;
  a.groups = 1;
  a.rows = n + (int64_t)a.NS * 8;
  a.rstride = (n + 2) * 64;
  std::vector<double2> stage(g_runs ? 2 * a.rstride : 2 * a.rows * 64);
  std::vector<int> rt(g_runs ? 2 * a.rstride : 1);
  emu::StageArgs sa{zx64.data(), zn64.data(), 2 * n, 2, 1, n, kB, 1, a.rows, 2, nullptr,
                    stage.data()};
  if (g_runs) {
    for (unsigned ax = 0; ax < 2; ++ax)
      for (int l = 0; l < 64; ++l) {
        blockIdx.x = 0;
        blockIdx.y = ax;
        threadIdx.x = l;
        emu::zmpc_runs_stage_kernel(sa, stage.data(), rt.data(), a.rstride);
      }
    a.rs = stage.data();
    a.rt = rt.data();
  } else {
    // rows: [axis][group][row][64] (z_ref, half-width), rows past n − 1 the last sample
    for (int ax = 0; ax < 2; ++ax)
      for (int64_t t = 0; t < a.rows; ++t)
        for (int l = 0; l < 64; ++l) {
          const int64_t ts = t < n ? t : n - 1;
          const double hi = zx[ts * 2 + ax], lo = zn[ts * 2 + ax];
          stage[((size_t)ax * a.rows + t) * 64 + l] = double2{(hi + lo) / 2, (hi - lo) / 2};
        }
    a.hl = stage.data();
  }
  a.x0 = x064.data();
  a.kick = kstep >= 0 ? kick64.data() : nullptr;
  a.kick_step = kstep;
  a.kick_steps = nullptr;
  a.perm = nullptr;
  a.out = hist.data();
  std::vector<int32_t> status(kB, 0);
  a.status = status.data();
  std::vector<double> ck((size_t)2 * a.NS * 9 * 64);
  a.ck = ck.data();
  a.queue = nullptr;
  a.prof = nullptr;
  std::vector<char> stacks((size_t)64 << EMU_STACK_SHIFT);
  for (unsigned w = 0; w < 2; ++w) {  // task w: axis w of the walk (G = 1: task = block)
    blockIdx.x = w;
    blockIdx.y = 0;
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
  // every copy must equal the first (the same walk on every lane)
  int st = 0, same = 1;
  for (int b = 0; b < kB; ++b) {
    st |= status[b];
    same &= std::memcmp(&hist[(size_t)b * n * 6], hist.data(), sizeof(double) * n * 6) == 0;
  }
  fwrite(hist.data(), 8, n * 6, stdout);
  fprintf(stderr, "lanes %s\nstatus %d\n", same ? "equal" : "DIFFER", st);
  return 0;
}
