// Sanitizer driver of oracle/strict_lq_cpu.c (tests/test_sanitizers.py, test infrastructure
// only): one strict rollout of B walks of a shared CoP from a binary input file, the history to
// stdout, built with -fsanitize=address,undefined together with the restatement.
// Input: int32 N, int64 n, int64 B, f64 T, h/g, Q, R, zmax[n][2], zmin[n][2], x0[B][2][3],
// kick[B], int64 kick step.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int zmpc_cpu_strict_rollout(int64_t B, int64_t n, int N, double T, double T2_2, double T3_6,
                            double hg, double Q, double R, const double* zmax,
                            const double* zmin, int64_t bstride, const double* x0,
                            const double* kick, int64_t kick_step, double* hist,
                            int32_t* status, uint64_t* passes, int threads);

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int32_t N = 0;
  int64_t n = 0, B = 0, ks = -1;
  double T, hg, Q, R;
  int ok = fread(&N, 4, 1, f) == 1 && fread(&n, 8, 1, f) == 1 && fread(&B, 8, 1, f) == 1 &&
           fread(&T, 8, 1, f) == 1 && fread(&hg, 8, 1, f) == 1 && fread(&Q, 8, 1, f) == 1 &&
           fread(&R, 8, 1, f) == 1;
  if (!ok || n < 1 || B < 1 || N < 1) return 2;
  double* zx = malloc(sizeof(double) * n * 2);
  double* zn = malloc(sizeof(double) * n * 2);
  double* x0 = malloc(sizeof(double) * B * 6);
  double* kick = malloc(sizeof(double) * B);
  double* hist = malloc(sizeof(double) * B * n * 6);
  int32_t* st = malloc(sizeof(int32_t) * B);
  uint64_t* ps = malloc(sizeof(uint64_t) * B);
  ok = fread(zx, 8, n * 2, f) == (size_t)(n * 2) && fread(zn, 8, n * 2, f) == (size_t)(n * 2) &&
       fread(x0, 8, B * 6, f) == (size_t)(B * 6) && fread(kick, 8, B, f) == (size_t)B &&
       fread(&ks, 8, 1, f) == 1;
  fclose(f);
  if (!ok) return 2;
  const int rc = zmpc_cpu_strict_rollout(B, n, N, T, T * T / 2, T * T * T / 6, hg, Q, R, zx, zn,
                                         0, x0, kick, ks, hist, st, ps, 2);
  int bad = 0;
  for (int64_t b = 0; b < B; ++b) bad |= st[b];
  fwrite(hist, 8, B * n * 6, stdout);
  fprintf(stderr, "rc %d status %d\n", rc, bad);
  free(zx);
  free(zn);
  free(x0);
  free(kick);
  free(hist);
  free(st);
  free(ps);
  return rc != 0;
}
