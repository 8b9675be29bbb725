#!/bin/bash
# Round 4 check: the tests named in $2 (pytest -k expression, optional) first, then the whole GPU
# suite, then the config-3 and default bench lines (strict baseline for the LQ rework).
set -u
OUT=gpurun_out/${1:-r4a}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${2:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "$2" > "$OUT/pytest_new.log" 2>&1
  rc=$?; echo "new tests rc=$rc"; tail -3 "$OUT/pytest_new.log"; [ $rc -ne 0 ] && exit $rc
fi
if [ "${3:-full}" = "full" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
rc=$?; echo "config3 rc=$rc"; cut -c1-400 "$OUT/bench_c3.json"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
rc=$?; echo "config4 rc=$rc"; cut -c1-300 "$OUT/bench_c4.json"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
rc=$?; echo "config2 rc=$rc"; cut -c1-300 "$OUT/bench_c2.json"; exit $rc
