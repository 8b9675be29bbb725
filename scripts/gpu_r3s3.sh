#!/bin/bash
# Round 3: lean selects in sweep A + kick order (order.hip): strict GPU tests, configs 3 / 4
# bench lines with and without the order (ZMPC_STRICT_ORDER=0).
set -u
OUT=gpurun_out/r3s3
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "strict" --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_strict.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_strict.log"; [ $rc -ne 0 ] && exit $rc
for o in 1 0; do
  for c in 4 3; do
    ZMPC_STRICT_ORDER=$o timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c${c}_o${o}.json" 2> "$OUT/bench_c${c}_o${o}.err"
    rc=$?; echo "c$c o$o rc=$rc"; cut -c1-200 "$OUT/bench_c${c}_o${o}.json"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
