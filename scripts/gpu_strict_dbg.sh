#!/bin/bash
# Strict-kernel diagnostics: phase cycle counters (ZMPC_DEBUG_STRICT) + timing.
set -u
TAG=${1:-sdbg}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k strict > "$OUT/pytest_strict.log" 2>&1
rc=$?; echo "pytest strict rc=$rc"; tail -3 "$OUT/pytest_strict.log"
case $rc in 0|1) ;; *) exit $rc;; esac
for B in 2048; do
  ZMPC_DEBUG_STRICT=1 timeout -k 10 300 python bench.py --strict --batch $B --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/dbg_$B.json" 2> "$OUT/dbg_$B.err"
  rc=$?; echo "dbg B=$B rc=$rc"; grep "zmpc strict dbg" "$OUT/dbg_$B.err"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python bench.py --strict --batch 8192 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_strict.json" 2> "$OUT/bench_strict.err"
rc=$?; echo "bench strict rc=$rc"; python -c "import json;d=json.load(open('$OUT/bench_strict.json'));print(d['value'], d['roofline']['kernel_ms'])"
exit $rc
