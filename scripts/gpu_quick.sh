#!/bin/bash
# Quick iteration: GPU parity tests, rollout ablation, bench (no profiler).
set -u
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -15 "$OUT/pytest_gpu.log"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python scripts/ablate_rollout.py > "$OUT/ablate.jsonl" 2> "$OUT/ablate.err"
rc=$?; echo "ablate rc=$rc"; cat "$OUT/ablate.jsonl"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --cpu-seconds 3 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"

[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --strict --batch ${STRICT_B:-8192} --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_strict.json" 2> "$OUT/bench_strict.err"
rc=$?; echo "bench strict rc=$rc"; cat "$OUT/bench_strict.json"; tail -3 "$OUT/bench_strict.err"
exit $rc
