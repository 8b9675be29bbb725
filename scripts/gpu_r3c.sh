#!/bin/bash
# Round 3: plan timings, full GPU suite, strict LQ window-traffic diagnostic.
set -u
OUT=gpurun_out/r3c
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/plan_timing.py > "$OUT/plan_timing.jsonl" 2>&1
rc=$?; echo "plan rc=$rc"; cat "$OUT/plan_timing.jsonl"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest_gpu.log"; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20
case $rc in 0|1) ;; *) exit $rc;; esac
for D in 0 1; do
  ZMPC_DEBUG_LQ=$D timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c3_dbg$D.json" 2> "$OUT/c3_dbg$D.err"
  rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c3_dbg$D.err"; exit $rc; }
  python -c "import json; d=json.load(open('$OUT/c3_dbg$D.json')); print('dbg $D', '%.3e' % d['value'], d['roofline']['kernel_ms'], d['roofline']['passes_per_solve'])"
done
exit 0
