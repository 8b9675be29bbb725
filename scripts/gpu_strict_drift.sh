#!/bin/bash
# Strict LQ: bounded-drift A/B at config-3 size (ZMPC_STRICT_LQ_DRIFT), one kernel variant.
set -u
OUT=gpurun_out/${1:-sdrift}
B=${2:-65536}
V=${3:-8x2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "strict" --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for D in 0 1 2 4 1000; do
  env ZMPC_STRICT_LQ=$V ZMPC_STRICT_LQ_DRIFT=$D timeout -k 10 300 python bench.py --config 3 --batch $B --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/d$D.json" 2> "$OUT/d$D.err"
  rc=$?; if [ $rc -ne 0 ]; then tail -5 "$OUT/d$D.err"; exit $rc; fi
  python -c "import json; d=json.load(open('$OUT/d$D.json')); print('drift $D', '%.3e' % d['value'], d['roofline']['kernel_ms'])"
  env ZMPC_STRICT_LQ=$V ZMPC_STRICT_LQ_DRIFT=$D ZMPC_DEBUG_STRICT=1 timeout -k 10 300 python scripts/strict_once.py $B > "$OUT/dbg_d$D.log" 2>&1
  rc=$?; grep "dbg" "$OUT/dbg_d$D.log" | tail -1; [ $rc -ne 0 ] && exit $rc
done
exit 0
