#!/bin/bash
# Strict path: GPU tests, config 3/4 bench lines, then the config-3 profile (stats + PMC).
# Usage: bash scripts/gpu_strict_round.sh <tag> [noprof]     outputs under gpurun_out/<tag>/
set -u
TAG=${1:-sround}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for C in 3 4; do
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c$C.json" 2> "$OUT/c$C.err"
  rc=$?; if [ $rc -ne 0 ]; then tail -5 "$OUT/c$C.err"; exit $rc; fi
  python -c "import json; d=json.load(open('$OUT/c$C.json')); r=d['roofline']; print('config $C', '%.3e' % d['value'], '%.2f ms' % r['kernel_ms'], 'frac %.3f' % r['frac'], 'pps %.3f' % r['passes_per_solve'], 'lane_eff %.3f' % r['lane_efficiency'], 'ws %.3f' % r['working_set_slot_frac'])"
done
[ "${2:-}" = noprof ] && exit 0
bash scripts/gpu_strict_prof.sh "$TAG/prof" 3
