#!/bin/bash
# Strict LQ lane drift A/B with the round-3 warm start (config 3): ZMPC_STRICT_LQ_DRIFT 2/4/6.
set -u
OUT=gpurun_out/${1:-r3drift}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do
  for d in 4 2 6; do
    ZMPC_STRICT_LQ_DRIFT=$d timeout -k 10 300 python bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline \
      > "$OUT/c3_d${d}_$i.json" 2> "$OUT/c3_d${d}_$i.err"
    rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c3_d${d}_$i.err"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], r['kernel_ms'], r['passes_per_solve'], r['lane_efficiency'])" "$OUT/c3_d${d}_$i.json"
  done
done
