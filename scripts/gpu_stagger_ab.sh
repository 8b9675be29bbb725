#!/bin/bash
# A/B of the persistent config-2 kernel's scheduling knobs (ZMPC_PERS_STAGGER "units,mode,dyn":
# mode bit 16 = priority hand-off after each walk, bit 15 (+dyn) = per-XCD dynamic walk queue).
set -u
OUT=gpurun_out/${1:-stagger}
mkdir -p "$OUT"
V='[{}, {"ZMPC_PERS_STAGGER": "0,65536,0"}, {"ZMPC_PERS_STAGGER": "0,32768,1"}, {"ZMPC_PERS_STAGGER": "0,98304,1"}]'
timeout -k 10 300 python3 scripts/ab_rollout.py "$V" '[[4096, 150, 420], [6144, 150, 420]]' > "$OUT/ab.jsonl" 2> "$OUT/ab.err"
rc=$?; cat "$OUT/ab.jsonl"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 scripts/pers_trace.py "$OUT/trace" "$V" 4096
