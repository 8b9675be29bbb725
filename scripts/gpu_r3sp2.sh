#!/bin/bash
# Round 3: config-2 phase ablation and kernel variants with the sparse-difference correlation
# (default.json CoP data), plus the dense reference rows.
set -u
OUT=gpurun_out/${1:-r3sp2}
mkdir -p "$OUT"
export TMPDIR=/tmp
ABL_DATA=cop timeout -k 10 400 python scripts/ablate_rollout.py 8,6,17,19,11,12 0,1,4,8,12,15 4096 > "$OUT/ablation_cop.jsonl" 2> "$OUT/ablation.err"
rc=$?; cat "$OUT/ablation_cop.jsonl"; [ $rc -ne 0 ] && exit $rc
ABL_DATA=cop timeout -k 10 300 python scripts/ablate_rollout.py 8,6,11,12 0 2048,8192,16384 > "$OUT/batch_cop.jsonl" 2>> "$OUT/ablation.err"
rc=$?; cat "$OUT/batch_cop.jsonl"; exit $rc
