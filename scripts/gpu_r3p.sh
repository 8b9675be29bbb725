#!/bin/bash
# Round 3: strict LQ axis diagnostic (y waves alone vs both axes).
set -u
OUT=gpurun_out/r3p
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python scripts/strict_axis_diag.py 65536 0,2,4,0,2 > "$OUT/strict_axis_diag.jsonl" 2>&1
rc=$?; cat "$OUT/strict_axis_diag.jsonl"; exit $rc
