#!/bin/bash
# Round 3: Herdt pass diagnostic (lane-pair passes needed vs wave passes), config 6.
set -u
OUT=gpurun_out/r3z
mkdir -p "$OUT"
export TMPDIR=/tmp
ZMPC_HERDT_PROF=1 timeout -k 10 300 python scripts/herdt_once.py 32768 > "$OUT/herdt_prof.log" 2>&1
rc=$?; cat "$OUT/herdt_prof.log" | tail -5; exit $rc
