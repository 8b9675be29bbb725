#!/bin/bash
# Round 3: counter list, default bench + kernel stats, plan-build kernel stats, horizon sweep.
set -u
OUT=gpurun_out/r3e
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1; echo "list rc=$?"
timeout -k 10 300 python bench.py --cpu-seconds 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench.err"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run -- python3 bench.py --no-cpu-baseline > "$OUT/prof_c2.log" 2>&1
rc=$?; echo "prof c2 rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/prof_c2.log"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_plan" -o run -- python3 scripts/plan_timing.py 150 512 2048 > "$OUT/prof_plan.log" 2>&1
rc=$?; echo "prof plan rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/prof_plan.log"; exit $rc; }
timeout -k 10 600 python -u bench.py --sweep-horizon 10:300:10 > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
rc=$?; echo "sweep rc=$rc"; tail -2 "$OUT/sweep.jsonl"; [ $rc -ne 0 ] && tail -5 "$OUT/sweep.err"
exit $rc
