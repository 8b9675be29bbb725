#!/bin/bash
# Round-2 measurement session: smoke, config 2 (default) bench, config 6 (Herdt) bench with
# its CPU leg, then rocprofv3 kernel stats of both.  Each GPU step has its own time limit.
set -u
OUT=gpurun_out/${1:-r2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > "$OUT/bench_config2.json" 2> "$OUT/bench_config2.err"
rc=$?; echo "bench2 rc=$rc"; cat "$OUT/bench_config2.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_config2.err"; exit $rc; }
timeout -k 10 600 python bench.py --config 6 --steps 5 --warmup 1 --cpu-seconds 8 > "$OUT/bench_config6.json" 2> "$OUT/bench_config6.err"
rc=$?; echo "bench6 rc=$rc"; cat "$OUT/bench_config6.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_config6.err"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof6" -o run -- \
    python3 bench.py --config 6 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/prof6.json" 2> "$OUT/prof6.err"
rc=$?; echo "prof6 rc=$rc"
exit $rc
