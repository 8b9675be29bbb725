#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash / timeout / abort stops the session
# (pytest exit 1 = failing tests only, which still lets the measurement steps run).
# Usage: bash scripts/gpu_session.sh [tag]     (outputs under gpurun_out/<tag>/)
set -u
TAG=${1:-session}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
if fatal $rc; then echo "stopping after pytest rc=$rc"; exit $rc; fi

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
if [ $rc -ne 0 ]; then exit $rc; fi

timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
if [ $rc -ne 0 ]; then exit $rc; fi

timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"
find "$OUT/prof" -name "*stats*" | head -5
exit $rc
