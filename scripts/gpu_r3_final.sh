#!/bin/bash
# Round 3 closing validation: full GPU suite, smoke, config-2 profile round (kernel stats, HBM
# PMC passes, bench with traffic), the default bench line with its CPU leg, every config's line.
set -u
OUT=gpurun_out/${1:-r3fin}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_profile_round.sh ${1:-r3fin}/prof > "$OUT/prof.log" 2>&1
rc=$?; echo "profile round rc=$rc"; tail -2 "$OUT/prof.log" | cut -c1-200; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
rc=$?; echo "default bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_configs.sh ${1:-r3fin}/configs > "$OUT/configs.log" 2>&1
rc=$?; cat "$OUT/configs.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --config 6 --steps 3 --warmup 1 --cpu-seconds 5 > "$OUT/configs/config6.json" 2> "$OUT/configs/config6.err"
rc=$?; echo "config6 rc=$rc"; exit $rc
