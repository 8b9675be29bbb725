#!/bin/bash
# Round 3 checkpoint: full GPU suite, smoke, config-2 profile round (kernel stats, HBM PMC
# passes, bench with traffic), then every config's bench line.
set -u
OUT=gpurun_out/r3q
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_profile_round.sh r3q/prof > "$OUT/prof.log" 2>&1
rc=$?; echo "profile round rc=$rc"; tail -3 "$OUT/prof.log"; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_configs.sh r3q/configs > "$OUT/configs.log" 2>&1
rc=$?; cat "$OUT/configs.log"; exit $rc
