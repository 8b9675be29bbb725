#!/bin/bash
# Round 3: counter tests (ABI 6) + config-2 kernel time vs batch (ramp vs steady state).
set -u
OUT=gpurun_out/r3s
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_herdt.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "counters" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python scripts/ablate_rollout.py 8 0,12 1024,2048,3072,4096,6144,8192,16384 > "$OUT/batch.jsonl" 2>&1 || exit $?
cat "$OUT/batch.jsonl"
