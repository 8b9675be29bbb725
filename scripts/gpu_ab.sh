#!/bin/bash
# A/B session: rollout parity subset, then scripts/ab_rollout.py over env variants.
# usage: bash scripts/gpu_ab.sh <tag> '<variants json>' '<shapes json>' [pytest -k expr]
set -u
TAG=$1; VARS=$2; SHAPES=$3; KEXPR=${4:-"rollout or walk or batch or config2 or shared or kick or empty"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
    --timeout 240 --timeout-method thread -k "$KEXPR" > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest_gpu.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/ab_rollout.py "$VARS" "$SHAPES" > "$OUT/ab.jsonl" 2> "$OUT/ab.err"
rc=$?; echo "ab rc=$rc"; cat "$OUT/ab.jsonl"
exit $rc
