#!/bin/bash
# Round 3: fast-FIR h in LDS (variant 20) A/B + phase ablation of the default + SQ counters.
set -u
OUT=gpurun_out/r3m
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "variants_agree or config2 or controller_com" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python scripts/ablate_rollout.py 8,20,17,8,20,17 0 4096 > "$OUT/ab.jsonl" 2>&1 || exit $?
timeout -k 10 600 python scripts/ablate_rollout.py 8 1,2,4,8,12,13,15 4096 > "$OUT/ablation.jsonl" 2>&1 || exit $?
cat "$OUT/ab.jsonl" "$OUT/ablation.jsonl"
timeout -k 10 400 bash scripts/gpu_rollout_pmc.sh r3m/pmc 4096 > "$OUT/pmc.log" 2>&1
rc=$?; echo "pmc rc=$rc"; tail -40 "$OUT/pmc.log"
exit $rc
