#!/bin/bash
# Same-box A/B of two builds of the library on the strict bench configs: alternates
# the product library and ZMPC_LIB=<other> three times per config.
# Usage: scripts/gpu_ab.sh TAG OTHER_LIB [CONFIGS...]
set -u
T=$1; OTHER=$2; shift 2
CONFIGS=${*:-3 4}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in $CONFIGS; do
  for r in 1 2 3; do
    timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/c${c}_new_$r.json" 2> "$OUT/c${c}_new_$r.err" || exit $?
    ZMPC_LIB=$PWD/$OTHER timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/c${c}_old_$r.json" 2> "$OUT/c${c}_old_$r.err" || exit $?
    python - "$OUT/c${c}_new_$r.json" "$OUT/c${c}_old_$r.json" <<'PY'
import json, sys
n, o = (json.loads(open(p).read().strip().splitlines()[-1]) for p in sys.argv[1:])
print(f"config {n['config'].get('workload','?')[:40]}: new {n['ms_per_step']:.2f} ms  other {o['ms_per_step']:.2f} ms", flush=True)
PY
  done
done
