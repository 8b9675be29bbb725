#!/bin/bash
# Same-box A/B/n of library builds on bench configs: the product library and each ZMPC_LIB
# given, alternated three times per config.
# Usage: scripts/gpu_abn.sh TAG "CONFIGS" LIB...
set -u
T=$1; CONFIGS=$2; shift 2
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in $CONFIGS; do
  for r in 1 2 3; do
    line="config $c run $r: product"
    timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/c${c}_product_$r.json" 2> "$OUT/c${c}_product_$r.err" || exit $?
    line="$line $(python -c "import json,sys;print('%.2f'%json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['ms_per_step'])" "$OUT/c${c}_product_$r.json")"
    for lib in "$@"; do
      b=$(basename "$lib" .so)
      ZMPC_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/c${c}_${b}_$r.json" 2> "$OUT/c${c}_${b}_$r.err" || exit $?
      line="$line | $b $(python -c "import json,sys;print('%.2f'%json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['ms_per_step'])" "$OUT/c${c}_${b}_$r.json")"
    done
    echo "$line"
  done
done
