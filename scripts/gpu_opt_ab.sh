#!/bin/bash
# Same-box A/B of two bench variants of one config, alternated three times.
# Usage: scripts/gpu_opt_ab.sh TAG CONFIG "A: env/bench args" "B: env/bench args"
#   e.g. scripts/gpu_opt_ab.sh r5l 4 "" "--option strict_bounds=2"
#        (a leading VAR=value word is exported for that run only)
set -u
T=$1; C=$2; A=$3; B=$4
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, spec
  local env=() args=()
  for w in $2; do if [[ "$w" == *=* && "$w" != --* && ${#args[@]} -eq 0 ]]; then env+=("$w"); else args+=("$w"); fi; done
  env "${env[@]}" timeout -k 10 300 python bench.py --config "$C" --steps 5 --warmup 2 --no-cpu-baseline "${args[@]}" > "$OUT/c${C}_$1.json" 2> "$OUT/c${C}_$1.err"
}
for r in 1 2 3; do
  run "a$r" "$A" || exit $?
  run "b$r" "$B" || exit $?
  python - "$OUT/c${C}_a$r.json" "$OUT/c${C}_b$r.json" <<'PY'
import json, sys
a, b = (json.loads(open(p).read().strip().splitlines()[-1]) for p in sys.argv[1:])
print(f"A {a['ms_per_step']:.2f} ms   B {b['ms_per_step']:.2f} ms", flush=True)
PY
done
