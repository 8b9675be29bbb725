#!/bin/bash
# All SURVEY §8d single-GPU workloads through bench.py (one JSON line each).
set -u
OUT=gpurun_out/${1:-configs}
mkdir -p "$OUT"
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python3 bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/$name.err"; exit $rc; }
  return 0
}
run config2 300 --config 2
run config5 300 --config 5 --steps 5 --warmup 1 --cpu-seconds 5
run config4_unc 300 --config 4 --unconstrained --steps 3 --warmup 1 --cpu-seconds 5
run config3 400 --config 3 --steps 2 --warmup 1 --cpu-seconds 5
run config4 400 --config 4 --steps 1 --warmup 1 --cpu-seconds 5
echo done
