#!/bin/bash
# Strict checkpoint policy A/B with the kick-ordered lanes and the round-3 warm start:
# config 4 (shared CoP; default cached) vs ZMPC_STRICT_NT=1, config 3 (default NT) vs =0.
set -u
OUT=gpurun_out/${1:-r3nt}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do
  for c in 4 3; do
    for m in auto 0 1; do
      if [ "$m" = auto ]; then unset ZMPC_STRICT_NT; else export ZMPC_STRICT_NT=$m; fi
      timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline \
        > "$OUT/c${c}_nt${m}_$i.json" 2> "$OUT/c${c}_nt${m}_$i.err"
      rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c${c}_nt${m}_$i.err"; exit $rc; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], r['kernel_ms'])" "$OUT/c${c}_nt${m}_$i.json"
    done
  done
done
