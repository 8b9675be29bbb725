#!/bin/bash
# Round 3: multi-rank bench rehearsal on one GPU (2 ranks, gloo) + config 4/5 bench lines.
set -u
OUT=gpurun_out/r3h
mkdir -p "$OUT"
export TMPDIR=/tmp
env -u WORLD_SIZE timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_2rank_gloo.json" 2> "$OUT/bench_2rank_gloo.err"
rc=$?; echo "2-rank rc=$rc"; cat "$OUT/bench_2rank_gloo.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_2rank_gloo.err"; exit $rc; }
timeout -k 10 300 python bench.py --config 4 --unconstrained --cpu-seconds 3 > "$OUT/bench_c4u.json" 2> "$OUT/bench_c4u.err"
rc=$?; echo "c4u rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_c4u.err"; exit $rc; }
timeout -k 10 300 python bench.py --config 5 --cpu-seconds 3 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
rc=$?; echo "c5 rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_c5.err"; exit $rc; }
timeout -k 10 300 python bench.py --config 3 --cpu-seconds 3 --steps 5 --warmup 1 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
rc=$?; echo "c3 rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_c3.err"; exit $rc; }
timeout -k 10 300 python bench.py --config 6 --cpu-seconds 3 --steps 5 --warmup 1 > "$OUT/bench_c6.json" 2> "$OUT/bench_c6.err"
rc=$?; echo "c6 rc=$rc"; [ $rc -ne 0 ] && tail -5 "$OUT/bench_c6.err"
for f in c4u c5 c3 c6; do python -c "import json; d=json.load(open('$OUT/bench_$f.json')); r=d['roofline']; print('$f', '%.3e' % d['value'], '%.4f ms' % r['kernel_ms'], r['unit'], '%.3f' % r['frac'])"; done
exit $rc
