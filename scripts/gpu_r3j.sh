#!/bin/bash
# Round 3: DPP-scan defaults — full GPU suite, config 2/4u A/B against the shuffle scan, profile.
set -u
OUT=gpurun_out/r3j
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
for V in 8 15; do
  ZMPC_ROLLOUT_VARIANT=$V timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/c2_v$V.json" 2> "$OUT/c2_v$V.err" || exit $?
  python -c "import json; d=json.load(open('$OUT/c2_v$V.json')); r=d['roofline']; print('c2 v $V', '%.3e' % d['value'], '%.2f us' % (r['kernel_ms']*1e3), '%.3f' % r['frac'])"
done
for V in 8 16; do
  ZMPC_ROLLOUT_VARIANT=$V timeout -k 10 120 python bench.py --config 4 --unconstrained --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/c4u_v$V.json" 2> "$OUT/c4u_v$V.err" || exit $?
  python -c "import json; d=json.load(open('$OUT/c4u_v$V.json')); r=d['roofline']; print('c4u v $V', '%.3e' % d['value'], '%.2f us' % (r['kernel_ms']*1e3), '%.3f' % r['frac'])"
done
timeout -k 10 300 python bench.py --cpu-seconds 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print('bench', '%.3e' % d['value'], '%.2f us' % (r['kernel_ms']*1e3), '%.3f' % r['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o run -- python3 bench.py --no-cpu-baseline > "$OUT/prof_c2.log" 2>&1
rc=$?; echo "prof rc=$rc"
exit $rc
