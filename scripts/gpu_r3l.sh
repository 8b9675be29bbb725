#!/bin/bash
# Round 3: fast-FIR default (variant 8 → one walk per workgroup for odd CW) — full GPU suite,
# config-2 A/B against the previous default (17) and the persistent fast-FIR grid (19), the
# default bench line and its rocprof kernel stats.
set -u
OUT=gpurun_out/r3l
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
for R in 1 2 3; do
for V in 8 17 19; do
  ZMPC_ROLLOUT_VARIANT=$V timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/c2_v${V}_$R.json" 2> "$OUT/c2_v${V}_$R.err" || exit $?
  python -c "import json; d=json.load(open('$OUT/c2_v${V}_$R.json')); r=d['roofline']; print('c2 v $V', '%.3e' % d['value'], '%.2f us' % (r['kernel_ms']*1e3), '%.3f' % r['frac'])"
done
done
timeout -k 10 300 python bench.py --cpu-seconds 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print('bench', '%.3e' % d['value'], '%.2f us' % (r['kernel_ms']*1e3), '%.3f' % r['frac'], r.get('kernel'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o run -- python3 bench.py --no-cpu-baseline > "$OUT/prof_c2.log" 2>&1
rc=$?; echo "prof rc=$rc"
exit $rc
