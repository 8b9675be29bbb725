#!/bin/bash
# Round 3: pipelined persistent kernel (variant 21, table pointers opaque per walk, replay
# indices laundered) vs the default (new build) vs the default of the base build.
set -u
OUT=gpurun_out/r3x
mkdir -p "$OUT"
export TMPDIR=/tmp
D=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "variants_agree or fast_fir" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for R in 1 2 3; do
  ZMPC_LIB=$D/libzmpc_base.so timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/c2_base_$R.json" 2> "$OUT/c2_base_$R.err" || exit $?
  python -c "import json; d=json.load(open('$OUT/c2_base_$R.json')); r=d['roofline']; print('c2 base v8', '%.3e' % d['value'], '%.2f us' % (r['kernel_ms']*1e3))"
  for V in 8 21; do
    ZMPC_ROLLOUT_VARIANT=$V timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/c2_v${V}_$R.json" 2> "$OUT/c2_v${V}_$R.err" || exit $?
    python -c "import json; d=json.load(open('$OUT/c2_v${V}_$R.json')); r=d['roofline']; print('c2 new v$V', '%.3e' % d['value'], '%.2f us' % (r['kernel_ms']*1e3))"
  done
done
timeout -k 10 600 python scripts/ablate_rollout.py 21,8 0,12 4096,8192 > "$OUT/ablation.jsonl" 2>&1 || exit $?
cat "$OUT/ablation.jsonl"
