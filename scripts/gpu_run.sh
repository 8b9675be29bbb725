#!/bin/bash
# One runner for every GPU-box session (replaces the per-session scripts of rounds 4-5).
# Steps run in the order given, each under its own time limit; the first failing step ends the
# call (no GPU step runs after a failure, a fault or a time limit).  Output: gpurun_out/<TAG>/.
#
# Usage: bash scripts/gpu_run.sh TAG STEP [STEP ...]
#   tests[:<pytest -k expr>]           GPU tests (pytest -m gpu), one process
#   smoke                              __graft_entry__.smoke()
#   bench:<name>:<bench.py args>       one bench line -> <name>.json
#   profile:<workload>:<kernel>:<args> rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes
#                                      (scripts/gpu_profile_round.sh) -> <TAG>_<workload>/
#   ab:<other lib>:<c1,c2..>[:<reps>] same-box A/B of the product library against another build
#                                      (ZMPC_LIB) on bench --config c, alternating (AB_STEPS,
#                                      AB_EXTRA: more bench.py arguments)
#   lqprof:<config>                    strict LQ phase clocks (diagnostics build, ZMPC_LQ_PROF)
#   envab:<VAR>:<v1,v2..>:<config>:<reps> the diagnostics build at each value of an environment
#                                      switch (e.g. ZMPC_LQ_NLCK), alternating, kernel ms
#   ablate:<dbg bits>:<batches>        unconstrained phase ablation (diagnostics build,
#                                      ZMPC_DEBUG_ROLLOUT; default.json CoP data), e.g. ablate:0,1,4:4096
#   py:<name>:<script and args>        a diagnostic script (python) -> <name>.log; DIAG=1 in the
#                                      step name (pyd:...) loads the diagnostics build
#   sq:<B>                             SQ instruction / wait counters of the unconstrained rollout
#                                      (scripts/gpu_rollout_pmc.sh, CoP walks)
#   envsweep:<VAR>:<value>:<LO:HI:STEP> the diagnostics build's horizon sweep (strict leg) with an
#                                      environment switch set
#   sweep:<name>:<lib|->:<LO:HI:STEP>  the horizon sweep with the product library or another one
#   res                                register/scratch report of every kernel (host-side, no GPU)
set -u
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for s in "$@"; do
  kind=${s%%:*}
  rest=${s#*:}
  case $kind in
    tests)
      K=()
      [ "$rest" != "tests" ] && K=(-k "$rest")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
        --timeout-method thread -p no:cacheprovider "${K[@]}" > "$OUT/pytest.log" 2>&1
      rc=$?; tail -3 "$OUT/pytest.log"; step tests $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; tail -1 "$OUT/smoke.log"; step smoke $rc ;;
    bench)
      name=${rest%%:*}; args=${rest#*:}
      timeout -k 10 600 python bench.py $args > "$OUT/$name.json" 2> "$OUT/$name.err"
      rc=$?; cut -c1-400 "$OUT/$name.json"; [ $rc -ne 0 ] && tail -5 "$OUT/$name.err"
      step "bench $name" $rc ;;
    profile)
      wl=${rest%%:*}; rest=${rest#*:}; k=${rest%%:*}; args=${rest#*:}
      bash scripts/gpu_profile_round.sh "${TAG}_$wl" "$wl" "$k" $args > "$OUT/prof_$wl.log" 2>&1
      rc=$?; tail -1 "$OUT/prof_$wl.log" | cut -c1-300; step "profile $wl" $rc ;;
    ab)
      lib=${rest%%:*}; rest=${rest#*:}; cfgs=${rest%%:*}; reps=${rest#*:}
      [ "$reps" = "$cfgs" ] && reps=3
      for c in ${cfgs//,/ }; do
        for r in $(seq 1 "$reps"); do
          for side in new old; do
            if [ $side = new ]; then L=(); else L=(env ZMPC_LIB=$PWD/$lib); fi
            timeout -k 10 300 "${L[@]}" python bench.py --config $c --steps ${AB_STEPS:-10} \
              --warmup 2 --no-cpu-baseline --no-dense-leg ${AB_EXTRA:-} \
              > "$OUT/ab_c${c}_${side}_$r.json" 2> "$OUT/ab_c${c}_${side}_$r.err"
            step "ab $c $side $r" $?
          done
          python - "$OUT/ab_c${c}_new_$r.json" "$OUT/ab_c${c}_old_$r.json" <<'PY'
import json, sys
n, o = (json.loads(open(p).read().strip().splitlines()[-1]) for p in sys.argv[1:])
print(f"{n['config']['workload'][:48]}: new {n['roofline']['kernel_ms']:.5f} ms  "
      f"other {o['roofline']['kernel_ms']:.5f} ms", flush=True)
PY
        done
      done ;;
    envab)
      var=${rest%%:*}; rest=${rest#*:}; vals=${rest%%:*}; rest=${rest#*:}; c=${rest%%:*}; reps=${rest#*:}
      for r in $(seq 1 "$reps"); do
        for v in ${vals//,/ }; do
          env ZMPC_LIB=$PWD/model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal/libzmpc_diag.so \
            $var=$v timeout -k 10 300 python bench.py --config $c --steps ${AB_STEPS:-5} --warmup 2 \
            --no-cpu-baseline --no-dense-leg > "$OUT/envab_c${c}_${var}_${v}_$r.json" 2> "$OUT/envab_c${c}_${var}_${v}_$r.err"
          step "envab $var=$v" $?
          python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'])" "$OUT/envab_c${c}_${var}_${v}_$r.json" "$var=$v"
        done
      done ;;
    lqprof)
      ZMPC_LIB=$PWD/model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal/libzmpc_diag.so \
        ZMPC_LQ_PROF=1 timeout -k 10 300 python bench.py --config "$rest" --steps 1 --warmup 1 \
        --no-cpu-baseline > "$OUT/lqprof_c$rest.json" 2> "$OUT/lqprof_c$rest.err"
      rc=$?; grep "lq prof" "$OUT/lqprof_c$rest.err" | tail -2; step lqprof $rc ;;
    ablate)
      bits=${rest%%:*}; bs=${rest#*:}
      ZMPC_LIB=$PWD/model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal/libzmpc_diag.so \
        ABL_DATA=cop timeout -k 10 600 python scripts/ablate_rollout.py 8 "$bits" "$bs" \
        > "$OUT/ablate.jsonl" 2> "$OUT/ablate.err"
      rc=$?; cat "$OUT/ablate.jsonl"; step ablate $rc ;;
    py|pyd)
      name=${rest%%:*}; args=${rest#*:}
      L=()
      [ $kind = pyd ] && L=(env ZMPC_LIB=$PWD/model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal/libzmpc_diag.so)
      timeout -k 10 600 "${L[@]}" python -u $args > "$OUT/$name.log" 2>&1
      rc=$?; tail -4 "$OUT/$name.log" | cut -c1-400; step "py $name" $rc ;;
    sq)
      bash scripts/gpu_rollout_pmc.sh "$TAG/sq" "$rest" > "$OUT/sq.log" 2>&1
      rc=$?; tail -3 "$OUT/sq.log"; step sq $rc ;;
    envsweep)
      var=${rest%%:*}; rest=${rest#*:}; v=${rest%%:*}; rng=${rest#*:}
      env ZMPC_LIB=$PWD/model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal/libzmpc_diag.so \
        $var=$v timeout -k 10 600 python bench.py --sweep-horizon $rng --no-cpu-baseline \
        > "$OUT/envsweep_${var}_$v.jsonl" 2> "$OUT/envsweep_${var}_$v.err"
      rc=$?; python -c "import json,sys; [print(d['N'], '%.3e' % d['gpu_batched_strict']) for d in map(json.loads, open(sys.argv[1])) if 'N' in d]" "$OUT/envsweep_${var}_$v.jsonl"
      step envsweep $rc ;;
    sweep)
      name=${rest%%:*}; rest=${rest#*:}; lib=${rest%%:*}; rng=${rest#*:}
      L=()
      [ "$lib" != "-" ] && L=(env ZMPC_LIB=$PWD/$lib)
      timeout -k 10 600 "${L[@]}" python bench.py --sweep-horizon $rng --no-cpu-baseline \
        > "$OUT/sweep_$name.jsonl" 2> "$OUT/sweep_$name.err"
      rc=$?; python -c "import json,sys; [print(sys.argv[2], d['N'], '%.3e' % d['gpu_batched_strict']) for d in map(json.loads, open(sys.argv[1])) if 'N' in d]" "$OUT/sweep_$name.jsonl" "$name"
      step "sweep $name" $rc ;;
    res)
      for f in rollout strict_lq strict_scan herdt; do
        make -s -C model-predictive-control-for-bipedal-locomotion_amd/csrc resources RES=$f
        python scripts/res_summary.py /tmp/zmpc_res/$f.txt > "$OUT/res_$f.txt"
      done
      step res 0 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
