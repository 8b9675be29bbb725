set -u
O=gpurun_out/nt; mkdir -p $O
timeout -k 10 300 python3 scripts/ab_rollout.py '[{}, {"ZMPC_LIB": "model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal/libzmpc_nt.so"}, {}]' '[[4096, 150, 420], [16384, 150, 420]]' > $O/ab.jsonl 2>&1 || exit $?
for v in base nt base2 nt2; do
  if [ "${v#nt}" != "$v" ]; then export ZMPC_LIB=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal/libzmpc_nt.so; else unset ZMPC_LIB; fi
  timeout -k 10 300 python3 bench.py --config 6 --steps 3 --warmup 1 --no-cpu-baseline > $O/c6_$v.json 2> $O/c6_$v.err || exit $?
  timeout -k 10 300 python3 bench.py --config 4 --unconstrained --steps 5 --warmup 1 --no-cpu-baseline > $O/c4u_$v.json 2> $O/c4u_$v.err || exit $?
done
