#!/bin/bash
# Round-3 job M: learning stability: CartPole on both engines and MuJoCo PPO over 300 updates,
# constant vs linear lr schedule, two seeds each. One JSON line per report, headed by the run's label.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3m
mkdir -p $O
run() {   # label, args...
  local lab=$1; shift
  echo "## $lab" >> $O/curves.txt
  timeout -k 10 240 python -u scripts/learn_curve.py "$@" >> $O/curves.txt 2> $O/err.txt || { echo "FAIL $lab"; tail -3 $O/err.txt; exit 1; }
  echo "$lab: $(tail -n 1 $O/curves.txt)"
}
: > $O/curves.txt
for seed in 1 2; do
  for eng in native torch; do
    for sch in constant linear; do
      run "cartpole $eng $sch seed$seed" --preset cartpole_cpu --updates 3000 --report 300 --engine $eng --seed $seed device=cuda:0 num_envs=64 cuda_graph=true lr_schedule=$sch total_updates=3000
    done
  done
  for sch in constant linear; do
    run "mujoco $sch seed$seed" --preset mujoco_ppo_dp8 --updates 300 --report 30 --seed $seed lr_schedule=$sch total_updates=300
  done
done
