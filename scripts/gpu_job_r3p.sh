#!/bin/bash
# Round-3 job P: learning-stability variants (CartPole A2C both engines, MuJoCo PPO 300 updates), 3 seeds each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3p
mkdir -p $O
run() {
  local lab=$1; shift
  echo "## $lab" >> $O/curves.txt
  timeout -k 10 240 python -u scripts/learn_curve.py "$@" >> $O/curves.txt 2> $O/err.txt || { echo "FAIL $lab"; tail -3 $O/err.txt; exit 1; }
}
: > $O/curves.txt
for seed in 1 2 3; do
  for eng in native torch; do
    for v in "lr=5e-4 critic_lr=2e-3" "lr=5e-4 critic_lr=2e-3 ent_coef=0.01" "lr=3e-4 critic_lr=1e-3 ent_coef=0.01"; do
      run "cartpole $eng [$v] linear seed$seed" --preset cartpole_cpu --updates 4000 --report 400 --engine $eng --seed $seed device=cuda:0 num_envs=64 cuda_graph=true lr_schedule=linear total_updates=4000 $v
    done
  done
  for v in "lr=1e-4 critic_lr=3e-4" "lr=3e-4 critic_lr=1e-3 ppo_epochs=4" "lr=3e-4 critic_lr=1e-3 lr_schedule=linear total_updates=300 ppo_epochs=4" "lr=1e-4 critic_lr=1e-3 lr_schedule=linear total_updates=300"; do
    run "mujoco [$v] seed$seed" --preset mujoco_ppo_dp8 --updates 300 --report 30 --seed $seed $v
  done
done
python3 - <<'PY'
import json
lab=None
out=open("gpurun_out/r3p/summary.txt","w")
for line in open("gpurun_out/r3p/curves.txt"):
    if line.startswith("##"):
        lab=line[3:].strip(); out.write("\n"+lab+": ")
    else:
        out.write("%d " % round(json.loads(line)["ep_return"]))
out.close()
print(open("gpurun_out/r3p/summary.txt").read())
PY
