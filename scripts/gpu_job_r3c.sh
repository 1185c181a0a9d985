#!/bin/bash
# Round-3 job C: learning curves with the linear lr schedule (CartPole both engines, MuJoCo PPO 300 updates).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
for eng in native torch; do
  timeout -k 10 300 python -u scripts/learn_curve.py --preset cartpole_cpu --updates 3000 --report 300 --engine $eng \
    device=cuda:0 num_envs=64 cuda_graph=true lr_schedule=linear total_updates=3000 > $O/cp_$eng.jsonl 2> $O/cp_$eng.err || { tail -3 $O/cp_$eng.err; exit 1; }
  echo "cartpole $eng: $(python3 -c "import json;print([round(json.loads(l)['ep_return']) for l in open('$O/cp_$eng.jsonl')])")"
done
timeout -k 10 400 python -u scripts/learn_curve.py --preset mujoco_ppo_dp8 --updates 300 --report 30 \
  lr_schedule=linear total_updates=300 > $O/mj_lin.jsonl 2> $O/mj_lin.err || { tail -3 $O/mj_lin.err; exit 1; }
echo "mujoco linear: $(python3 -c "import json;print([round(json.loads(l)['ep_return']) for l in open('$O/mj_lin.jsonl')])")"
bash scripts/gpu_job_trace.sh mj_r3 mlp_rollout_kernel 1 4 "" python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 8 --warmup 1 || exit 1
timeout -k 10 300 python -u scripts/learn_curve.py --preset pendulum_ppo --updates 100 --report 10 > $O/pend_ppo.jsonl 2> $O/pend_ppo.err || { tail -3 $O/pend_ppo.err; exit 1; }
echo "pendulum_ppo: $(python3 -c "import json;print([round(json.loads(l)['ep_return']) for l in open('$O/pend_ppo.jsonl')])")"
