#!/bin/bash
# Learning curves on the device engines (pong A2C native, CartPole MLP vs torch engine, MuJoCo PPO, async PS).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-learn}
mkdir -p $O
timeout -k 10 240 python -u scripts/learn_curve.py --preset pong_a2c --updates 40000 --report 4000 > $O/pong.jsonl 2> $O/pong.err || { tail -5 $O/pong.err; exit 1; }
cat $O/pong.jsonl
for eng in native torch; do
  timeout -k 10 200 python -u scripts/learn_curve.py --preset cartpole_cpu --updates 3000 --report 300 --engine $eng device=cuda:0 num_envs=64 cuda_graph=true > $O/cp_$eng.jsonl 2> $O/cp_$eng.err || { tail -5 $O/cp_$eng.err; exit 1; }
  echo "cartpole $eng"; cat $O/cp_$eng.jsonl
done
timeout -k 10 200 python -u scripts/learn_curve.py --preset mujoco_ppo_dp8 --updates 300 --report 30 > $O/mj.jsonl 2> $O/mj.err || { tail -5 $O/mj.err; exit 1; }
echo mujoco; cat $O/mj.jsonl
timeout -k 10 300 python -u scripts/a3c_gpu_curve.py --workers 2 --updates 4000 --report 250 --out $O/a3c > $O/a3c.log 2>&1 || { tail -20 $O/a3c.log; exit 1; }
grep '"role": "worker"' $O/a3c.log | cut -c1-1500
