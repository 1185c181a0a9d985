#!/bin/bash
# MuJoCo-shape PPO: rollout phase stamps, DP world-1 vs no-DP update time
set -o pipefail
timeout -k 10 200 python -u scripts/microbench_rollout.py || exit 1
for f in "" "--dp-world1"; do
  timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 5 --warmup 2 $f 2>/dev/null | cut -c1-120 || exit 1
done
