#!/bin/bash
# MuJoCo-shape PPO: no DP vs DP at world 1 (strict)
set -o pipefail
for dp in "" "--dp-world1"; do
  timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 5 --warmup 2 $dp 2>/dev/null \
    | cut -c1-140 || exit 1
done
