#!/bin/bash
# DP at world 1 (RCCL, one-graph update) vs no DP: MuJoCo-shape PPO, Breakout-shape PPO, headline A2C schedules
set -o pipefail
for c in mujoco_ppo_dp8 breakout_ppo; do
  timeout -k 10 300 python -u scripts/bench_configs.py --configs $c --updates 5 --warmup 2 || exit 1
  timeout -k 10 300 python -u scripts/bench_configs.py --configs $c --updates 5 --warmup 2 --dp-world1 || exit 1
done
for o in "" "--dp-world1" "--dp-world1 --overlap lag1" "--dp-world1 --bucket-dtype bf16"; do
  echo "bench $o: $(timeout -k 10 120 python -u bench.py --steps 200 --warmup 10 $o 2>/dev/null | tail -1)" || exit 1
done
