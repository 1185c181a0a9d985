#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4bg
timeout -k 10 400 python3 -u scripts/bench_configs.py --configs mujoco_ppo_dp8,breakout_ppo --updates 8 --warmup 2 > gpurun_out/r4bg/configs.log 2>&1
