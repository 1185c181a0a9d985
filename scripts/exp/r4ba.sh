#!/bin/bash
# MuJoCo-shape PPO kernel trace (per update)
set -o pipefail
O=gpurun_out/r4ba
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 2 --warmup 1 > $O/tr.log 2>&1 && \
python3 scripts/trace_summary.py $(find $O/tr -name "*kernel_trace.csv") --updates 1 --marker mlp_rollout --per-update 1 > $O/mujoco_trace_summary.txt ; \
find $O/tr -name "*.csv" -size +6M -delete
