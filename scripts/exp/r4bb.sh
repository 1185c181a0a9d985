#!/bin/bash
# optimiser operand loads ahead of the norm reduction: GPU suite + configs + headline
set -o pipefail
O=gpurun_out/r4bb
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 400 python3 -u scripts/bench_configs.py --configs breakout_ppo,mujoco_ppo_dp8 --updates 8 --warmup 2 > $O/configs.log 2>&1 && \
timeout -k 10 180 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
