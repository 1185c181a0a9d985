#!/bin/bash
# 4-env rollout tiles: MFMA layout probe, MLP tests, rollout phase stamps, MuJoCo-shape PPO update time
set -o pipefail
timeout -k 5 60 ./scripts/probes/mfma4x4 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -15 || exit 1
timeout -k 10 200 python -u scripts/microbench_rollout.py 2>/dev/null | tail -12 || exit 1
timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 5 --warmup 2 2>/dev/null | cut -c1-120
