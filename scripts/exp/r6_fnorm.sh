#!/bin/bash
# whole-segment norm of the MLP optimiser item path: numerics, then MuJoCo DP world-1 cost with it
set -o pipefail
O=gpurun_out/fnorm; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mlp.py \
  -k "item_path or spec_train or trainer or multi_group" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dp.py \
  -k "mlp or mujoco" > $O/tests_dp.log 2>&1 || { tail -30 $O/tests_dp.log; exit 1; }
tail -2 $O/tests_dp.log
for dp in "" "--dp-world1"; do
  timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 5 \
    --warmup 2 $dp 2>/dev/null | cut -c1-140 || exit 1
done
