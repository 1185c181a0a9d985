#!/bin/bash
# SPEC actor's fused Gaussian loss head: MLP numerics, MuJoCo learning, DP; then phases and update time
set -o pipefail
O=gpurun_out/fgh; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mlp.py \
  tests/test_gpu_learning.py tests/test_gpu_r4.py tests/test_gpu_dp.py -k "mlp or mujoco or MLP or spec" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u scripts/microbench_mlp_train.py > $O/mb.json 2> $O/mb.err || { tail -5 $O/mb.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/mb.json')); [print(k, v) for k, v in d.items() if k.startswith('tower0') or 'launch' in k or 'step' in k]"
timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 5 --warmup 2 2>/dev/null | cut -c1-120
