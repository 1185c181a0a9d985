#!/bin/bash
# MLP SPEC head/store ordering A/B: numerics, standalone microbench, MuJoCo config bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6head}
mkdir -p $O
python -c "from actor_critic_algs_on_tensorflow_amd import _native; _native.load(raise_on_error=True)" || exit 3
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/microbench_mlp_train.py > $O/mb.json 2> $O/mb.err || { tail -5 $O/mb.err; exit 1; }
cat $O/mb.json
timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 5 --warmup 2 > $O/configs.jsonl 2> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
cat $O/configs.jsonl
