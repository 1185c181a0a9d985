#!/bin/bash
# MLP-engine microbenchmarks (train-kernel phase stamps, rollout phases) + the MLP / optimiser GPU tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mb
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "opt or adam or rmsprop or mlp" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
timeout -k 10 200 python -u scripts/microbench_mlp_train.py > $O/mlp_train.json 2> $O/mlp_train.err || { tail -5 $O/mlp_train.err; exit 1; }
cat $O/mlp_train.json
timeout -k 10 200 python -u scripts/microbench_rollout.py > $O/rollout.json 2>&1 || exit 1
cat $O/rollout.json
timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 5 --warmup 2 > $O/cfg.jsonl 2> $O/cfg.err || { tail -5 $O/cfg.err; exit 1; }
cat $O/cfg.jsonl
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 3 --warmup 1 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-200
find $O/prof -name "*.csv" -size +6M -delete
