#!/bin/bash
# trunk backward addressing rewrite: bitwise tests + Breakout PPO + headline
set -e
mkdir -p gpurun_out/r4av
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_r2.py tests/test_gpu_r3.py > gpurun_out/r4av/tests.log 2>&1
timeout -k 10 300 python3 -u scripts/bench_configs.py --configs breakout_ppo --updates 10 --warmup 3 > gpurun_out/r4av/breakout.log 2>&1
timeout -k 10 180 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r4av/bench.log 2>&1
