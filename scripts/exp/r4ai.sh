# Software-pipelined bf16-staged trunk forward: trunk tests, standalone A/B at B = 4096, Breakout PPO.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_r2.py tests/test_gpu_r4.py -x -q --timeout 120 --timeout-method thread -k "trunk" && \
timeout -k 10 120 python -u scripts/exp/trunk_fwd_ab.py && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2
