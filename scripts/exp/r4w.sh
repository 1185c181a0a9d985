# Engine on the bf16-staged trunk forward: trainer-level bitwise tests, Breakout PPO A/B.
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_r4.py tests/test_gpu_r3.py -x -q --timeout 120 --timeout-method thread && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 --engine-opts '{"trunk_fwd_staged": false}'
