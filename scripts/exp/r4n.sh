# Split per-env fused rollout step (two workgroups per env): bitwise tests, Breakout PPO A/B, and the kernel trace.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_r4.py tests/test_gpu_r2.py tests/test_gpu_r3.py -x -q --timeout 120 --timeout-method thread -k "fused or trunk" && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 --engine-opts '{"fused_env_split": false}'
