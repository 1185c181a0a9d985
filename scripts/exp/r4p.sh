# Fused env step with the head's loads first and the conv2 fragments after the render: bitwise tests, phase stamps,
# Breakout PPO A/B (split / whole).
set -o pipefail
O=gpurun_out/${TAG:-r4p}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_r4.py tests/test_gpu_r2.py tests/test_gpu_r3.py -x -q --timeout 120 --timeout-method thread -k "fused or trunk" && \
timeout -k 10 300 python -u scripts/exp/env_step_phases.py > $O/phases.json && cat $O/phases.json && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 --engine-opts '{"fused_env_split": false}'
