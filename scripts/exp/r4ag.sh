# Trunk data-gradient kernel with software-pipelined operand reads: bitwise tests, phases, Breakout PPO.
set -o pipefail
O=gpurun_out/${TAG:-r4ag}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_r2.py tests/test_gpu_r3.py tests/test_gpu_r4.py -x -q --timeout 120 --timeout-method thread -k "bwd or trunk or fused" && \
timeout -k 10 120 python -u scripts/exp/trunk_bwd_phases.py > $O/phases.json && cat $O/phases.json && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2
