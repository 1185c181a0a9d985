set -o pipefail
O=gpurun_out/r4j
timeout -k 10 600 python -u -m pytest tests/test_gpu_r4.py tests/test_gpu_r2.py -x -q --timeout 120 --timeout-method thread && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo,mujoco_ppo_dp8 --updates 5 --warmup 2 && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 5 --warmup 2 --dp-world1 && \
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 scripts/bench_configs.py --configs breakout_ppo --updates 2 --warmup 1 > $O/tr.log 2>&1 && \
python3 scripts/trace_summary.py $(find $O/tr -name "*kernel_trace.csv") --updates 1 --marker pong_fused_env_step --per-update 128 > $O/breakout_trace_summary.txt && head -12 $O/breakout_trace_summary.txt && \
find $O/tr -name "*.csv" -size +6M -delete
