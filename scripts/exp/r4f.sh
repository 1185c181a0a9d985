set -o pipefail
timeout -k 10 120 python -u -m pytest tests/test_gpu_r4.py -x -q --timeout 100 --timeout-method thread -k "gemm_big or ppo_head" && \
timeout -k 10 300 python -u scripts/exp/gemm_big_bench.py && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4f/tr -o run -- python3 scripts/bench_configs.py --configs breakout_ppo --updates 2 --warmup 1 > gpurun_out/r4f/tr.log 2>&1 && \
python3 scripts/trace_summary.py $(find gpurun_out/r4f/tr -name "*kernel_trace.csv") --updates 1 --marker pong_fused_env_step --per-update 128 > gpurun_out/r4f/breakout_trace_summary.txt && head -40 gpurun_out/r4f/breakout_trace_summary.txt && \
find gpurun_out/r4f/tr -name "*.csv" -size +6M -delete
