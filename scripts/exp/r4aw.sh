#!/bin/bash
# kernel traces: Breakout PPO and the headline A2C config, per-update summaries
set -o pipefail
O=gpurun_out/r4aw
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 scripts/bench_configs.py --configs breakout_ppo --updates 2 --warmup 1 > $O/tr.log 2>&1 && \
python3 scripts/trace_summary.py $(find $O/tr -name "*kernel_trace.csv") --updates 1 --marker pong_fused_env_step --per-update 128 > $O/breakout_trace_summary.txt && \
find $O/tr -name "*.csv" -size +6M -delete && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trh -o run -- python3 bench.py --steps 20 --warmup 5 > $O/trh.log 2>&1 && \
python3 scripts/trace_summary.py $(find $O/trh -name "*kernel_trace.csv") --updates 20 --marker pong_fused_step --per-update 5 > $O/headline_trace_summary.txt && \
find $O/trh -name "*.csv" -size +6M -delete
