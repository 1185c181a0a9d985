# kernel traces of the DP schedules at RCCL world 1 (headline strict, Breakout PPO)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5dptr; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/a2c -o run -- python3 bench.py --steps 40 --warmup 5 --dp-world1 > $O/a2c.log 2>&1 || { tail -5 $O/a2c.log; exit 1; }
python3 scripts/trace_summary.py $(find $O/a2c -name "*kernel_trace.csv") --updates 30 --marker pong_fused_step --per-update 5 > $O/a2c_sum.txt && head -24 $O/a2c_sum.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/br -o run -- python3 scripts/bench_configs.py --configs breakout_ppo --updates 2 --warmup 1 --dp-world1 > $O/br.log 2>&1 || { tail -5 $O/br.log; exit 1; }
python3 scripts/trace_summary.py $(find $O/br -name "*kernel_trace.csv") --updates 1 --marker pong_fused_env_step --per-update 128 > $O/br_sum.txt && head -30 $O/br_sum.txt
find $O -name "*.csv" -size +6M -delete
