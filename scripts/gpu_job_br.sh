#!/bin/bash
# Breakout-shape PPO: config bench + kernel trace summary (rocpd database).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/br
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 > $O/cfg.jsonl 2> $O/cfg.err || { tail -5 $O/cfg.err; exit 1; }
cat $O/cfg.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 scripts/bench_configs.py --configs breakout_ppo --updates 3 --warmup 1 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python3 scripts/rocpd_top.py $(find $O/prof -name "*.db" | head -1) 4 30
