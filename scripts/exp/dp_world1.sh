#!/bin/bash
# the data-parallel updates at RCCL world size 1 -- ms per update with and without the DP
# schedule, and the per-update kernel trace of the DP update (RCCL kernels included) for Breakout PPO and MuJoCo PPO.
# Usage (on the GPU box): bash scripts/gpu.sh TAG cmd=scripts/exp/dp_world1.sh
set -o pipefail
O=gpurun_out/dp_world1
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo,mujoco_ppo_dp8 --updates 5 --warmup 2 \
  > $O/plain.jsonl 2> $O/plain.err || { tail -5 $O/plain.err; exit 1; }
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo,mujoco_ppo_dp8 --updates 5 --warmup 2 \
  --dp-world1 > $O/dp.jsonl 2> $O/dp.err || { tail -5 $O/dp.err; exit 1; }
cat $O/plain.jsonl $O/dp.jsonl
for cfg in mujoco_ppo_dp8 breakout_ppo; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$cfg -o run -- python3 \
    scripts/bench_configs.py --configs $cfg --updates 2 --warmup 1 --dp-world1 > $O/tr_$cfg.log 2>&1 \
    || { tail -5 $O/tr_$cfg.log; exit 1; }
  m=$([ $cfg = mujoco_ppo_dp8 ] && echo "mlp_rollout 1" || echo "pong_fused_env_step 128")
  python3 scripts/trace_summary.py $(find $O/tr_$cfg -name "*kernel_trace.csv") --updates 1 --marker ${m% *} \
    --per-update ${m#* } > $O/${cfg}_dp_trace_summary.txt && head -30 $O/${cfg}_dp_trace_summary.txt
  grep -iE "nccl|rccl|allreduce|reduce_scatter" $O/${cfg}_dp_trace_summary.txt | head -10
  find $O/tr_$cfg -name "*.csv" -size +6M -delete
done
