#!/bin/bash
# kernel trace of MuJoCo-shape PPO under DP at world 1 (RCCL, one graph per update) + whether the direct path engaged
set -o pipefail
O=gpurun_out/${TAG:-dptrace}
mkdir -p $O
timeout -k 10 120 python -c "
import os, torch, torch.distributed as dist
os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT='29533')
dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
from actor_critic_algs_on_tensorflow_amd.parallel.dp import DataParallel
dp = DataParallel(); print('direct comm', hex(dp._comm))
dist.destroy_process_group()" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 2 --warmup 1 --dp-world1 > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
python3 scripts/trace_summary.py $(find $O/tr -name "*kernel_trace.csv") --updates 1 --marker mlp_rollout --per-update 1 > $O/summary.txt && head -30 $O/summary.txt
find $O/tr -name "*.csv" -size +6M -delete
