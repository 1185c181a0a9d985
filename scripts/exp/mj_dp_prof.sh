#!/bin/bash
# MuJoCo-shape PPO under DP at world 1: per-kernel stats (what the DP step adds per minibatch)
set -o pipefail
O=gpurun_out/mjdp; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 3 --warmup 1 --dp-world1 > /dev/null 2>&1 || exit 1
f=$(find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | sed -n 1p); cut -d, -f1-6 "$f" | cut -c1-150 | sed -n 1,16p
