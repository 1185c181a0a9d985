#!/bin/bash
# 4-row MuJoCo train path: kernel stats with / without it
set -o pipefail
O=gpurun_out/rows4; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for r in 1 0; do
  ACA_MLP_ROWS4=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof$r -o run -- \
    python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 3 --warmup 1 > /dev/null 2>&1 || exit 1
  f=$(find $GRAFT_REPO_ROOT/$O/prof$r -name "*kernel_stats.csv" | sed -n 1p); cut -d, -f1-8 "$f" | sed -n 1,12p
done
