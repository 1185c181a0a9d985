#!/bin/bash
# Non-headline configs (Breakout PPO / MuJoCo PPO) over env knob sets. Usage: bash scripts/gpu_job_cfg.sh TAG CONFIG UPDATES "K=V ..." ...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; CFG=$2; UPD=$3; shift 3
O=gpurun_out/$TAG
mkdir -p $O
i=0
for knobs in "$@"; do
  i=$((i+1))
  env $knobs timeout -k 10 300 python -u scripts/bench_configs.py --configs $CFG --updates $UPD --warmup 2 > $O/c$i.jsonl 2> $O/c$i.err || { echo "cfg fail [$knobs]"; tail -5 $O/c$i.err; exit 1; }
  echo "[$knobs] $(tail -1 $O/c$i.jsonl)"
done
