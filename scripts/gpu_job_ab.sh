#!/bin/bash
# A/B of env knobs on a bench_configs config. Usage: bash scripts/gpu_job_ab.sh TAG CONFIG UPDATES "K=V ..." ...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; CFG=$2; UPD=$3; shift 3
O=gpurun_out/$TAG
mkdir -p $O
i=0
for knobs in "$@"; do
  i=$((i+1))
  env $knobs timeout -k 10 300 python -u scripts/bench_configs.py --configs $CFG --updates $UPD --warmup 2 > $O/ab_$i.jsonl 2> $O/ab_$i.err || { echo "fail [$knobs]"; tail -5 $O/ab_$i.err; exit 1; }
  echo "[$knobs] $(cat $O/ab_$i.jsonl)"
done
