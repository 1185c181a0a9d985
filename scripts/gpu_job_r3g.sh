#!/bin/bash
# Round-3 job G: Breakout PPO rollout trunk form (row-split fused step up to B envs) x serial backward.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
i=0
for knobs in "ACA_TRUNK_ROWS_MAX_B=64" "ACA_TRUNK_ROWS_MAX_B=128" "ACA_TRUNK_ROWS_MAX_B=128 ACA_SERIAL_BWD=1" "ACA_TRUNK_ROWS_MAX_B=256"; do
  i=$((i+1))
  env $knobs timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/br$i.jsonl 2> $O/br$i.err || { tail -3 $O/br$i.err; exit 1; }
  echo "[$knobs] $(python3 -c "import json;d=json.loads(open('$O/br$i.jsonl').read().splitlines()[-1]);print(d['ms_per_update'])")"
done
