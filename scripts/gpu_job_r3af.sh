#!/bin/bash
# Round-3 job AF: Breakout PPO rollout through the fused row-split step (ACA_TRUNK_ROWS_MAX_B=128: 7 x 128 row
# workgroups per step) vs the per-env trunk + fc + policy/env launches (default 64).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3af
mkdir -p $O
for k in 128 64 128 64; do
  ACA_TRUNK_ROWS_MAX_B=$k timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/c.jsonl 2> $O/c.err || { tail -3 $O/c.err; exit 1; }
  echo "[breakout ACA_TRUNK_ROWS_MAX_B=$k] $(python3 -c "import json;d=json.loads(open('$O/c.jsonl').read().splitlines()[-1]);print(d['ms_per_update'])")"
done
