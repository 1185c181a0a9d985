#!/bin/bash
# Round-3 job R: knob sweep on the current tree -- headline (fc split-K planes, conv weight-gradient planes, early
# weight loads) and Breakout PPO (weight-gradient plane counts). One bench process per setting.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3r
mkdir -p $O
for knobs in "" "ACA_FC_MAX_PLANES=16" "ACA_FC_MAX_PLANES=8" "ACA_WGRAD_PLANES=32" "ACA_WGRAD_PLANES=128" "ACA_FUSED_EARLY_W=1" "ACA_TRUNK_MODE=1"; do
  env $knobs timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  echo "[pong $knobs] $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'])")"
done
for knobs in "" "ACA_NHWC_PLANES=128" "ACA_NHWC3_PLANES=128" "ACA_CONV1_PLANES=64" "ACA_NHWC_PLANES=128 ACA_NHWC3_PLANES=128 ACA_CONV1_PLANES=64"; do
  env $knobs timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/c.jsonl 2> $O/c.err || { tail -3 $O/c.err; exit 1; }
  echo "[breakout $knobs] $(python3 -c "import json;d=json.loads(open('$O/c.jsonl').read().splitlines()[-1]);print(d['ms_per_update'])")"
done
