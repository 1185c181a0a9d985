#!/bin/bash
# Headline bench A/B over env knob sets (2 runs each, 400 steps) + one driver-shaped run (20 steps) of the first.
# Usage: bash scripts/gpu_job_bench.sh TAG "" "K=V ..." ...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
i=0
for knobs in "$@"; do
  for rep in 1 2; do
    i=$((i+1))
    env $knobs timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b$i.json 2> $O/b$i.err || { echo "bench fail [$knobs]"; tail -5 $O/b$i.err; exit 1; }
    echo "[$knobs] rep $rep: $(python3 -c "import json;d=json.load(open('$O/b$i.json'));print(d['value'], d['ms_per_step'])")"
  done
done
env $1 timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/drv.json 2> $O/drv.err && echo "driver-shaped [$1]: $(python3 -c "import json;d=json.load(open('$O/drv.json'));print(d['value'], d['ms_per_step'])")"
