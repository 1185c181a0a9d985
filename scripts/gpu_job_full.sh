#!/bin/bash
# Full GPU test suite, then the headline bench (driver settings x3 + a long run) and Breakout / MuJoCo PPO configs.
# Usage: bash scripts/gpu_job_full.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-full}
O=gpurun_out/$TAG
mkdir -p $O
python -c "from actor_critic_algs_on_tensorflow_amd import _native; _native.load(raise_on_error=True)" || exit 3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -3; grep -E "FAILED|Error|assert" $O/tests.log | head -20
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || { tail -5 $O/bench_$i.err; exit 1; }
  echo "bench20 $i: $(python3 -c "import json;d=json.load(open('$O/bench_$i.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/bench_400.json 2> $O/bench_400.err || { tail -5 $O/bench_400.err; exit 1; }
echo "bench400: $(python3 -c "import json;d=json.load(open('$O/bench_400.json'));print(d['value'], d['ms_per_step'])")"
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo,mujoco_ppo_dp8 --updates 5 --warmup 2 > $O/configs.jsonl 2> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
cat $O/configs.jsonl
