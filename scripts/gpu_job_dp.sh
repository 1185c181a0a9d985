#!/bin/bash
# DP segment tests + returns scan tests + headline bench. Usage: bash scripts/gpu_job_dp.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-dp}
O=gpurun_out/$TAG
mkdir -p $O
python -c "from actor_critic_algs_on_tensorflow_amd import _native; _native.load(raise_on_error=True)" || exit 3
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -3; grep -E "FAILED|Error|assert" $O/tests.log | head -20
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || { tail -5 $O/bench_$i.err; exit 1; }
  echo "bench20 $i: $(python3 -c "import json;d=json.load(open('$O/bench_$i.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/bench_400.json 2> $O/bench_400.err || { tail -5 $O/bench_400.err; exit 1; }
echo "bench400: $(python3 -c "import json;d=json.load(open('$O/bench_400.json'));print(d['value'], d['ms_per_step'])")"
