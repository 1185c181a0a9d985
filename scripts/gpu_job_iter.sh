#!/bin/bash
# One build -> measure iteration on the GPU box: round-2 GPU tests, microbench, headline bench (A/B env knobs),
# kernel-trace summary of the headline. Usage: bash scripts/gpu_job_iter.sh TAG ["ENV=1 ENV2=0" ...]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-iter}
shift
O=gpurun_out/$TAG
mkdir -p $O
python -c "from actor_critic_algs_on_tensorflow_amd import _native; _native.load(raise_on_error=True)" || exit 3
timeout -k 10 400 python -u -m pytest tests/test_gpu_r2.py tests/test_gpu_kernels.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread > $O/tests_r2.log 2>&1
rc=$?; echo "tests_r2 rc=$rc"; tail -5 $O/tests_r2.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u scripts/microbench_r2.py --out $O/mb.json > $O/mb.log 2>&1; rc=$?
echo "mb rc=$rc"; cat $O/mb.json 2>/dev/null || tail -20 $O/mb.log
[ $rc -ne 0 ] && exit $rc
for knobs in "" "$@"; do
  env $knobs timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 > $O/bench.json 2> $O/bench.err || { echo "bench fail [$knobs]"; tail -5 $O/bench.err; exit 1; }
  echo "bench [$knobs]: $(python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 60 --warmup 10 > $O/trace.log 2>&1 && \
python3 scripts/trace_summary.py $(find $O/trace -name "*kernel_trace.csv") --updates 40 --marker pong_policy_step --per-update 5 > $O/trace_summary.txt && cat $O/trace_summary.txt
rc=$?
find $O -name "*.csv" -size +4M -delete
exit $rc
