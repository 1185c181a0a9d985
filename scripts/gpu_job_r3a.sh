#!/bin/bash
# Round-3 checkpoint job: full GPU suite, headline bench (fused finaliser+optimiser), Pendulum learning sweep.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
python -c "from actor_critic_algs_on_tensorflow_amd import _native; _native.load(raise_on_error=True)" || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" $O/tests.log | tail -3; grep -E "FAILED|Error" $O/tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
ACA_FUSED_FINOPT=0 timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/bench_nofuse.json 2> $O/bench_nofuse.err || exit 1
cat $O/bench_nofuse.json
timeout -k 10 700 python -u scripts/pendulum_sweep.py --updates 10000 --out $O/pend > $O/sweep.jsonl 2> $O/sweep.err
grep summary $O/sweep.jsonl
