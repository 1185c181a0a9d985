#!/bin/bash
# Round-3 job K (session restart): full GPU suite on the rebuilt tree, headline bench, the other BASELINE configs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O
python -c "from actor_critic_algs_on_tensorflow_amd import _native; _native.load(raise_on_error=True)" || exit 3
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^E |FAILED" $O/tests.log | head -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u bench.py > $O/bench20.json 2> $O/bench20.err && cat $O/bench20.json || exit 1
timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/bench400.json 2> $O/bench400.err && cat $O/bench400.json || exit 1
timeout -k 10 400 python -u scripts/bench_configs.py --configs breakout_ppo,mujoco_ppo_dp8 > $O/cfg.jsonl 2> $O/cfg.err && cat $O/cfg.jsonl
timeout -k 10 300 bash scripts/gpu_job_trace.sh a2c_pong pong_fused_step 5 200 "" python3 bench.py --steps 400 --warmup 20 && cp gpurun_out/trace/a2c_pong_summary.txt $O/
