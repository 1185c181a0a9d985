#!/bin/bash
# Round-3 job W: PPO minibatches gathered by index + the 16-wave PPO loss launch: tests, Breakout A/B, headline planes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_kernels.py tests/test_gpu_r2.py tests/test_gpu_learning.py -m gpu -x -q --timeout 120 --timeout-method thread -k "index or mb_gather or loss or production_batch or fused_head or ppo or conv1" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E |FAILED" $O/t.log | head -12; [ $rc -eq 0 ] || exit $rc
for knob in 1 0 1 0; do
  ACA_MB_INDEX=$knob timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/c.jsonl 2> $O/c.err || { tail -3 $O/c.err; exit 1; }
  echo "[breakout ACA_MB_INDEX=$knob] $(python3 -c "import json;d=json.loads(open('$O/c.jsonl').read().splitlines()[-1]);print(d['ms_per_update'])")"
done
for knobs in "" "ACA_FC_MAX_PLANES=16" "" "ACA_FC_MAX_PLANES=16"; do
  env $knobs timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  echo "[pong $knobs] $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 300 bash scripts/gpu_job_trace.sh breakout pong_policy_step 128 2 "" python3 scripts/bench_configs.py --configs breakout_ppo --updates 4 && cp gpurun_out/trace/breakout_summary.txt $O/
