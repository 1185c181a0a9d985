#!/bin/bash
# Round-3 job X: 8-wave per-env trunk forward for rollout batches: tests, Breakout A/B, trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3x
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_kernels.py tests/test_gpu_r2.py tests/test_gpu_mlp.py tests/test_a3c_gpu_mode.py -m gpu -x -q --timeout 120 --timeout-method thread -k "trunk or index or engine or fused or adam or opt or optim" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E |FAILED" $O/t.log | head -12; [ $rc -eq 0 ] || exit $rc
for knob in 256 0 256 0; do
  ACA_TRUNK_FWD_WIDE_MAX_B=$knob timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/c.jsonl 2> $O/c.err || { tail -3 $O/c.err; exit 1; }
  echo "[breakout ACA_TRUNK_FWD_WIDE_MAX_B=$knob] $(python3 -c "import json;d=json.loads(open('$O/c.jsonl').read().splitlines()[-1]);print(d['ms_per_update'])")"
done
timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b.json 2> $O/b.err && echo "[pong] $(cat $O/b.json)"
timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 > $O/m.jsonl 2> $O/m.err && echo "[mujoco] $(tail -n 1 $O/m.jsonl)"
timeout -k 10 300 bash scripts/gpu_job_trace.sh breakout pong_policy_step 128 2 "" python3 scripts/bench_configs.py --configs breakout_ppo --updates 4 && cp gpurun_out/trace/breakout_summary.txt $O/
