#!/bin/bash
# Round-3 job Q: MLP weight-gradient launch with Adam folded in: tests, MuJoCo PPO A/B + trace; headline re-check.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3q
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_learning.py::test_native_pong_a2c_learns > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E |FAILED" $O/t.log | head -12; [ $rc -eq 0 ] || exit $rc
for knob in 1 0 1; do
  ACA_MLP_FUSED_OPT=$knob timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 > $O/c.jsonl 2> $O/c.err || { tail -3 $O/c.err; exit 1; }
  echo "[ACA_MLP_FUSED_OPT=$knob] $(tail -n 1 $O/c.jsonl)"
done
timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b.json 2> $O/b.err && cat $O/b.json
timeout -k 10 300 bash scripts/gpu_job_trace.sh mujoco mlp_rollout 1 10 "" python3 scripts/bench_configs.py --configs mujoco_ppo_dp8 && cp gpurun_out/trace/mujoco_summary.txt $O/
timeout -k 10 300 bash scripts/gpu_job_trace.sh breakout pong_policy_step 128 2 "" python3 scripts/bench_configs.py --configs breakout_ppo --updates 4 && cp gpurun_out/trace/breakout_summary.txt $O/
