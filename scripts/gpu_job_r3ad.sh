#!/bin/bash
# Round-3 job AD: MuJoCo-shape PPO with Adam folded into the MLP weight-gradient launch behind the XCD-sharded grid
# barrier (ACA_MLP_FUSED_OPT=1) vs weight-gradient launch + opt_multi (0): tests, A/B, kernel trace of the fused form.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3ad
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_mlp.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused_adam or shadows" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E |FAILED" $O/t.log | head -12; [ $rc -eq 0 ] || exit $rc
for k in 1 0 1 0; do
  ACA_MLP_FUSED_OPT=$k timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 > $O/c.jsonl 2> $O/c.err || { tail -3 $O/c.err; exit 1; }
  echo "[mujoco ACA_MLP_FUSED_OPT=$k] $(python3 -c "import json;d=json.loads(open('$O/c.jsonl').read().splitlines()[-1]);print(d['ms_per_update'])")"
done
timeout -k 10 300 bash scripts/gpu_job_trace.sh mujoco_fused mlp_rollout 1 4 "ACA_MLP_FUSED_OPT=1" python3 scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 4 && cp gpurun_out/trace/mujoco_fused_summary.txt $O/
