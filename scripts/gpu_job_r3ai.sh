#!/bin/bash
# Round-3 job AI: large-batch policy/value head forward kernel (heads.hip head_fwd, ACA_HEAD_FWD_MIN_B=512 default)
# vs the generic GEMM (ACA_HEAD_FWD_MIN_B=0): tests, Breakout PPO A/B, kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3ai
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "head_fwd or production_batch or ppo or deterministic or index" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E |FAILED" $O/t.log | head -12; [ $rc -eq 0 ] || exit $rc
for k in 512 0 512 0; do
  ACA_HEAD_FWD_MIN_B=$k timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/c.jsonl 2> $O/c.err || { tail -3 $O/c.err; exit 1; }
  echo "[breakout ACA_HEAD_FWD_MIN_B=$k] $(python3 -c "import json;d=json.loads(open('$O/c.jsonl').read().splitlines()[-1]);print(d['ms_per_update'])")"
done
timeout -k 10 300 bash scripts/gpu_job_trace.sh breakout_hf pong_policy_step 128 2 "" python3 scripts/bench_configs.py --configs breakout_ppo --updates 4 && cp gpurun_out/trace/breakout_hf_summary.txt $O/
