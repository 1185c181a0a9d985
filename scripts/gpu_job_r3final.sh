#!/bin/bash
# Round-3 final tree: smoke(), full GPU suite, headline bench (driver setting x3 + 400 steps), Breakout / MuJoCo
# PPO configs, headline kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3final
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 bash scripts/gpu_job_full.sh r3final_full || exit 1
cp gpurun_out/r3final_full/*.json gpurun_out/r3final_full/configs.jsonl $O/ 2>/dev/null
grep -E "passed|failed" gpurun_out/r3final_full/tests.log | tail -1 > $O/tests_summary.txt
timeout -k 10 300 bash scripts/gpu_job_trace.sh pong_final pong_fused_step 5 200 "" python3 bench.py --steps 400 --warmup 20 && cp gpurun_out/trace/pong_final_summary.txt $O/
