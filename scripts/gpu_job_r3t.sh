#!/bin/bash
# Round-3 job T: fc plane reduce with 16 loads in flight per round + a2c_head bootstrap over the whole workgroup.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3t
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_r2.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "a2c or fused or bitwise or fc_parts or policy or planes" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E |FAILED" $O/t.log | head -12; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  echo "[bench] $(cat $O/b.json)"
done
timeout -k 10 120 python -u scripts/microbench_fused_step.py --out $O/mb_step.json > $O/mb.log 2>&1 && cat $O/mb_step.json
timeout -k 10 120 python -u scripts/microbench_a2c_head.py --out $O/mb_head.json > $O/mbh.log 2>&1 && cat $O/mb_head.json
timeout -k 10 300 bash scripts/gpu_job_trace.sh a2c_pong pong_fused_step 5 200 "" python3 bench.py --steps 400 --warmup 20 && cp gpurun_out/trace/a2c_pong_summary.txt $O/
