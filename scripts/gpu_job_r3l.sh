#!/bin/bash
# Round-3 job L: a2c_head (bootstrap value + A2C head in one 32-workgroup launch): tests, headline A/B, trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_r2.py -m gpu -x -q --timeout 120 --timeout-method thread -k "a2c_head or fused_head or bitwise or a2c" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E |FAILED" $O/t.log | head -12; [ $rc -eq 0 ] || exit $rc
for knob in 1 0 1; do
  ACA_A2C_HEAD=$knob timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  echo "[ACA_A2C_HEAD=$knob] $(cat $O/b.json)"
done
timeout -k 10 300 bash scripts/gpu_job_trace.sh a2c_pong pong_fused_step 5 200 "" python3 bench.py --steps 400 --warmup 20 && cp gpurun_out/trace/a2c_pong_summary.txt $O/
