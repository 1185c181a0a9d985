#!/bin/bash
# Round-3 job O: fc fold (fc product inside the row-split trunk launch): tests, headline A/B, trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_r2.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -rA -k "fold or a2c_head or fused or bitwise or a2c or trunk" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E |FAILED" $O/t.log | head -12; [ $rc -eq 0 ] || exit $rc
for knob in 1 0 1; do
  ACA_FC_FOLD=$knob timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  echo "[ACA_FC_FOLD=$knob] $(cat $O/b.json)"
done
timeout -k 10 300 bash scripts/gpu_job_trace.sh a2c_pong pong_fused_step 5 200 "" python3 bench.py --steps 400 --warmup 20 && cp gpurun_out/trace/a2c_pong_summary.txt $O/
