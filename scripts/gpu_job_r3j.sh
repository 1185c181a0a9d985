#!/bin/bash
# Round-3 job J: lean-LDS per-env trunk forward (2 workgroups per CU): trunk / engine tests, Breakout A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_r2.py tests/test_gpu_kernels.py tests/test_gpu_learning.py tests/test_gpu_r3.py -m gpu -x -q --timeout 120 --timeout-method thread -k "trunk or fused or engine or persistent" > $O/t.log 2>&1
rc=$?; echo "trunk tests rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E |FAILED" $O/t.log | head -8; [ $rc -eq 0 ] || exit $rc
for knobs in "ACA_TRUNK_FWD_U8=0" "ACA_TRUNK_FWD_U8=1"; do
  for rep in 1 2; do
    env $knobs timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/br.jsonl 2> $O/br.err || { tail -3 $O/br.err; exit 1; }
    echo "[$knobs] $(tail -n 1 $O/br.jsonl)"
  done
done
