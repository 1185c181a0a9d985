#!/bin/bash
# Round-3 job F: Breakout PPO update time over the kernel / stream-schedule knobs (20 updates each).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
i=0
for knobs in "" "ACA_SERIAL_BWD=1" "ACA_SERIAL_BWD=1 ACAMD_GEMM32=0" "ACA_SERIAL_BWD=1 ACA_WGRAD_GEMM=0" "ACA_WGRAD_GEMM=0 ACAMD_GEMM32=0"; do
  i=$((i+1))
  env $knobs timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/br$i.jsonl 2> $O/br$i.err || { tail -3 $O/br$i.err; exit 1; }
  echo "[$knobs] $(python3 -c "import json;d=json.loads(open('$O/br$i.jsonl').read().splitlines()[-1]);print(d['ms_per_update'])")"
done
timeout -k 10 400 python -u -m pytest tests/test_a3c_gpu_mode.py tests/test_gpu_r3.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/a3c.log 2>&1
rc=$?; echo "a3c/r3 tests rc=$rc"; grep -E "passed|failed" $O/a3c.log | tail -2; grep -E "^E " $O/a3c.log | head -10
