#!/bin/bash
# Round-3 job D: Breakout PPO kernel traces (new wgrad / GEMM32 kernels vs round-2 kernels), then the full GPU suite.
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpu_job_trace.sh br_new mb_gather_kernel 16 3 "" python -u scripts/bench_configs.py --configs breakout_ppo --updates 6 --warmup 1 || exit 1
bash scripts/gpu_job_trace.sh br_old mb_gather_kernel 16 3 "ACA_WGRAD_GEMM=0 ACAMD_GEMM32=0" python -u scripts/bench_configs.py --configs breakout_ppo --updates 6 --warmup 1 || exit 1
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "FAILED" $O/tests.log | head -20
exit $rc
