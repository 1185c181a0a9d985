#!/bin/bash
# Round-3 job N: a2c_head phase stamps, then the learning-stability sweep (job M).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3n
timeout -k 10 120 python -u scripts/microbench_a2c_head.py --out gpurun_out/r3n/mb_head.json > gpurun_out/r3n/mb.log 2>&1 || { tail -5 gpurun_out/r3n/mb.log; exit 1; }
cat gpurun_out/r3n/mb_head.json
bash scripts/gpu_job_r3m.sh
