#!/bin/bash
# Round-3 job S: phase stamps of the fused rollout step and the first-observation trunk.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3s
timeout -k 10 120 python -u scripts/microbench_fused_step.py --out gpurun_out/r3s/mb_step.json > gpurun_out/r3s/mb.log 2>&1 || { tail -8 gpurun_out/r3s/mb.log; exit 1; }
cat gpurun_out/r3s/mb_step.json
