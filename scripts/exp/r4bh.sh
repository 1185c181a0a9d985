#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4bh
timeout -k 10 240 python3 -u scripts/exp/rows_step_phases.py > gpurun_out/r4bh/phases.log 2>&1
