#!/bin/bash
# per-env fused step phase stamps: fragment-ordered vs row-major conv2/conv3 weights
set -o pipefail
mkdir -p gpurun_out/r4ay
timeout -k 10 240 python3 -u scripts/exp/env_step_phases.py > gpurun_out/r4ay/phases.log 2>&1
