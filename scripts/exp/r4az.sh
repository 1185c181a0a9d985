#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4az
timeout -k 10 300 python3 -u scripts/exp/fc_bwd_b160.py > gpurun_out/r4az/fc_bwd.log 2>&1
