#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4be
timeout -k 10 200 python3 -u scripts/exp/opt_ab.py --save gpurun_out/r4be/opt_old.pt > gpurun_out/r4be/old.log 2>&1
