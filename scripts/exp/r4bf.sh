#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4bf
timeout -k 10 200 python3 -u scripts/exp/opt_ab.py --ref tmp_optab/opt_old.pt > gpurun_out/r4bf/new.log 2>&1
