#!/bin/bash
# fragment-ordered weights A/B on the s16 trunk forward
set -e
mkdir -p gpurun_out/r4at
timeout -k 10 120 python3 -u scripts/exp/trunk_fwd_ab.py > gpurun_out/r4at/ab.log 2>&1
