#!/bin/bash
# A3C CartPole learning test on the previous optimiser kernel (A/B of the operand-load reorder)
set -o pipefail
O=gpurun_out/r4bd
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_a3c_gpu_mode.py -k learns -x -q --timeout 300 --timeout-method thread > $O/run1.log 2>&1 ; true
