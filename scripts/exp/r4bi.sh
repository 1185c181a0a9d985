#!/bin/bash
# rows fused step with conv1's frame 0..2 k-steps run before the head: bitwise tests, phases, headline
set -o pipefail
O=gpurun_out/r4bi
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_r2.py tests/test_gpu_r3.py tests/test_gpu_r4.py > $O/tests.log 2>&1 && \
timeout -k 10 240 python3 -u scripts/exp/rows_step_phases.py > $O/phases.log 2>&1 && \
for i in 1 2 3; do timeout -k 10 180 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_$i.log 2>&1 || exit 1; done
