#!/bin/bash
# row-split trunk on fragment-ordered weights: GPU suite + headline x3
set -o pipefail
O=gpurun_out/r4bj
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
for i in 1 2 3; do timeout -k 10 180 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_$i.log 2>&1 || exit 1; done
