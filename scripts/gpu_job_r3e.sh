#!/bin/bash
# Round-3 job E: the reference update (preset a3c, lr cap 0.01) on the native MLP engine vs the torch engine on the
# GPU; kernel microbenchmarks of the Breakout learner products.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 300 python -u scripts/pendulum_sweep.py --configs cap001,cap001_torch --updates 1500 --reports 6 > $O/cap.jsonl 2> $O/cap.err || { tail -3 $O/cap.err; exit 1; }
cat $O/cap.jsonl
timeout -k 10 300 python -u scripts/microbench_r3.py > $O/mb.json 2> $O/mb.err || { tail -5 $O/mb.err; exit 1; }
cat $O/mb.json
