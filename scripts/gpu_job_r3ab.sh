#!/bin/bash
# Round-3 job AB: conv1 sub-phase stamps (probe build ab/libacamd_probe.so: wave 0 after its A-fragment issue and
# after each of its three M tiles).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3ab
mkdir -p $O
ACAMD_LIB=ab/libacamd_probe.so timeout -k 10 120 python -u scripts/microbench_fused_step.py --out $O/mb_probe.json > $O/mb_probe.log 2>&1 || { tail -5 $O/mb_probe.log; exit 1; }
cat $O/mb_probe.json
