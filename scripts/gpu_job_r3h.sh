#!/bin/bash
# Round-3 job H: headline A/B of the fused rollout step's early conv2/conv3 weight loads (+ its bitwise tests).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
ACA_FUSED_EARLY_W=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_r2.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused or deterministic or trunk" > $O/t.log 2>&1
rc=$?; echo "fused tests (early W) rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for e in 0 1; do
    ACA_FUSED_EARLY_W=$e timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b_${e}_${rep}.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
    echo "early=$e rep=$rep $(python3 -c "import json;d=json.load(open('$O/b_${e}_${rep}.json'));print(d['value'], d['ms_per_step'])")"
  done
done
