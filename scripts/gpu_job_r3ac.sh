#!/bin/bash
# Round-3 job AC: fused rollout step with the conv2 / conv3 weight fragments requested after the policy head
# (ACA_FUSED_WPOS=2, new default) vs after conv1 (0, the previous default) and at entry (1): tests, phases, bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3ac
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "trunk or fused_step or fused_rollout or a2c or pong or rows or deterministic" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E |FAILED" $O/t.log | head -12; [ $rc -eq 0 ] || exit $rc
for w in 2 0; do
  ACA_FUSED_WPOS=$w timeout -k 10 120 python -u scripts/microbench_fused_step.py --out $O/mb_$w.json > $O/mb_$w.log 2>&1 || { tail -5 $O/mb_$w.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/mb_$w.json'));print('wpos $w', {kk: round(vv,2) for kk,vv in d['pong_fused_step'].items()})"
done
for w in 2 0 1 2 0 1; do
  ACA_FUSED_WPOS=$w timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  echo "[pong wpos=$w] $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'])")"
done
