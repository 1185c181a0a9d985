#!/bin/bash
# Round-3 job AA: row-split trunk with conv1 / conv2 / conv3 A fragments read ahead of the MFMAs: trunk tests,
# in-kernel phase stamps and a headline A/B against the previous build (ab/libacamd_base.so).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3aa
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "trunk or fused_step or fused_rollout or production_batch or a2c or pong or rows" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E |FAILED" $O/t.log | head -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/microbench_fused_step.py --out $O/mb_new.json > $O/mb_new.log 2>&1 || { tail -5 $O/mb_new.log; exit 1; }
ACAMD_LIB=ab/libacamd_base.so timeout -k 10 120 python -u scripts/microbench_fused_step.py --out $O/mb_base.json > $O/mb_base.log 2>&1 || { tail -5 $O/mb_base.log; exit 1; }
python3 -c "
import json
for t in ('base','new'):
    d=json.load(open('$O/mb_%s.json'%t))
    print(t, {k: {kk: round(vv,2) for kk,vv in v.items()} for k,v in d.items()})
"
for lib in "" base "" base; do
  if [ -n "$lib" ]; then export ACAMD_LIB=ab/libacamd_base.so; else unset ACAMD_LIB; fi
  timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  echo "[pong ${lib:-new}] $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'])")"
done
