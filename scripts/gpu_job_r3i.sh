#!/bin/bash
# Round-3 job I: correctness of the new trunk kernels, then headline early-W A/B and Breakout persistent-forward A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_r3.py -m gpu -x -q --timeout 120 --timeout-method thread -k "persistent" > $O/t0.log 2>&1
rc=$?; echo "persistent trunk test rc=$rc"; grep -E "passed|failed" $O/t0.log | tail -2; grep -E "^E " $O/t0.log | head -5; [ $rc -eq 0 ] || exit $rc
ACA_FUSED_EARLY_W=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_r2.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused or deterministic or trunk" > $O/t.log 2>&1
rc=$?; echo "fused tests (early W) rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E " $O/t.log | head -5; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for e in 0 1; do
    ACA_FUSED_EARLY_W=$e timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b_${e}_${rep}.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
    echo "early=$e rep=$rep $(python3 -c "import json;d=json.load(open('$O/b_${e}_${rep}.json'));print(d['value'], d['ms_per_step'])")"
  done
done
for knobs in "ACA_TRUNK_FWD_PERSIST=0" "ACA_TRUNK_FWD_PERSIST=256" "ACA_TRUNK_FWD_PERSIST=512"; do
  env $knobs timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/br.jsonl 2> $O/br.err || { tail -3 $O/br.err; exit 1; }
  echo "[$knobs] $(tail -n 1 $O/br.jsonl)"
done
