#!/bin/bash
# Round-3 job U: a2c_head / fc_value with one round of plane loads; fused MLP Adam with the XCD-sharded barrier.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3u
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_r2.py tests/test_gpu_mlp.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "a2c or fused or bitwise or fc_parts or policy or planes or shadows" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E |FAILED" $O/t.log | head -12; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  echo "[bench] $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 120 python -u scripts/microbench_a2c_head.py --out $O/mb_head.json > $O/mbh.log 2>&1 && python3 -c "import json;d=json.load(open('$O/mb_head.json'));print(d['a2c_head_boot'], d['phases_boot'])"
for knob in 1 0 1; do
  ACA_MLP_FUSED_OPT=$knob timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 > $O/c.jsonl 2> $O/c.err || { tail -3 $O/c.err; exit 1; }
  echo "[ACA_MLP_FUSED_OPT=$knob] $(python3 -c "import json;d=json.loads(open('$O/c.jsonl').read().splitlines()[-1]);print(d['ms_per_update'])")"
done
