# DP tail stage at the PPO learner batch: dWfc planes + finaliser vs the in-launch split reduction (world 1)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/dptail; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py -x -q --timeout 200 --timeout-method thread -k "ppo or rccl" \
  > $O/tests.log 2>&1 || { grep -E "FAILED|Error" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for eo in '{}' '{"dp_tail_planes": false}'; do
  timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 --dp-world1 \
    --engine-opts "$eo" > $O/c.jsonl 2>$O/c.err || { tail -5 $O/c.err; exit 1; }
  echo "breakout dp-world1 $eo $(python3 -c "import json;d=json.loads(open('$O/c.jsonl').readlines()[-1]);print(d['ms_per_update'])")"
done
done
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 > $O/c.jsonl 2>$O/c.err || { tail -5 $O/c.err; exit 1; }
echo "breakout plain $(python3 -c "import json;d=json.loads(open('$O/c.jsonl').readlines()[-1]);print(d['ms_per_update'])")"
