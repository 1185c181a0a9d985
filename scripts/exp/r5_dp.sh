# DP schedules: GPU DP tests + world-1 benches (headline strict/lag1, PPO configs DP vs not)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5dp; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_r5.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|Error|error" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for a in "" "--dp-world1" "--dp-world1 --bucket-dtype bf16" "--dp-world1 --overlap lag1"; do
  timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 $a > $O/b.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "bench [$a] $(python3 -c "import json;d=json.loads([l for l in open('$O/b.json') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'], d['config']['dp_schedule'])")"
  grep -c -v "^{" $O/b.json || true
done
timeout -k 10 400 python -u scripts/bench_configs.py --configs breakout_ppo,mujoco_ppo_dp8 --updates 5 --warmup 2 > $O/c0.jsonl 2>$O/c.err || { tail -5 $O/c.err; exit 1; }
timeout -k 10 400 python -u scripts/bench_configs.py --configs breakout_ppo,mujoco_ppo_dp8 --updates 5 --warmup 2 --dp-world1 > $O/c1.jsonl 2>>$O/c.err || { tail -5 $O/c.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r5dp/c0.jsonl", "gpurun_out/r5dp/c1.jsonl"):
    for l in open(f):
        d = json.loads(l); print(f[-9:], d["config"], d["ms_per_update"], d["dp_world1"])
PY
