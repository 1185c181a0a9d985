# late round-5 A/B: finaliser job split on the headline (400 and 20 steps), MuJoCo DP world-1 self-norm
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/late; mkdir -p $O
OPTS='{};{"fin_split": false}' bash scripts/exp/r5_sweep.sh || exit 1
for r in 1 2; do
for eo in '{}' '{"fin_split": false}'; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --engine-opts "$eo" > $O/b.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "bench20 $eo $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'])")"
done
done
for eo in '{"dp_self_norm": true}' '{"dp_self_norm": false}'; do
  timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 5 --warmup 2 --dp-world1 \
    --engine-opts "$eo" > $O/mj.jsonl 2>$O/mj.err || { tail -5 $O/mj.err; exit 1; }
  echo "mujoco dp-world1 $eo $(python3 -c "import json;d=json.loads(open('$O/mj.jsonl').readlines()[-1]);print(d['ms_per_update'])")"
done
