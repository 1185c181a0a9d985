# Breakout-shape PPO: fc_rollout at 128 envs (A/B), tests of the round-5 kernels
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5br; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_r5.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
DEF='{};{"fc_frag_big": 21};{"fc_frag_big": 17};{"fc_frag_big": 16};{"fc_frag_big": 18}'
IFS=";" read -ra LIST <<< "${BR_OPTS:-$DEF}"
for eo in "${LIST[@]}"; do
  timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 --engine-opts "$eo" > $O/c.jsonl 2>$O/c.err || { tail -5 $O/c.err; exit 1; }
  echo "$eo $(python3 -c "import json;d=json.loads(open('$O/c.jsonl').readlines()[-1]);print(d['ms_per_update'])")"
done
