# MLP engine A/B: its GPU tests, then MuJoCo PPO updates for each EngineOpts JSON in OPTS (';'-separated), two rounds
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mlpab; mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mlp.py \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
IFS=';' read -ra LIST <<< "$OPTS"
for r in 1 2; do
for eo in "${LIST[@]}"; do
  timeout -k 10 200 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 6 --warmup 2 \
    --engine-opts "$eo" > $O/mj.log 2>&1 || { tail -5 $O/mj.log; exit 1; }
  echo "mujoco $eo: $(python3 -c "import json;d=json.loads(open('$O/mj.log').read().strip().splitlines()[-1]);print(d['ms_per_update'])")"
done
done
