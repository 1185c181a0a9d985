# conv1 fold A/B: its tests, the headline at 400 steps (two rounds), Breakout PPO updates
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fold; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_r5.py \
  -k "conv1_fold" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
OPTS='{"conv1_fold": true};{"conv1_fold": false}' bash scripts/exp/r5_sweep.sh || exit 1
for eo in '{"conv1_fold": true}' '{"conv1_fold": false}'; do
  timeout -k 10 200 python -u scripts/bench_configs.py --configs breakout_ppo --updates 10 --warmup 2 \
    --engine-opts "$eo" > $O/br.log 2>&1 || { tail -5 $O/br.log; exit 1; }
  echo "breakout $eo: $(tail -1 $O/br.log)"
done
