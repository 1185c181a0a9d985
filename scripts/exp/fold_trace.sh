# conv1 fold: per-kernel times with the fold on / off (headline, 40 steps)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/foldtr; mkdir -p $O
for k in on off; do
  [ $k = on ] && eo='{"conv1_fold": true}' || eo='{"conv1_fold": false}'
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$k -o run -- python3 bench.py --steps 40 --warmup 5 \
    --engine-opts "$eo" > $O/$k.log 2>&1 || { tail -5 $O/$k.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | sort
