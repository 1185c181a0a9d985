# headline kernel traces for each EngineOpts JSON in OPTS (';'-separated): per-update kernel summaries
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/htab; mkdir -p $O
IFS=';' read -ra LIST <<< "$OPTS"
i=0
for eo in "${LIST[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr$i -o run -- python3 bench.py --steps 40 \
    --warmup 5 --engine-opts "$eo" > $O/tr$i.log 2>&1 || { tail -5 $O/tr$i.log; exit 1; }
  echo "== $eo"
  python3 scripts/trace_summary.py $(find $O/tr$i -name "*kernel_trace.csv") --updates 30 --marker pong_fused_step \
    --per-update 5 | head -12
  find $O/tr$i -name "*.csv" -size +6M -delete
done
