set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5fct; mkdir -p $O
for v in 1 5; do
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o run -- python3 bench.py --steps 40 --warmup 5 --engine-opts "{\"fc_frag\": $v}" > $O/tr_$v.log 2>&1 || exit 1
python3 scripts/trace_summary.py $(find $O/tr_$v -name "*kernel_trace.csv") --updates 30 --marker pong_fused_step --per-update 5 > $O/sum_$v.txt && head -16 $O/sum_$v.txt
find $O/tr_$v -name "*.csv" -size +6M -delete
done
