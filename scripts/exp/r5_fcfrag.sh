# rollout fc on the fragment-ordered Wfc written by the optimiser: tests, A/B of variants, trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5fcfrag; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_r5.py tests/test_gpu_r4.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
for eo in '{}' '{"fc_frag": 1}' '{"fc_frag": 5}' '{"fc_frag": 3}'; do
  timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 --engine-opts "$eo" > $O/b.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "$eo $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'])")"
done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --steps 40 --warmup 5 --engine-opts '{"fc_frag": 1}' > $O/tr.log 2>&1 || exit 1
python3 scripts/trace_summary.py $(find $O/tr -name "*kernel_trace.csv") --updates 30 --marker pong_fused_step --per-update 5 > $O/sum.txt && head -16 $O/sum.txt
find $O/tr -name "*.csv" -size +6M -delete
