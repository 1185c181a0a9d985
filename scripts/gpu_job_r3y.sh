#!/bin/bash
# Round-3 job Y: headline knob sweep over the per-sample / batched-position weight-gradient kernels at B = 160.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3y
mkdir -p $O
for knobs in "" "ACA_NHWC_WGRAD_MIN_B=128 ACA_NHWC3_WGRAD_MIN_B=128" "ACA_CONV1_WGRAD_MIN_B=128" "ACA_NHWC_WGRAD_MIN_B=128 ACA_NHWC3_WGRAD_MIN_B=128 ACA_CONV1_WGRAD_MIN_B=128" "ACA_NHWC_WGRAD_MIN_B=128 ACA_NHWC3_WGRAD_MIN_B=128 ACA_NHWC_PLANES=64 ACA_NHWC3_PLANES=64" ""; do
  env $knobs timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  echo "[pong $knobs] $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'])")"
done
# instruction-cache / issue-wait counters of the headline kernels (one pass, 8 SQ counters)
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY -d $O/pmc -o run -- python3 bench.py --steps 20 --warmup 5 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
echo "[pmc] done"
find $O -name "*.csv" -size +8M -delete
