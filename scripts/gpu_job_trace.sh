#!/bin/bash
# Kernel trace + per-update summary of one program under env knobs.
# Usage: bash scripts/gpu_job_trace.sh NAME MARKER PER_UPDATE UPDATES "K=V ..." program...
set -o pipefail
export TMPDIR=/tmp
name=$1 marker=$2 per=$3 upd=$4 knobs=$5; shift 5
O=gpurun_out/trace
mkdir -p $O
for kv in $knobs; do export "$kv"; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$name -o run -- "$@" > $O/$name.log 2>&1 || { echo "FAIL trace $name"; tail -5 $O/$name.log; exit 1; }
python3 scripts/trace_summary.py $(find $O/$name -name "*kernel_trace.csv") --updates $upd --marker $marker --per-update $per > $O/${name}_summary.txt && head -32 $O/${name}_summary.txt
find $O/$name -name "*.csv" -size +6M -delete
