#!/bin/bash
# Kernel traces (per-update budget) + PMC roofline passes of the headline and Breakout PPO, summaries on the box.
# Usage: bash scripts/gpu_job_prof2.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-prof2}
O=gpurun_out/$TAG
mkdir -p $O
PONG="python3 bench.py --steps 40 --warmup 5"
BR="python3 scripts/bench_configs.py --configs breakout_ppo --updates 2 --warmup 1"
MJ="python3 scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 2 --warmup 1"
SQ="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
trace() {   # name, marker, per-update, updates, program...
  local name=$1 marker=$2 per=$3 upd=$4; shift 4
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$name -o run -- "$@" > $O/$name.log 2>&1 || { echo "FAIL trace $name"; tail -5 $O/$name.log; return 1; }
  python3 scripts/trace_summary.py $(find $O/$name -name "*kernel_trace.csv") --updates $upd --marker $marker --per-update $per > $O/${name}_summary.txt && head -40 $O/${name}_summary.txt
}
pmc() {   # name, tail, counters..., -- program
  local name=$1 tail=$2; shift 2
  local c=()
  while [ "$1" != "--" ]; do c+=("$1"); shift; done; shift
  timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc "${c[@]}" -d $O/$name -o run -- "$@" > $O/$name.log 2>&1 || { echo "FAIL pmc $name"; tail -5 $O/$name.log; return 1; }
  echo "ok $name"
}
trace pong_trace pong_policy_step 5 30 $PONG && \
trace br_trace pong_policy_step 128 1 $BR && \
trace mj_trace mlp_rollout 1 1 $MJ && \
pmc pong_sq 600 $SQ -- $PONG && \
pmc pong_fetch 600 FETCH_SIZE GRBM_GUI_ACTIVE -- $PONG && \
pmc pong_write 600 WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -- $PONG && \
python3 scripts/pmc_table.py --tail 540 $(find $O/pong_sq $O/pong_fetch $O/pong_write -name "*counter_collection.csv") > $O/pong_pmc.txt && cat $O/pong_pmc.txt && \
pmc br_sq 0 $SQ -- $BR && \
pmc br_fetch 0 FETCH_SIZE GRBM_GUI_ACTIVE -- $BR && \
python3 scripts/pmc_table.py --tail 1200 $(find $O/br_sq $O/br_fetch -name "*counter_collection.csv") > $O/br_pmc.txt && cat $O/br_pmc.txt
rc=$?
find $O -name "*.csv" -size +6M -delete
du -sh $O
exit $rc
