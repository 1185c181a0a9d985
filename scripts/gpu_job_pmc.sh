#!/bin/bash
# PMC / roofline passes for the headline (pong A2C) and Breakout PPO configs: one counter group per rocprofv3 run,
# the program directly after --, CSV output summarised on the box (raw CSVs kept small; large ones removed).
# Usage: bash scripts/gpu_job_pmc.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-pmc}
O=gpurun_out/$TAG
mkdir -p $O
PONG="python3 bench.py --steps 20 --warmup 5"
BR="python3 scripts/bench_configs.py --configs breakout_ppo --updates 1 --warmup 1"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
run() {   # name, seconds, counters..., -- program
  local name=$1 secs=$2; shift 2
  local pmc=()
  while [ "$1" != "--" ]; do pmc+=("$1"); shift; done; shift
  timeout -s KILL $secs rocprofv3 --kernel-trace --output-format csv --pmc "${pmc[@]}" -d $O/$name -o run -- "$@" \
    > $O/$name.log 2>&1 || { echo "FAIL $name rc=$?"; tail -5 $O/$name.log; return 1; }
  echo "ok $name"
}
run pong_sq 120 $SQ -- $PONG && \
run pong_fetch 120 FETCH_SIZE GRBM_GUI_ACTIVE -- $PONG && \
run pong_write 120 WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -- $PONG && \
python3 scripts/pmc_table.py $(find $O/pong_sq $O/pong_fetch $O/pong_write -name "*counter_collection.csv") \
  > $O/pong_pmc_table.txt && cat $O/pong_pmc_table.txt && \
run br_sq 200 $SQ -- $BR && \
run br_fetch 200 FETCH_SIZE GRBM_GUI_ACTIVE -- $BR && \
python3 scripts/pmc_table.py --last 4 $(find $O/br_sq $O/br_fetch -name "*counter_collection.csv") \
  > $O/br_pmc_table.txt && cat $O/br_pmc_table.txt
rc=$?
# keep the summaries; drop raw CSVs over 8 MB so the copy-back stays under its cap
find $O -name "*.csv" -size +8M -delete
du -sh $O
exit $rc
