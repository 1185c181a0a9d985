#!/bin/bash
# Round-3 job AK: Breakout PPO PMC table on the final tree (stored GEMM plans: no tuning pass inside the profile).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3ak
mkdir -p $O
BR="python3 scripts/bench_configs.py --configs breakout_ppo --updates 2 --warmup 1"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc $SQ -d $O/br_sq -o run -- $BR > $O/br_sq.log 2>&1 || { tail -5 $O/br_sq.log; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/br_fetch -o run -- $BR > $O/br_fetch.log 2>&1 || { tail -5 $O/br_fetch.log; exit 1; }
python3 scripts/pmc_table.py --last 4 $(find $O/br_sq $O/br_fetch -name "*counter_collection.csv") > $O/br_pmc_table.txt && head -30 $O/br_pmc_table.txt
find $O -name "*.csv" -size +8M -delete
