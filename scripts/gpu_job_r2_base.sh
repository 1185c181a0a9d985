#!/bin/bash
# Round-2 baseline on one MI355X: GPU tests, headline bench, kernel trace, and PMC passes (one counter set per
# rocprofv3 run, program directly after --). Writes everything under gpurun_out/r2base/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2base
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?"; tail -3 $O/tests.log
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 > $O/bench.json 2> $O/bench.err && cat $O/bench.json && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench.py --steps 60 --warmup 10 > $O/trace.log 2>&1 && echo trace_ok && \
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $O/pmc_sq -o run -- python3 bench.py --steps 20 --warmup 5 > $O/pmc_sq.log 2>&1 && echo pmc_sq_ok && \
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/pmc_fetch -o run -- python3 bench.py --steps 20 --warmup 5 > $O/pmc_fetch.log 2>&1 && echo pmc_fetch_ok && \
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $O/pmc_write -o run -- python3 bench.py --steps 20 --warmup 5 > $O/pmc_write.log 2>&1 && echo pmc_write_ok && \
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $O/pmc_br_sq -o run -- python3 scripts/bench_configs.py --configs breakout_ppo --updates 2 --warmup 1 > $O/pmc_br_sq.log 2>&1 && echo pmc_br_ok && \
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/pmc_br_fetch -o run -- python3 scripts/bench_configs.py --configs breakout_ppo --updates 2 --warmup 1 > $O/pmc_br_fetch.log 2>&1 && echo pmc_br_fetch_ok
echo "done rc=$?"
find $O -name "*.csv" -o -name "*.db" | head -30
