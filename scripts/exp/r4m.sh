# Instruction mix / stall breakdown of the PPO-learner trunk kernels (scripts/exp/trunk_mix.py): three PMC passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4m}
mkdir -p $O
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
P3="SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
timeout -k 10 120 python3 scripts/exp/trunk_mix.py && \
for i in 1 2 3; do
  eval "C=\$P$i"
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $C -d $O/p$i -o run -- python3 scripts/exp/trunk_mix.py > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
python3 scripts/exp/pmc_mix_table.py $(find $O -name "*counter_collection.csv") | tee $O/mix.txt
