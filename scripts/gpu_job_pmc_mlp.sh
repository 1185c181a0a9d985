#!/bin/bash
# PMC pass over the MLP engine microbenchmarks (rollout kernel, train kernel): MFMA busy, LDS conflicts, waits.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_mlp
mkdir -p $O
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc $SQ -d $O/roll -o run -- python3 scripts/microbench_rollout.py > $O/roll.log 2>&1 || { echo FAIL roll; tail -5 $O/roll.log; exit 1; }
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc $SQ -d $O/train -o run -- python3 scripts/microbench_mlp_train.py > $O/train.log 2>&1 || { echo FAIL train; tail -5 $O/train.log; exit 1; }
python3 scripts/pmc_table.py $(find $O/roll -name "*counter_collection.csv") > $O/roll_table.txt 2>&1; head -20 $O/roll_table.txt
python3 scripts/pmc_table.py $(find $O/train -name "*counter_collection.csv") > $O/train_table.txt 2>&1; head -20 $O/train_table.txt
for f in $(find $O -name "*counter_collection.csv"); do python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in rows:
    k = r.get("Kernel_Name", r.get("Kernel-Name", ""))[:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[k] += 1
for k, d in agg.items():
    if "mlp" in k: print(k, {c: round(v) for c, v in sorted(d.items())})
PY
done
find $O -name "*.csv" -size +6M -delete
