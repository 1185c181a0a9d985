#!/bin/bash
# ppo_head without its last-arriver ticket (statistics summed by the finaliser) + padded LDS planes: tests, Breakout,
# and the head's kernel time / LDS conflicts
set -o pipefail
O=gpurun_out/phead; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_r4.py \
  tests/test_gpu_learning.py tests/test_gpu_dp.py tests/test_gpu_r3.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 2>/dev/null | cut -c1-120 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc -o run -- \
  python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py --configs breakout_ppo --updates 2 --warmup 1 > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, os, collections
root = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/phead/pmc"
f = glob.glob(root + "/**/*counter_collection.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if "ppo_head" in r["Kernel_Name"] or "grad_finalize" in r["Kernel_Name"]:
        agg[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    c, a = v.get("SQ_LDS_BANK_CONFLICT", 0), v.get("SQ_LDS_IDX_ACTIVE", 0)
    print(k, "ldsC% =", round(100 * c / a, 1) if a else None)
PY
