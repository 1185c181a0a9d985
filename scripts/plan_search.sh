#!/bin/bash
# End-to-end GEMM plan selection: isolated per-shape tuning does not always pick the plan set that is fastest
# inside the captured update (cache state, co-running side-stream kernels). Run the headline bench N times with
# fresh tuning, record each run's plans, re-measure every plan set, and keep the fastest as gemm_plans.json.
# Usage: bash scripts/plan_search.sh N
set -o pipefail
export TMPDIR=/tmp
N=${1:-5}
O=gpurun_out/ps
mkdir -p $O
for i in $(seq 1 $N); do
  ACAMD_GEMM_PLANS=0 ACA_BENCH_SAVE_PLANS=$O/plans_$i.json timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 \
      > $O/fresh_$i.json 2> $O/fresh_$i.err || { tail -5 $O/fresh_$i.err; exit 1; }
  echo "fresh $i: $(python3 -c "import json;print(json.load(open('$O/fresh_$i.json'))['value'])")"
done
for rep in 1 2; do
  for i in $(seq 1 $N); do
    ACAMD_GEMM_PLANS=$O/plans_$i.json timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 \
        > $O/re_${i}_$rep.json 2> $O/re_${i}_$rep.err || { tail -5 $O/re_${i}_$rep.err; exit 1; }
    echo "replay plans_$i rep $rep: $(python3 -c "import json;print(json.load(open('$O/re_${i}_$rep.json'))['value'])")"
  done
done
