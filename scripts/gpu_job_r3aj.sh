#!/bin/bash
# Round-3 job AJ: measured GEMM plans for the Breakout PPO shapes (best of 3 tuning rounds, the headline's stored
# plans kept) -> gpurun_out/r3aj/plans.json; Breakout / headline benches with that file vs the shipped one.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3aj
mkdir -p $O
timeout -k 10 600 python -u scripts/dump_gemm_plans.py --configs breakout_ppo --rounds 3 --keep-existing --out $O/plans.json > $O/dump.log 2>&1 || { tail -5 $O/dump.log; exit 1; }
tail -1 $O/dump.log
for p in new old new old; do
  if [ $p = new ]; then export ACAMD_GEMM_PLANS=$O/plans.json; else unset ACAMD_GEMM_PLANS; fi
  timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/c.jsonl 2> $O/c.err || { tail -3 $O/c.err; exit 1; }
  echo "[breakout plans=$p] $(python3 -c "import json;d=json.loads(open('$O/c.jsonl').read().splitlines()[-1]);print(d['ms_per_update'])")"
done
export ACAMD_GEMM_PLANS=$O/plans.json
timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
echo "[pong plans=new] $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'])")"
