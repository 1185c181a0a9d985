#!/bin/bash
# Round-3 job AG: GEMM m/n-contiguous LDS tiles XOR-swizzled (conflict-free transposed reads) vs the
# padded layout (ab/libacamd_base.so): GEMM / conv / engine tests, headline + Breakout A/B, LDS counters.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3ag
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or conv or production_batch or deterministic or trunk or fc or wgrad or ppo" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E |FAILED" $O/t.log | head -12; [ $rc -eq 0 ] || exit $rc
for lib in "" base "" base; do
  if [ -n "$lib" ]; then export ACAMD_LIB=ab/libacamd_base.so; else unset ACAMD_LIB; fi
  timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  echo "[pong ${lib:-new}] $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'])")"
done
for lib in "" base "" base; do
  if [ -n "$lib" ]; then export ACAMD_LIB=ab/libacamd_base.so; else unset ACAMD_LIB; fi
  timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/c.jsonl 2> $O/c.err || { tail -3 $O/c.err; exit 1; }
  echo "[breakout ${lib:-new}] $(python3 -c "import json;d=json.loads(open('$O/c.jsonl').read().splitlines()[-1]);print(d['ms_per_update'])")"
done
unset ACAMD_LIB
for lib in new base; do
  if [ $lib = base ]; then export ACAMD_LIB=ab/libacamd_base.so; fi
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d $O/pmc_$lib -o run -- python3 bench.py --steps 20 --warmup 5 > $O/pmc_$lib.log 2>&1 || { tail -5 $O/pmc_$lib.log; exit 1; }
done
find $O -name "*.csv" -size +8M -delete
echo done
