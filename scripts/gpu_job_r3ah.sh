#!/bin/bash
# Round-3 job AH: per-operand runtime vector flags in the non-VEC GEMM instantiations (the aligned operand of a
# product against an unaligned [512, A+1] head weight moves in 16-byte loads) vs the previous build
# (ab/libacamd_base.so): GEMM / engine tests, Breakout PPO A/B, Breakout kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3ah
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or conv or production_batch or deterministic or ppo or head" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/t.log | tail -2; grep -E "^E |FAILED" $O/t.log | head -12; [ $rc -eq 0 ] || exit $rc
for lib in "" base "" base; do
  if [ -n "$lib" ]; then export ACAMD_LIB=ab/libacamd_base.so; else unset ACAMD_LIB; fi
  timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/c.jsonl 2> $O/c.err || { tail -3 $O/c.err; exit 1; }
  echo "[breakout ${lib:-new}] $(python3 -c "import json;d=json.loads(open('$O/c.jsonl').read().splitlines()[-1]);print(d['ms_per_update'])")"
done
unset ACAMD_LIB
timeout -k 10 300 bash scripts/gpu_job_trace.sh breakout_vec pong_policy_step 128 2 "" python3 scripts/bench_configs.py --configs breakout_ppo --updates 4 && cp gpurun_out/trace/breakout_vec_summary.txt $O/
