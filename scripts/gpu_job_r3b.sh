#!/bin/bash
# Round-3 job B: new kernel tests first, then the full GPU suite, headline bench A/B, Breakout PPO bench (new wgrad
# kernel A/B), Pendulum learning sweep.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
python -c "from actor_critic_algs_on_tensorflow_amd import _native; _native.load(raise_on_error=True)" || exit 3
timeout -k 10 300 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_dp.py -k "rccl or r3 or wgrad_gemm or finalize_opt" -m gpu -x -v --timeout 120 --timeout-method thread > $O/new.log 2>&1
rc=$?; echo "new tests rc=$rc"; grep -E "passed|failed" $O/new.log | tail -2; grep -E "^E |FAILED" $O/new.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
ACA_FUSED_FINOPT=0 timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 > $O/bench_nofuse.json 2> $O/bench_nofuse.err || exit 1
cat $O/bench_nofuse.json
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/br.jsonl 2> $O/br.err || { tail -5 $O/br.err; exit 1; }
tail -n 2 $O/br.jsonl
ACA_WGRAD_GEMM=0 ACAMD_GEMM32=0 timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/br_old.jsonl 2> $O/br_old.err || exit 1
tail -n 2 $O/br_old.jsonl
ACAMD_GEMM32=0 timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo > $O/br_wg.jsonl 2> $O/br_wg.err || exit 1
tail -n 2 $O/br_wg.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "FAILED" $O/tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/pendulum_sweep.py --updates 10000 --out $O/pend > $O/sweep.jsonl 2> $O/sweep.err
grep summary $O/sweep.jsonl
