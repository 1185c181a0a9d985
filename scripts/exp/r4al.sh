# Finaliser with 64-plane load rounds for many-plane jobs: GPU suite, Breakout PPO + trace, headline.
set -o pipefail
O=gpurun_out/${TAG:-r4al}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 && \
timeout -k 10 300 python -u bench.py --steps 400 --warmup 20
