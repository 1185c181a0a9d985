# gemm_big variants + Breakout A/B (ppo_head stats fix, gemm_big on/off)
set -o pipefail
timeout -k 10 300 python -u scripts/exp/gemm_big_bench.py && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 --engine-opts '{"big_gemm_min_b": 0}' && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 --engine-opts '{"ppo_head": false}'
