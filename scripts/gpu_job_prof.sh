set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pong -o run -- python3 bench.py --steps 60 --warmup 10 > gpurun_out/prof_pong.log 2>&1 && echo pong_ok && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mj -o run -- python3 scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 4 --warmup 1 > gpurun_out/prof_mj.log 2>&1 && echo mj_ok && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_br -o run -- python3 scripts/bench_configs.py --configs breakout_ppo --updates 4 --warmup 1 > gpurun_out/prof_br.log 2>&1 && echo br_ok
