set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_kernels.py tests/test_gpu_dp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t1.log 2>&1 && tail -3 gpurun_out/t1.log && \
timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 > gpurun_out/bench1.json 2> gpurun_out/bench1.err && cat gpurun_out/bench1.json && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8,breakout_ppo --updates 10 --warmup 2 > gpurun_out/configs1.jsonl 2>&1 && cat gpurun_out/configs1.jsonl && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mujoco -o run -- python3 scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 3 --warmup 1 > gpurun_out/prof_mujoco.log 2>&1 && echo prof_ok
