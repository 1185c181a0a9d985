set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t2.log 2>&1 && tail -3 gpurun_out/t2.log && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 10 --warmup 2 > gpurun_out/configs2.jsonl 2>&1 && cat gpurun_out/configs2.jsonl && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mujoco2 -o run -- python3 scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 3 --warmup 1 > gpurun_out/prof_mujoco2.log 2>&1 && echo prof_ok
