set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tall.log 2>&1 && tail -3 gpurun_out/tall.log && \
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/bench_v.json 2> gpurun_out/bench_v.err && cat gpurun_out/bench_v.json && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 10 --warmup 2 > gpurun_out/configs_v.jsonl 2>&1 && tail -1 gpurun_out/configs_v.jsonl && \
timeout -k 10 120 python -u scripts/microbench_rollout.py > gpurun_out/mb_rollout.json 2>&1 && cat gpurun_out/mb_rollout.json
