# Adam step offsets for the MLP PPO learner: the new bitwise test + the GPU suite, MuJoCo A/B.
set -o pipefail
O=gpurun_out/${TAG:-r4as}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_r4.py -x -q --timeout 120 --timeout-method thread -k "adam_step_offsets" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 5 --warmup 2 && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 5 --warmup 2 --engine-opts '{"adam_step_offsets": false}' && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 5 --warmup 2
