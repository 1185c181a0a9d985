# 1024 norm-partial slots + quarter-plane finaliser jobs: the GPU tests from where r4am stopped, then all, benches.
set -o pipefail
O=gpurun_out/${TAG:-r4an}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_r2.py tests/test_gpu_r4.py -x -q --timeout 120 --timeout-method thread > $O/tests_a.log 2>&1; rc=$?; tail -3 $O/tests_a.log; [ $rc -eq 0 ] && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo,mujoco_ppo_dp8 --updates 5 --warmup 2 && \
timeout -k 10 300 python -u bench.py --steps 400 --warmup 20
