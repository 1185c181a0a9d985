#!/bin/bash
# round 6: MLP engine SPEC path -- numerics (test_gpu_mlp, learning), MuJoCo-shape PPO bench + kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6mlp}
mkdir -p $O
python -c "from actor_critic_algs_on_tensorflow_amd import _native; _native.load(raise_on_error=True)" || exit 3
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py ${EXTRA_TESTS} -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|error" $O/tests.log | tail -3; grep -E "FAILED|Error" $O/tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 5 --warmup 2 > $O/configs.jsonl 2> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
cat $O/configs.jsonl
bash scripts/gpu.sh ${TAG:-r6mlp} trace=mujoco
