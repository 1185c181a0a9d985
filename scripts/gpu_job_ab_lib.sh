#!/bin/bash
# A/B of library builds (ACAMD_LIB) on the MLP engine: GPU MLP tests on the last build, then per build the train-kernel
# microbench and the MuJoCo-shape PPO config. Usage: bash scripts/gpu_job_ab_lib.sh v1 v2 ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ablib
mkdir -p $O
last=${@: -1}
export ACAMD_LIB=$PWD/actor_critic_algs_on_tensorflow_amd/_C/libacamd_$last.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_learning.py -x -q --timeout 250 --timeout-method thread -k "mlp or cartpole or mujoco" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -5; exit $rc; }
for v in "$@"; do
  export ACAMD_LIB=$PWD/actor_critic_algs_on_tensorflow_amd/_C/libacamd_$v.so
  timeout -k 10 200 python -u scripts/microbench_mlp_train.py > $O/mb_$v.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u scripts/bench_configs.py --configs mujoco_ppo_dp8 --updates 5 --warmup 2 > $O/cfg_$v.jsonl 2>/dev/null || exit 1
  echo "$v: $(python3 -c "import json;d=json.load(open('$O/mb_$v.json'));print('train', d['train_launch_us'], 'step', d['minibatch_step_us'], 'dg3', d['tower0_us_from_start'].get('dg_3'), 'crit_dg2', d['tower1_us_from_start'].get('dg_2'))") $(python3 -c "import json;print(json.loads(open('$O/cfg_$v.jsonl').read().strip().splitlines()[-1])['ms_per_update'])")"
done
