#!/bin/bash
# the reference A3C runner topology (A3C/runner.sh: 1 PS + 3 workers) on Pendulum-v0 at the
# reference geometry -- each worker update is 6 whole 200-step episodes (1200 steps), L = 40, lr cap 0.1 -- with the
# GPU-native workers sharing one GPU (gloo control plane), the chief checkpointing every 600 global steps; the
# latest chief checkpoint scored by the eval CLI. Usage: SEED=3 bash scripts/exp/a3c_runner_gpu.sh
set -o pipefail
ITERS=${ITERS:-3000}
SEED=${SEED:-12321}
PORT=${PORT:-29631}
O=gpurun_out/a3c_runner/seed$SEED
mkdir -p $O/logs $O/ck
common="--worker_num 3 --ps_num 1 --initport $PORT --max_iters $ITERS --outdir $O/logs --checkpoint_dir $O/ck \
  --device cuda:0 --num_envs 6 --n_steps 200 --seed $SEED --save_every 600 --stdout_freq 100"
timeout -k 10 800 python -u -m actor_critic_algs_on_tensorflow_amd.cli.train ps 0 $common --quiet > $O/ps0.out 2>&1 &
pids=($!)
for i in 0 1 2; do
  timeout -k 10 800 python -u -m actor_critic_algs_on_tensorflow_amd.cli.train worker $i $common > $O/w$i.out 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
[ $rc -eq 0 ] || { echo "runner exit $rc"; tail -5 $O/w0.out $O/ps0.out; exit $rc; }
ls $O/ck
latest=$(ls $O/ck/*.index | sed 's/\.index$//' | sort -t- -k3 -n | tail -1)
echo "latest chief checkpoint: $latest"
timeout -k 10 200 python -u -m actor_critic_algs_on_tensorflow_amd.cli.test_model Pendulum-v0 $latest --num_episodes 10 \
  --animate_not > $O/eval.txt 2>&1 && tail -1 $O/eval.txt
grep -h "avg_rew\|Average" $O/logs/worker_0.log 2>/dev/null | tail -3
tail -3 $O/w0.out
