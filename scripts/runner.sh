#!/usr/bin/env bash
# A3C launcher (A3C/runner.sh): starts the PS task(s) then the workers as background jobs on this host.
# Every process joins one torch.distributed gloo group at 127.0.0.1:$initport.
env=${env:-Pendulum-v0}
workers=${workers:-3}
ps=${ps:-1}
mode=${mode:-train}
initport=${initport:-2849}
cd "$(dirname "$0")/.."
for ((i=0; i<ps; i++)); do
  python -m actor_critic_algs_on_tensorflow_amd.cli.train ps $i --worker_num $workers --env $env --ps_num $ps \
      --initport $initport &
done
for ((i=0; i<workers; i++)); do
  python -m actor_critic_algs_on_tensorflow_amd.cli.train worker $i --mode $mode --env $env --worker_num $workers \
      --ps_num $ps --initport $initport &
done
wait
