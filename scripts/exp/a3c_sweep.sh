#!/bin/bash
# the reference A3C update at the reference geometry (whole 200-step Pendulum-v0 episodes,
# 1200-step batches, L = 40, lr cap 0.1), desired_kl swept over {5e-4, 1e-3, 2e-3, 5e-3, 1e-2} on two seeds (one
# that learns and one that collapses at the default 2e-3 in the CPU runs of profiles/r4_a3c_parity_and_seeds.txt);
# each final checkpoint (reference variable names) scored by the eval CLI.
# Usage (on the GPU box): bash scripts/gpu.sh TAG cmd=scripts/exp/a3c_sweep.sh   [UPDATES=3000 SEEDS="3 4"]
set -o pipefail
O=gpurun_out/a3c_sweep
mkdir -p $O
U=${UPDATES:-3000}
for seed in ${SEEDS:-3 4}; do
  for kl in 5e-4 1e-3 2e-3 5e-3 1e-2; do
    t=s${seed}_kl$kl
    timeout -k 10 300 python -u scripts/a3c_ref_geometry.py --desired-kl $kl --updates $U --reports 30 --seed $seed \
      --device cuda:0 --save $O/model-Pendulum-$t --out $O/$t.jsonl > $O/$t.log 2>&1 || { tail -5 $O/$t.log; exit 1; }
    timeout -k 10 200 python -u -m actor_critic_algs_on_tensorflow_amd.cli.test_model Pendulum-v0 \
      $O/model-Pendulum-$t --num_episodes 10 --animate_not > $O/eval_$t.txt 2>&1 || { tail -5 $O/eval_$t.txt; exit 1; }
    echo "seed $seed kl $kl: $(tail -1 $O/$t.jsonl | cut -c1-160) | eval: $(tail -1 $O/eval_$t.txt)"
  done
done
