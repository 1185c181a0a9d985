#!/bin/bash
# the reference A3C update at the reference geometry (whole 200-step Pendulum-v0 episodes,
# 1200-step batches, L = 40, lr cap 0.1), desired_kl swept over {5e-4, 1e-3, 2e-3, 5e-3, 1e-2}; each final
# checkpoint (reference variable names) scored by the eval CLI. Then the runner topology (1 PS + 3 workers, gloo,
# one GPU shared) at the best desired_kl, chief checkpoints scored the same way.
# Usage (on the GPU box): bash scripts/gpu.sh TAG cmd=scripts/exp/a3c_sweep.sh   [UPDATES=3000 GSTEPS=3000]
set -o pipefail
O=gpurun_out/a3c_sweep
mkdir -p $O
U=${UPDATES:-3000}
for kl in 5e-4 1e-3 2e-3 5e-3 1e-2; do
  timeout -k 10 400 python -u scripts/a3c_ref_geometry.py --desired-kl $kl --updates $U --reports 30 --device cuda:0 \
    --save $O/model-Pendulum-kl$kl --out $O/kl$kl.jsonl > $O/kl$kl.log 2>&1 || { tail -5 $O/kl$kl.log; exit 1; }
  tail -1 $O/kl$kl.jsonl
  timeout -k 10 200 python -u -m actor_critic_algs_on_tensorflow_amd.cli.test_model Pendulum-v0 \
    $O/model-Pendulum-kl$kl --num_episodes 10 --animate_not > $O/eval_kl$kl.txt 2>&1 || { tail -5 $O/eval_kl$kl.txt; exit 1; }
  echo "kl $kl eval: $(tail -1 $O/eval_kl$kl.txt)"
done
