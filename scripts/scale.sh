#!/bin/bash
# Weak-scaling sweep of the headline bench on one node: N = 1, 2, 4, 8 GPUs (one rank per GPU over RCCL/xGMI),
# one JSON line per N on stdout (the bench.py contract). Extra args go to bench.py (e.g. --bucket-dtype bf16,
# --overlap lag1). Usage: scripts/scale.sh [--steps K] [--warmup W] [bench args...]
#   NS="1 2 4 8" PORT=29500 scripts/scale.sh --steps 200 --warmup 20
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
NS=${NS:-"1 2 4 8"}
PORT=${PORT:-29500}
NGPU=$(python3 -c "import torch; print(torch.cuda.device_count())")
for n in $NS; do
  if [ "$n" -gt "$NGPU" ]; then
    echo "skip N=$n: only $NGPU GPUs visible" >&2
    continue
  fi
  if [ "$n" -eq 1 ]; then
    timeout -k 10 600 python3 bench.py --gpus 1 "$@" || exit $?
  else
    timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
      --master-port $((PORT + n)) bench.py --gpus "$n" "$@" || exit $?
  fi
done
