#!/usr/bin/env bash
# Synchronous data-parallel A2C/PPO on one node: one process per GPU over RCCL (torch.distributed "nccl").
#   NGPU=8 PRESET=a2c_dp8 scripts/launch_dp.sh [extra train() overrides as key=value]
NGPU=${NGPU:-8}
PRESET=${PRESET:-a2c_dp8}
PORT=${PORT:-29500}
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPU" --master-addr 127.0.0.1 \
  --master-port "$PORT" -m actor_critic_algs_on_tensorflow_amd.cli.dp_train --preset "$PRESET" "$@"
