#!/usr/bin/env bash
# MI355X collective mode: one process per GPU (torchrun over RCCL/xGMI).
#   NGPU=8 tools/run_gpu.sh configs/sparse_lr_1b.conf [--steps N] [--set k=v ...]
set -euo pipefail
cd "$(dirname "$0")/.."
CONF=${1:-configs/sparse_lr_10m.conf}
[ $# -gt 0 ] && shift
NGPU=${NGPU:-1}
PORT=${MASTER_PORT:-29531}
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPU" \
  --master-addr 127.0.0.1 --master-port "$PORT" \
  -m swiftsnails_amd.launch --role gpu --config "$CONF" "$@"
