#!/usr/bin/env bash
# MI355X collective mode: one process per GPU (torchrun over RCCL/xGMI).
#   NGPU=8 tools/run_gpu.sh configs/sparse_lr_1b.conf [--steps N] [--set k=v ...]
# Restart after a failure: MAX_RESTARTS=k relaunches every rank up to k times
# (torchrun); with `resume_from: latest` and `param_backup_period` set, each
# relaunch resumes from the newest complete backup.
set -euo pipefail
cd "$(dirname "$0")/.."
CONF=${1:-configs/sparse_lr_10m.conf}
[ $# -gt 0 ] && shift
NGPU=${NGPU:-1}
PORT=${MASTER_PORT:-29531}
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPU" \
  --max-restarts "${MAX_RESTARTS:-0}" --master-addr 127.0.0.1 --master-port "$PORT" \
  -m swiftsnails_amd.launch --role gpu --config "$CONF" "$@"
