#!/usr/bin/env bash
# Master role of the host (TCP) cluster — reference src/tools/run_master.sh
# (`./swift_master -config ./master.conf`).
#   tools/run_master.sh [CONFIG] [--set key=value ...]
set -euo pipefail
cd "$(dirname "$0")/.."
CONF=${1:-configs/dense_lr_cpu.conf}
[ $# -gt 0 ] && shift
exec python -m swiftsnails_amd.launch --role master --config "$CONF" "$@"
