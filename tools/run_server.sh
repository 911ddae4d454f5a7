#!/usr/bin/env bash
# Server role of the host (TCP) cluster — reference src/tools/run_server.sh.
#   tools/run_server.sh [CONFIG] [--dim D] [--set key=value ...]
set -euo pipefail
cd "$(dirname "$0")/.."
CONF=${1:-configs/dense_lr_cpu.conf}
[ $# -gt 0 ] && shift
exec python -m swiftsnails_amd.launch --role server --config "$CONF" "$@"
