#!/usr/bin/env bash
# Worker role of the host (TCP) cluster — reference src/tools/run_worker.sh,
# which saves stdin to data.txt and passes `-data data.txt` (Hadoop streaming
# feeds each reducer its split on stdin).  Same here: with no --data argument
# and a non-terminal stdin, stdin is saved to a temporary data file.
#   tools/run_worker.sh [CONFIG] [--app module:Class] [--data FILE] [--set k=v ...]
set -euo pipefail
cd "$(dirname "$0")/.."
CONF=${1:-configs/dense_lr_cpu.conf}
[ $# -gt 0 ] && shift
EXTRA=()
if [[ " $* " != *" --data "* && " $* " != *" -data "* ]] && [ ! -t 0 ]; then
  DATA=$(mktemp "${TMPDIR:-/tmp}/ss_worker_data.XXXXXX")
  trap 'rm -f "$DATA"' EXIT
  cat > "$DATA"
  [ -s "$DATA" ] && EXTRA=(--data "$DATA")
fi
python -m swiftsnails_amd.launch --role worker --config "$CONF" "${EXTRA[@]}" "$@"
