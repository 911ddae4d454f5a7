#!/usr/bin/env bash
# Local multi-process cluster on the host (reference src/tools/cluster_test.sh,
# which starts the Hadoop server/worker jobs plus a local master): one master,
# S servers and W workers over TCP loopback, each in its own process.
#   SERVERS=2 WORKERS=2 tools/cluster_test.sh [CONFIG] [--set k=v ...]
set -uo pipefail
cd "$(dirname "$0")/.."
CONF=${1:-configs/dense_lr_cpu.conf}
[ $# -gt 0 ] && shift
S=${SERVERS:-1}
W=${WORKERS:-1}
PORT=${PORT:-$(python -c 'import socket;s=socket.socket();s.bind(("127.0.0.1",0));print(s.getsockname()[1])')}
LOG=${LOG_DIR:-$(mktemp -d "${TMPDIR:-/tmp}/ss_cluster.XXXXXX")}
COMMON=(--config "$CONF" --set "listen_addr=tcp://127.0.0.1:$PORT"
        --set "master_addr=tcp://127.0.0.1:$PORT" --set "expected_node_num=$((S + W))" "$@")
pids=()
python -m swiftsnails_amd.launch --role master "${COMMON[@]}" > "$LOG/master.log" 2>&1 &
mpid=$!
for i in $(seq 1 "$S"); do
  python -m swiftsnails_amd.launch --role server "${COMMON[@]}" > "$LOG/server$i.log" 2>&1 &
  pids+=($!)
done
for i in $(seq 1 "$W"); do
  python -m swiftsnails_amd.launch --role worker "${COMMON[@]}" > "$LOG/worker$i.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}" "$mpid"; do
  wait "$p" || rc=$?
done
echo "cluster finished rc=$rc, logs in $LOG"
exit $rc
