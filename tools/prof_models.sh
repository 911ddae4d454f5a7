#!/usr/bin/env bash
# rocprofv3 kernel stats for the secondary models (1 GPU) -> gpurun_out/prof_<model>/
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
export TMPDIR=/tmp
prof() {
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${name}${SUFFIX:-}" -o run \
    -- python3 -m swiftsnails_amd.launch "$@" > "$OUT/prof_${name}${SUFFIX:-}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1|2) ;; *) exit $rc;; esac
}
prof fm --config configs/fm_10b.conf --steps 10 --warmup 3 --set num_features=1000000000 --set table_stats=0
prof w2v --config configs/word2vec_1m_4x4.conf --steps 10 --warmup 3 --set server_ranks=all --set worker_ranks=all --set table_stats=0
