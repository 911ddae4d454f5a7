#!/usr/bin/env bash
# secondary-config throughput on 1 GPU via the launcher (JSON lines -> gpurun_out/models.log)
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
run() {
  echo "=== $*" | tee -a "$OUT/models.log"
  timeout -k 10 400 python -m swiftsnails_amd.launch "$@" 2>&1 | tail -3 | tee -a "$OUT/models.log"
  rc=${PIPESTATUS[0]}
  case $rc in 0|1|2) ;; *) echo "FATAL rc=$rc"; exit $rc;; esac
}
run --config configs/word2vec_1m_4x4.conf --steps 30 --warmup 5 --set server_ranks=all --set worker_ranks=all
run --config configs/fm_10b.conf --steps 30 --warmup 5 --set num_features=1000000000
run --config configs/sparse_lr_10m.conf --steps 30 --warmup 5
