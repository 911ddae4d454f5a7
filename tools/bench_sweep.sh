#!/usr/bin/env bash
# bench sensitivity sweep (1 GPU)
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
for a in "$@"; do
  echo "=== bench $a"
  timeout -k 10 300 python bench.py $a 2>&1 | grep -E '^\{|Error|error' | tee -a "$OUT/sweep.log"
  rc=${PIPESTATUS[0]}
  case $rc in 0|1|2) ;; *) echo "FATAL rc=$rc"; exit $rc;; esac
done
