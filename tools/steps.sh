#!/usr/bin/env bash
# Run GPU steps in order, each under its own time limit, stopping at the first
# fault / abort / timeout.  Usage: tools/steps.sh 'name|seconds|command' ...
# Output of each step: gpurun_out/<name>.log; summary: gpurun_out/steps.log.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "=== $name ($to s): $cmd" | tee -a "$OUT/steps.log"
  t0=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 )) s)" | tee -a "$OUT/steps.log"
  tail -n 12 "$OUT/$name.log"
  case $rc in 0|1|2|5) ;; *) echo "FATAL in $name (rc=$rc): stop" | tee -a "$OUT/steps.log"; exit $rc ;; esac
done
echo "steps done" | tee -a "$OUT/steps.log"
