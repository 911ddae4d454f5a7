#!/usr/bin/env bash
# PMC counter passes on the 1-GPU bench (counters only with --kernel-trace/--stats).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${ARGS:-"--steps 4 --warmup 2"}
i=0
SETS=${SETS:-"TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_sum|SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM|FETCH_SIZE|WRITE_SIZE TCC_EA0_WRREQ_sum|SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"}
IFS='|' read -ra SETARR <<< "$SETS"
for set in "${SETARR[@]}"; do
  i=$((i+1))
  echo "=== pass $i: $set"
  timeout -s KILL 60 rocprofv3 --kernel-trace --stats --pmc $set --output-format csv -d "$OUT/p$i" -o run -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -3 "$OUT/p$i.log"
  case $rc in 0|1|2) ;; *) echo "FATAL"; exit $rc;; esac
done
