#!/usr/bin/env bash
# PMC counter passes (one counter set per rocprofv3 run, --kernel-trace/--stats
# only) over a model run through the launcher.
#   MNAME=w2v MODEL_ARGS="--config configs/word2vec_1m_4x4.conf --steps 3 --warmup 2" \
#   SETS="SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES ...|FETCH_SIZE" tools/prof_pmc_model.sh
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
MNAME=${MNAME:-fm}; MODEL_ARGS=${MODEL_ARGS:-"--config configs/fm_10b.conf --steps 3 --warmup 2 --set num_features=1000000000 --set table_stats=0"}
SETS=${SETS:-"SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT|FETCH_SIZE|WRITE_SIZE TCC_EA0_WRREQ_sum|TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_sum"}
rm -rf $OUT/pmc_$MNAME
mkdir -p $OUT/pmc_$MNAME
IFS='|' read -ra SETARR <<< "$SETS"
i=0
for set in "${SETARR[@]}"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --stats --pmc $set --output-format csv -d $OUT/pmc_$MNAME/p$i -o run -- python3 -m swiftsnails_amd.launch $MODEL_ARGS > $OUT/pmc_$MNAME/p$i.log 2>&1 || { tail $OUT/pmc_$MNAME/p$i.log; exit 1; }
done
python tools/pmc_summary.py $OUT/pmc_$MNAME
