# PMC passes of the fast path's kernels at HEAD (bytes per kernel, wave waits)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s38; mkdir -p $O
cd /tmp; export PYTHONPATH=$R
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_LDS" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc $set --output-format csv -d $O/pmc/p$i -o run -- python3 $R/bench.py --steps 4 --warmup 2 > $O/pmc_p$i.log 2>&1 || { echo "pmc pass $i rc=$?"; tail -3 $O/pmc_p$i.log; exit 1; }
  echo "pmc pass $i ok"
done
python3 $R/tools/pmc_summary.py $O/pmc > $O/pmc_summary.md 2>&1; cat $O/pmc_summary.md
echo done
