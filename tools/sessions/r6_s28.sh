# the N>1 path at one rank with the default SS_XCHG=auto (records): serial + pipelined kernel stats, PMC passes of the record path's kernels
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s28; mkdir -p $O
cd /tmp; export PYTHONPATH=$R
export SS_ENGINE_GENERAL=xgmi
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/ser -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/ser.log 2>&1 || { tail $O/ser.log; exit 1; }
python3 $R/tools/kstats.py --range timed $O/ser > $O/ser_stats.txt 2>&1; head -20 $O/ser_stats.txt
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/pipe -o run -- python3 $R/bench.py --steps 24 --warmup 8 > $O/pipe.log 2>&1 || { tail $O/pipe.log; exit 1; }
python3 $R/tools/kstats.py --range timed $O/pipe > $O/pipe_stats.txt 2>&1; head -20 $O/pipe_stats.txt
export SS_XCHG=records
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc $set --output-format csv -d $O/pmc/p$i -o run -- python3 $R/bench.py --steps 4 --warmup 2 --cal-steps 0 > $O/pmc_p$i.log 2>&1 || { echo "pmc pass $i rc=$?"; tail -3 $O/pmc_p$i.log; exit 1; }
  echo "pmc pass $i ok"
done
python3 $R/tools/pmc_summary.py $O/pmc --by-grid > $O/pmc_summary.md 2>&1; cat $O/pmc_summary.md
echo done
