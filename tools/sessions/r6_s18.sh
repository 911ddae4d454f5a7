# record exchange at one rank: serial and pipelined kernel traces (what bounds it against the fast path)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s18; mkdir -p $O
cd /tmp; export PYTHONPATH=$R
export SS_ENGINE_GENERAL=xgmi SS_XCHG=records
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/ser_rec -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/ser_rec.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/pipe_rec -o run -- python3 $R/bench.py --steps 24 --warmup 8 > $O/pipe_rec.log 2>&1 || exit $?
cd $R
python tools/kstats.py --range timed $O/ser_rec > $O/ser_rec_stats.txt 2>&1
python tools/kstats.py --range timed $O/pipe_rec > $O/pipe_rec_stats.txt 2>&1
head -24 $O/ser_rec_stats.txt; head -24 $O/pipe_rec_stats.txt
echo done
