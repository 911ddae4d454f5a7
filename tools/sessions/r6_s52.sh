# final-tree kernel tables: fast path serialised + pipelined, one-rank N>1 path (auto exchange) serialised, attributed to the timed range
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s52; mkdir -p $O
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/fser -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/fser.log 2>&1 || { tail $O/fser.log; exit 1; }
python3 $R/tools/kstats.py --range timed $O/fser > $O/fser_stats.txt 2>&1; head -14 $O/fser_stats.txt
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/fpipe -o run -- python3 $R/bench.py --steps 24 --warmup 8 > $O/fpipe.log 2>&1 || { tail $O/fpipe.log; exit 1; }
python3 $R/tools/kstats.py --range timed $O/fpipe > $O/fpipe_stats.txt 2>&1; head -14 $O/fpipe_stats.txt
SS_ENGINE_GENERAL=xgmi HIP_LAUNCH_BLOCKING=1 timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/xser -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/xser.log 2>&1 || { tail $O/xser.log; exit 1; }
python3 $R/tools/kstats.py --range timed $O/xser > $O/xser_stats.txt 2>&1; head -20 $O/xser_stats.txt
grep '^{' $O/xser.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('exchange', d['config']['exchange'], d['ms_per_step'])"
echo done
