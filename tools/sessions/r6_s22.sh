# where k_bd_reduce's time goes (fast path, serialised): SS_BD_DBG measurement bits (wrong results; timing only)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s22; mkdir -p $O
cd /tmp; export PYTHONPATH=$R
for v in 0 1 2 4 8 3 7; do
  SS_BD_DBG=$v HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/d$v -o run -- python3 $R/bench.py --steps 20 --warmup 5 --init zero > $O/d$v.log 2>&1 || { tail $O/d$v.log; exit 1; }
  python3 $R/tools/kstats.py --range timed $O/d$v > $O/d$v.txt 2>&1
  echo "dbg=$v $(grep k_bd_reduce $O/d$v.txt | head -1)"
done
echo done
