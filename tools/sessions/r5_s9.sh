set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s9; mkdir -p $O
cd /tmp
for d in 4 8; do
  SS_ENGINE_DEPTH=$d timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_d$d -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $O/prof_d$d.log 2>&1 || exit $?
  grep -h ms_per_step $O/prof_d$d.log | cut -c 150-260
done
