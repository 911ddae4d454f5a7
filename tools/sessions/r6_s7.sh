# pipelined (not serialised) kernel traces of the fast path and the N>1 1-rank path: which kernels the route stream overlaps
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s7; mkdir -p $O
cd /tmp; export PYTHONPATH=$R
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/fast_pipe -o run -- python3 $R/bench.py --steps 24 --warmup 8 > $O/fast_pipe.log 2>&1 || exit $?
SS_ENGINE_GENERAL=xgmi timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/x_pipe -o run -- python3 $R/bench.py --steps 24 --warmup 8 > $O/x_pipe.log 2>&1 || exit $?
cd $R
python tools/timeline.py $O/fast_pipe/run_kernel_trace.csv 60 > $O/fast_timeline.txt
python tools/timeline.py $O/x_pipe/run_kernel_trace.csv 90 > $O/x_timeline.txt
echo done
