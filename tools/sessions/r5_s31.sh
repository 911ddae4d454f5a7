# N>1 path at one rank: pipelined kernel trace + serial stats (current tree)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s31; mkdir -p $O
cd /tmp; export PYTHONPATH=$R
SS_ENGINE_GENERAL=xgmi timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/pipe -o run -- python3 $R/bench.py --steps 30 --warmup 10 --cal-steps 0 > $O/pipe.log 2>&1 || exit $?
SS_ENGINE_GENERAL=xgmi HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ser -o run -- python3 $R/bench.py --steps 25 --warmup 2 --cal-steps 0 > $O/ser.log 2>&1 || exit $?
