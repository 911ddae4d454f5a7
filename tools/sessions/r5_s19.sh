# scatter write amplification vs the open-line frontier: chunks per launch
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s19; mkdir -p $O
cd /tmp
for nch in 128 64 32; do
  SS_BD_NCH=$nch HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ser_$nch -o run -- python3 $R/bench.py --steps 25 --warmup 2 > $O/ser_$nch.log 2>&1 || exit $?
  SS_BD_NCH=$nch timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc WRITE_SIZE TCC_EA0_WRREQ_sum --output-format csv -d $O/pmc_$nch -o run -- python3 $R/bench.py --steps 4 --warmup 2 > $O/pmc_$nch.log 2>&1 || exit $?
done
