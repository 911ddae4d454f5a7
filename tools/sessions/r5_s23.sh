# sorted scatter: 16K-key narrow tiles vs 8K; GPU suite (models + kernels + claim)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s23; mkdir -p $O
for r in 1 2 3; do
  for x in 16 8; do
    SS_BD_SKT=$x timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b_${x}_$r.json 2>$O/b_${x}_$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${x}_$r.json').read().splitlines()[-1]); print('skt=$x', d['ms_per_step'], d['config']['loss_last'])"
  done
done
cd /tmp
for x in 16 8; do
  SS_BD_SKT=$x HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ser_$x -o run -- python3 $R/bench.py --steps 25 --warmup 2 > $O/ser_$x.log 2>&1 || exit $?
  SS_BD_SKT=$x timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc WRITE_SIZE TCC_EA0_WRREQ_sum --output-format csv -d $O/pmc_$x -o run -- python3 $R/bench.py --steps 4 --warmup 2 > $O/pmc_$x.log 2>&1 || exit $?
done
