# A/B: XCD-aware scatter chunk order (SS_BD_XCD 1 vs 0): bench pairs, serial
# kernel stats and a WRITE_SIZE pass each
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s18; mkdir -p $O
for r in 1 2 3; do
  for x in 1 0; do
    SS_BD_XCD=$x timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b_${x}_$r.json 2>$O/b_${x}_$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${x}_$r.json').read().splitlines()[-1]); print('xcd=$x', d['ms_per_step'])"
  done
done
cd /tmp
for x in 1 0; do
  SS_BD_XCD=$x HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ser_$x -o run -- python3 $R/bench.py --steps 25 --warmup 2 > $O/ser_$x.log 2>&1 || exit $?
  SS_BD_XCD=$x timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc WRITE_SIZE TCC_EA0_WRREQ_sum --output-format csv -d $O/pmc_$x/p1 -o run -- python3 $R/bench.py --steps 4 --warmup 2 > $O/pmc_$x.log 2>&1 || exit $?
  SS_BD_XCD=$x timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc FETCH_SIZE --output-format csv -d $O/pmc_$x/p2 -o run -- python3 $R/bench.py --steps 4 --warmup 2 > $O/pmc2_$x.log 2>&1 || exit $?
done
