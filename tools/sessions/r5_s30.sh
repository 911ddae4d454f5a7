# with the 16K-tile sorted scatter: chunk count sweep (SS_BD_NCH) and route-record width
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s30; mkdir -p $O
for r in 1 2; do
  for x in 128 64 96 192 256; do
    SS_BD_NCH=$x timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b_${x}_$r.json 2>$O/b_${x}_$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${x}_$r.json').read().splitlines()[-1]); print('nch=$x', d['ms_per_step'])"
  done
done
