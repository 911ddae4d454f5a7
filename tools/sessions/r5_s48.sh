# one-GPU bench: the next route gated on this round's pull (SS_ROUTE_GATE 1 vs 0), interleaved
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s48; mkdir -p $O
for r in 1 2 3; do
  for x in 1 0; do
    SS_ROUTE_GATE=$x timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b_${x}_$r.json 2>$O/b_${x}_$r.err || { tail -20 $O/b_${x}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${x}_$r.json').read().splitlines()[-1]); print('gate=$x', d['ms_per_step'], d['value']/1e6, d['config']['loss_last'])"
  done
done
