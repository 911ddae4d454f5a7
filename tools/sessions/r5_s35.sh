# sparse LR merge: single-occurrence keys stored, not LDS-added (SS_LR_SINGLE 1 vs 0)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s35; mkdir -p $O
for r in 1 2 3; do
  for x in 1 0; do
    SS_LR_SINGLE=$x timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b_${x}_$r.json 2>$O/b_${x}_$r.err || exit $?
    SS_LR_SINGLE=$x SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cal-steps 0 > $O/x_${x}_$r.json 2>$O/x_${x}_$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${x}_$r.json').read().splitlines()[-1]); x=json.loads(open('$O/x_${x}_$r.json').read().splitlines()[-1]); print('single=$x', d['ms_per_step'], d['config']['loss_last'], 'xgmi', x['ms_per_step'], x['config']['loss_last'])"
  done
done
