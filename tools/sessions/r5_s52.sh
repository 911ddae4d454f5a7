# FM (config 5 shape per rank) at 4 ranks on one GPU: N>1 source bucket target 3072 (default) vs 1024; sparse LR 2 ranks
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s52; mkdir -p $O
for r in 1 2; do
  for t in 3072 1024; do
    SS_BD_TARGET_DIST=$t timeout -k 10 400 python tools/prof_world.py --world 4 --no-prof --launch --out $O/fm4_${t}_$r --timeout 300 -- --config configs/fm_10b.conf --steps 30 --warmup 10 --set table_capacity=120000000 > $O/fm4_${t}_$r.log 2>&1 || { tail -20 $O/fm4_${t}_$r.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/fm4_${t}_$r/rank0.log') if l.startswith('{')][-1]); print('fm world4 target=$t', d['ms_per_step'], d.get('loss'))"
    SS_BD_TARGET_DIST=$t timeout -k 10 400 python tools/prof_world.py --world 2 --no-prof --out $O/lr2_${t}_$r --timeout 300 -- --transport xgmi --cal-steps 0 > $O/lr2_${t}_$r.log 2>&1 || { tail -20 $O/lr2_${t}_$r.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/lr2_${t}_$r/rank0.log') if l.startswith('{')][-1]); print('lr world2 target=$t', d['ms_per_step'], d['config']['loss_last'])"
  done
done
