# N>1 unique-key layout: occurrences per source bucket (SS_BD_TARGET_DIST 1024 / 2048 / 3072) with 4 and 8 bench ranks on one GPU
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s49; mkdir -p $O
for w in 8 4; do
 for r in 1 2; do
  for t in 2048 1024 3072; do
    SS_BD_TARGET_DIST=$t timeout -k 10 400 python tools/prof_world.py --world $w --no-prof --out $O/w${w}_${t}_$r --timeout 300 -- --transport xgmi --cal-steps 0 > $O/w${w}_${t}_$r.log 2>&1 || { tail -20 $O/w${w}_${t}_$r.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/w${w}_${t}_$r/rank0.log') if l.startswith('{')][-1]); print('world$w target=$t', d['ms_per_step'], d['config']['loss_last'], d['config']['server_unique_keys_per_step'])"
  done
 done
done
