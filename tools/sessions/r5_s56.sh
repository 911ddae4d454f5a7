# N>1 path ring depth 8 vs 4 (SS_ENGINE_DEPTH), 1 rank and 4 ranks on one GPU, sparse LR
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s56; mkdir -p $O
for r in 1 2; do
  for d in 8 4; do
    SS_ENGINE_DEPTH=$d SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cal-steps 0 > $O/x_${d}_$r.json 2>$O/x_${d}_$r.err || { tail -20 $O/x_${d}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/x_${d}_$r.json').read().splitlines()[-1]); print('xgmi1 depth=$d', d['ms_per_step'], d['config']['loss_last'])"
    SS_ENGINE_DEPTH=$d timeout -k 10 400 python tools/prof_world.py --world 4 --no-prof --out $O/w4_${d}_$r --timeout 300 -- --transport xgmi --cal-steps 0 > $O/w4_${d}_$r.log 2>&1 || { tail -20 $O/w4_${d}_$r.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/w4_${d}_$r/rank0.log') if l.startswith('{')][-1]); print('world4 depth=$d', d['ms_per_step'], d['config']['loss_last'])"
  done
done
