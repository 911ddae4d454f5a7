# 8 bench ranks on one GPU (unique exchange), every rank under rocprofv3 --kernel-trace --stats: where the 8-rank step's kernel time goes
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s39; mkdir -p $O
cd $R
SS_XCHG=unique timeout -k 10 500 python tools/prof_world.py --world 8 --out $O/w8 --timeout 400 -- --transport xgmi --steps 30 --warmup 10 --cal-steps 0 > $O/w8.log 2>&1 || { tail -30 $O/w8.log; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('world8', d['ms_per_step'])" $O/w8/rank0.log
ls $O/w8 | head
echo done
