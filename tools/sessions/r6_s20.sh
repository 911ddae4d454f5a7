# record exchange with own records off the mailbox: sharded-eval tests (world 2 / 4), 2 / 4 / 8 ranks on one GPU vs unique
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s20; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_eval_sharded.py -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), d['config']['loss_last'], d['config'].get('exchange'))" "$@"; }
for w in 2 4 8; do
  for x in records unique; do
    SS_XCHG=$x timeout -k 10 500 python tools/prof_world.py --world $w --no-prof --out $O/w${w}_$x --timeout 400 -- --transport xgmi --steps 30 --warmup 10 > $O/w${w}_$x.log 2>&1 || { tail -20 $O/w${w}_$x.log; exit 1; }
    j $O/w${w}_$x/rank0.log "world$w $x"
  done
done
echo done
