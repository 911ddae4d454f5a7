# grouped records (SS_REC_GROUP=1: unique-layout source buckets, records grouped by server sub-bucket after the scatter) vs round 5's small record buckets (0) vs unique: tests, then N = 2 / 4 / 8 ranks on one GPU
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s43; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_eval_sharded.py tests/test_gpu_xgmi_tiers.py tests/test_gpu_oracle.py -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['config']; print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), c.get('exchange'), c['layout'].get('srv_sub_buckets'), c['layout'].get('record_group'), c['loss_last'])" "$@"; }
for w in 4 8 2; do
  for v in g1 g0 u; do
    case $v in g1) E="SS_XCHG=records SS_REC_GROUP=1";; g0) E="SS_XCHG=records SS_REC_GROUP=0";; u) E="SS_XCHG=unique";; esac
    env $E timeout -k 10 400 python tools/prof_world.py --world $w --no-prof --out $O/w${w}_$v --timeout 300 -- --transport xgmi --steps 30 --warmup 10 > $O/w${w}_$v.log 2>&1 || { tail -30 $O/w${w}_$v.log; exit 1; }
    j $O/w${w}_$v/rank0.log "world$w $v"
  done
done
echo done
