# record exchange, own records off the mailbox (cached rows, gradients read through spj): tests + one-rank A/B
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s19; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py -k "record_exchange" tests/test_gpu_eval_sharded.py -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), d['config']['loss_last'])" "$@"; }
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/$n.json 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  j $O/$n.json "$n"
}
for r in 1 2 3; do
  run own_$r SS_ENGINE_GENERAL=xgmi SS_XCHG=records
  run arena_$r SS_ENGINE_GENERAL=xgmi SS_XCHG=records SS_REC_OCC=arena
  run uniq_$r SS_ENGINE_GENERAL=xgmi
done
echo done
