# exchange calibration (SS_XCHG=auto): bench tests, one-rank / 2 / 4 ranks on one GPU with auto, fast path check
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s21; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_xgmi_tiers.py tests/test_gpu_models.py -k "bench or record_exchange" -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['config']; print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), c['loss_last'], c.get('exchange'), c.get('calibration',{}).get('exchange'))" "$@"; }
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/$n.json 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  j $O/$n.json "$n"
}
for r in 1 2; do
  run fast_$r SS_X=0
  run xauto_$r SS_ENGINE_GENERAL=xgmi
done
for w in 2 4; do
  timeout -k 10 500 python tools/prof_world.py --world $w --no-prof --out $O/w${w}_auto --timeout 400 -- --transport xgmi --steps 30 --warmup 10 > $O/w${w}_auto.log 2>&1 || { tail -20 $O/w${w}_auto.log; exit 1; }
  j $O/w${w}_auto/rank0.log "world$w auto"
done
echo done
