# count over two sub-chunks per scatter chunk (SS_BD_CSUB=2): dedup tests, A/B; then SS_XCHG=auto at 8 ranks on one GPU
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s25; mkdir -p $O
cd $R
SS_BD_CSUB=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_dedup_variants.py tests/test_gpu_oracle.py -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['config']; print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), c['loss_last'], c.get('exchange'))" "$@"; }
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/$n.json 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  j $O/$n.json "$n"
}
for r in 1 2 3; do
  run c1_$r SS_BD_CSUB=1
  run c2_$r SS_BD_CSUB=2
done
for r in 1 2; do
  run xc1_$r SS_BD_CSUB=1 SS_ENGINE_GENERAL=xgmi
  run xc2_$r SS_BD_CSUB=2 SS_ENGINE_GENERAL=xgmi
done
timeout -k 10 600 python tools/prof_world.py --world 8 --no-prof --out $O/w8_auto --timeout 500 -- --transport xgmi --steps 30 --warmup 10 > $O/w8_auto.log 2>&1 || { tail -30 $O/w8_auto.log; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['config']; print('world8 auto', d['ms_per_step'], round(d['value']/1e6,1), c.get('exchange'), c.get('calibration',{}).get('exchange'))" $O/w8_auto/rank0.log
echo done
