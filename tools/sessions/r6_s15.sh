# occurrence parameters in sample order (SS_OCC_ORDER=sample: the claimed pull stores occ[pj[p]], the forward streams occ[j], no pos_of) vs bucket order: oracle under both, A/B
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s15; mkdir -p $O
cd $R
SS_OCC_ORDER=sample timeout -k 10 600 python -u -m pytest tests/test_gpu_oracle.py tests/test_gpu_claim.py -q -rf --timeout 300 --timeout-method thread -k "oracle or claimed" > $O/pytest_sample.log 2>&1; rc=$?
tail -3 $O/pytest_sample.log
[ $rc -gt 1 ] && exit $rc
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), d['config']['loss_last'])" "$@"; }
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/$n.json 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  j $O/$n.json "$n"
}
for r in 1 2 3; do
  run bucket_$r SS_OCC_ORDER=bucket
  run sample_$r SS_OCC_ORDER=sample
done
for r in 1 2; do
  run xbucket_$r SS_ENGINE_GENERAL=xgmi SS_OCC_ORDER=bucket
  run xsample_$r SS_ENGINE_GENERAL=xgmi SS_OCC_ORDER=sample
done
cd /tmp; export PYTHONPATH=$R
SS_OCC_ORDER=sample HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/ser_sample -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/ser_sample.log 2>&1 || exit $?
echo done
