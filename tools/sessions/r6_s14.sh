# r6_s12.sh (generator groups, claim-set size) then r6_s13.sh (word2vec count / column-scan workgroup sizes) in one call
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s12; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_oracle.py tests/test_gpu_claim.py tests/test_convergence.py -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log
[ $rc -gt 1 ] && exit $rc
SS_CLAIM_TS=4096 timeout -k 10 600 python -u -m pytest tests/test_gpu_claim.py tests/test_gpu_oracle.py -q -rf --timeout 300 --timeout-method thread > $O/pytest_ts.log 2>&1; rc=$?
tail -3 $O/pytest_ts.log
[ $rc -gt 1 ] && exit $rc
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1))" "$@"; }
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/$n.json 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  j $O/$n.json "$n"
}
for r in 1 2 3; do
  run def_$r SS_GEN_R=4
  run gen1_$r SS_GEN_R=1
  run ts4k_$r SS_CLAIM_TS=4096
done
for r in 1 2; do
  run xdef_$r SS_ENGINE_GENERAL=xgmi
  run xts4k_$r SS_ENGINE_GENERAL=xgmi SS_CLAIM_TS=4096
done
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/ser_def -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/ser_def.log 2>&1 || exit $?
SS_CLAIM_TS=4096 HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/ser_ts -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/ser_ts.log 2>&1 || exit $?
bash $R/tools/sessions/r6_s13.sh
