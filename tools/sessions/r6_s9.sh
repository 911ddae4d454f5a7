# claimed pull: first-probe loads of KR keys per thread in flight (SS_CLAIM_KR 4 / 8 vs 1): tests, A/B, serial stats
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s9; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_oracle.py tests/test_gpu_claim.py tests/test_gpu_eval_sharded.py -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log
[ $rc -gt 1 ] && exit $rc
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1))" "$@"; }
for r in 1 2 3; do
  for v in 4 8 1; do
    SS_CLAIM_KR=$v timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/fast_${v}_$r.json 2>$O/fast_${v}_$r.err || { tail -20 $O/fast_${v}_$r.err; exit 1; }
    j $O/fast_${v}_$r.json "fast kr=$v"
  done
done
for r in 1 2; do
  for v in 4 1; do
    SS_CLAIM_KR=$v SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/x_${v}_$r.json 2>$O/x_${v}_$r.err || { tail -20 $O/x_${v}_$r.err; exit 1; }
    j $O/x_${v}_$r.json "xgmi1 kr=$v"
  done
done
cd /tmp; export PYTHONPATH=$R
for v in 4 8; do
  SS_CLAIM_KR=$v HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/fast_ser_$v -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/fast_ser_$v.log 2>&1 || exit $?
done
echo done
