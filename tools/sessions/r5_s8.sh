set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s8; mkdir -p $O
timeout -k 10 700 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_claim.py tests/test_gpu_eval_sharded.py tests/test_gpu_multiproc.py tests/test_gpu_xgmi_tiers.py > $O/pytest_x.log 2>&1
rc=$?; tail -4 $O/pytest_x.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for st in 1 0; do
    for w in 4 8; do
      SS_SRV_STAGE=$st timeout -k 10 400 python tools/prof_world.py --world $w --no-prof --out $O/w${w}_st${st}_$r --timeout 300 -- --transport xgmi --steps 30 --warmup 6 --cal-steps 0 > /dev/null 2>&1 || exit $?
      grep -h '"metric"' $O/w${w}_st${st}_$r/rank0.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('world$w stage$st', d['ms_per_step'], round(d['value']/1e6,1))"
    done
  done
done
