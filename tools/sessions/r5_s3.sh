set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s3; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_claim.py > $O/pytest_claim.log 2>&1
rc=$?; tail -3 $O/pytest_claim.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for v in "base:X=1" "prio:SS_MAIN_PRIO=1" "cu64:SS_ROUTE_CUS=64" "cu128:SS_ROUTE_CUS=128" "cu192:SS_ROUTE_CUS=192" "nch64:SS_BD_NCH=64" "x1:SS_ENGINE_GENERAL=xgmi" "x1noss:SS_ENGINE_GENERAL=xgmi,SS_SERVER_STREAM=0" "x0noss:SS_ENGINE_GENERAL=xgmi,SS_SERVER_STREAM=0,SS_CLAIM=0"; do
    IFS=: read name env <<< "$v"
    env ${env//,/ } timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/${name}_$r.json 2> $O/${name}_$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/${name}_$r.json').read().strip().splitlines()[-1]); print('$name', d['ms_per_step'], round(d['value']/1e6,1), d['config']['loss_last'])"
  done
done
cd /tmp && env SS_ENGINE_GENERAL=xgmi HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_x1_serial -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --cal-steps 0 > $O/prof_x1.log 2>&1 || exit $?
env SS_ENGINE_GENERAL=xgmi SS_CLAIM=0 HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_x0_serial -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --cal-steps 0 > $O/prof_x0.log 2>&1
