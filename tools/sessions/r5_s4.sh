set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s4; mkdir -p $O
for r in 1 2; do
  for v in "t256:X=1" "t128:SS_CLAIM_T=128" "t64:SS_CLAIM_T=64" "t256ct256:SS_BD_CT=256,SS_BD_CNT=256" "t256ct512:SS_BD_CT=512,SS_BD_CNT=512" "cas:SS_CLAIM=0" "x1:SS_ENGINE_GENERAL=xgmi" "x0:SS_ENGINE_GENERAL=xgmi,SS_CLAIM=0"; do
    IFS=: read name env <<< "$v"
    env ${env//,/ } timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/${name}_$r.json 2> $O/${name}_$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/${name}_$r.json').read().strip().splitlines()[-1]); print('$name', d['ms_per_step'], round(d['value']/1e6,1), d['config']['loss_last'])"
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -15 $O/pytest_gpu.log; exit $rc
