set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s4; mkdir -p $O
for r in 1 2; do
  for v in "base:X=1" "t512:SS_CLAIM_T=512" "t256:SS_CLAIM_T=256" "ct256:SS_BD_CT=256,SS_BD_CNT=256" "t512ct256:SS_CLAIM_T=512,SS_BD_CT=256,SS_BD_CNT=256"; do
    IFS=: read name env <<< "$v"
    env ${env//,/ } timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/${name}_$r.json 2> $O/${name}_$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/${name}_$r.json').read().strip().splitlines()[-1]); print('$name', d['ms_per_step'], round(d['value']/1e6,1), d['config']['loss_last'])"
  done
done
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -15 $O/pytest_gpu.log; exit $rc
