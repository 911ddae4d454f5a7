set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s10; mkdir -p $O
for r in 1 2 3; do
  for v in "d4:SS_ENGINE_DEPTH=4" "t3072d8:SS_BD_TARGET=3072,SS_ENGINE_DEPTH=8" "t3584d8:SS_BD_TARGET=3584,SS_ENGINE_DEPTH=8" "t3584:SS_BD_TARGET=3584" "t2560d8:SS_BD_TARGET=2560,SS_ENGINE_DEPTH=8"; do
    IFS=: read name env <<< "$v"
    env ${env//,/ } timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/${name}_$r.json 2> $O/${name}_$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/${name}_$r.json').read().strip().splitlines()[-1]); print('$name', d['ms_per_step'], round(d['value']/1e6,1))"
  done
done
