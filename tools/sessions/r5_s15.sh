set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s15; mkdir -p $O
p() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['ms_per_step'],4), round(d.get('samples_per_s', d.get('value', 0))/1e6,1), d.get('hipgraph'), d.get('pull_ahead'))"; }
for v in "base:X=1" "noss:SS_SERVER_STREAM=0" "sync:SS_CAL_PICK=sync" "nossync:SS_SERVER_STREAM=0,SS_CAL_PICK=sync" "eager:SS_GRAPH=0" "noss_eager:SS_SERVER_STREAM=0,SS_GRAPH=0"; do
  IFS=: read name env <<< "$v"
  env SS_ENGINE_GENERAL=xgmi ${env//,/ } timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/$name.json 2>$O/$name.err || exit $?
  p $O/$name.json $name
done
