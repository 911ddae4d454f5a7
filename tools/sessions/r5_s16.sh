set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s16; mkdir -p $O
R=$GRAFT_REPO_ROOT
p() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['ms_per_step'],4), d.get('hipgraph'), d.get('pull_ahead'))"; }
for r in 1 2; do
  for c in 12bafed d1ef0ae 5207642 14763ab HEAD; do
    d=$R/_bisect/$c; [ $c = HEAD ] && d=$R
    (cd $d && SS_ENGINE_GENERAL=xgmi SS_SERVER_STREAM=0 SS_NO_AUTOBUILD=1 timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/${c}_$r.json 2>$O/${c}_$r.err) || exit $?
    p $O/${c}_$r.json $c
  done
done
