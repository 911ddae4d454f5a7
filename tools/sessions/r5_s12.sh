set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s12; mkdir -p $O
p() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['ms_per_step'],4), round(d['samples_per_s']/1e6,1))"; }
for r in 1 2; do
  for d in 4 8; do
    SS_ENGINE_DEPTH=$d timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/w2v_d${d}_$r.json 2>$O/w2v.err || exit $?
    p $O/w2v_d${d}_$r.json w2v_d$d
    SS_ENGINE_DEPTH=$d timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/fm_10b.conf --steps 30 --warmup 8 --set table_capacity=2000000000 > $O/fm_d${d}_$r.json 2>$O/fm.err || exit $?
    p $O/fm_d${d}_$r.json fm_d$d
  done
done
timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set neg_mode=per_pair > $O/w2v_pp.json 2>$O/w2v_pp.err || exit $?
p $O/w2v_pp.json w2v_pp
