set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s13; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -rf --timeout 200 --timeout-method thread tests/test_gpu_models.py -k "w2v or word2vec" > $O/pytest_w2v.log 2>&1
rc=$?; tail -4 $O/pytest_w2v.log; [ $rc -le 1 ] || exit $rc
p() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['ms_per_step'],4), round(d['samples_per_s']/1e6,1))"; }
for r in 1 2; do
  for f in 1 0; do
    SS_W2V_FUSE=$f timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/w2v_f${f}_$r.json 2>$O/w2v.err || exit $?
    p $O/w2v_f${f}_$r.json w2v_fuse$f
    SS_W2V_FUSE=$f timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set neg_mode=per_pair > $O/pp_f${f}_$r.json 2>$O/pp.err || exit $?
    p $O/pp_f${f}_$r.json pp_fuse$f
  done
done
