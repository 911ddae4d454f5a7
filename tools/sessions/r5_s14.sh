set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s14; mkdir -p $O
p() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['ms_per_step'],4), round(d.get('samples_per_s', d.get('value', 0))/1e6,1))"; }
for r in 1 2; do
  SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/w2vx_$r.json 2>$O/w2vx.err || exit $?
  p $O/w2vx_$r.json w2v_xgmi_world1
  timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/w2v_$r.json 2>$O/w2v.err || exit $?
  p $O/w2v_$r.json w2v_1gpu
  SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/lrx_$r.json 2>$O/lrx.err || exit $?
  p $O/lrx_$r.json lr_xgmi_world1
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/lr_$r.json 2>$O/lr.err || exit $?
  p $O/lr_$r.json lr_1gpu
  timeout -k 10 200 python bench.py --batch 65536 --steps 50 --warmup 10 > $O/lr64k_$r.json 2>$O/lr64k.err || exit $?
  p $O/lr64k_$r.json lr_1gpu_b65536
  timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/sparse_lr_10m.conf --steps 50 --warmup 10 > $O/lr10m_$r.json 2>$O/lr10m.err || exit $?
  p $O/lr10m_$r.json lr_10m
done
timeout -k 10 400 python tools/prof_world.py --world 4 --no-prof --launch --out $O/w2v4 --timeout 300 -- --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > /dev/null 2>&1 || exit $?
grep -h '^{' $O/w2v4/rank0.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('w2v world4 one GPU', round(d['ms_per_step'],4), round(d['samples_per_s']/1e6,1))"
