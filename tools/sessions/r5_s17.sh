set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s17; mkdir -p $O
p() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['ms_per_step'],4), d.get('hipgraph'), d.get('pull_ahead'), d.get('calibration',{}).get('sync_ms'), d.get('calibration',{}).get('ahead_ms'))"; }
for r in 1 2; do
  SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/w2v_x_$r.json 2>$O/w2v_x_$r.err || exit $?
  p $O/w2v_x_$r.json w2v_xgmi
  SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/lr_x_$r.json 2>$O/lr_x_$r.err || exit $?
  tail -1 $O/lr_x_$r.json
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench_$r.json 2>$O/bench_$r.err || exit $?
  tail -1 $O/bench_$r.json
done
