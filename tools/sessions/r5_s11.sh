set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s11; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/bench_$r.json 2> $O/bench_$r.err || exit $?
  python -c "import json; d=json.loads(open('$O/bench_$r.json').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], round(d['value']/1e6,1), d['config']['init'], d['config']['loss_last'])"
done
timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/w2v.json 2>$O/w2v.err || exit $?
tail -c 400 $O/w2v.json; echo
timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/fm_10b.conf --steps 30 --warmup 8 --set table_capacity=2000000000 > $O/fm.json 2>$O/fm.err || exit $?
tail -c 300 $O/fm.json; echo
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -8 $O/pytest_gpu.log; exit $rc
