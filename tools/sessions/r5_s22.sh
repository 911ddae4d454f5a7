# round-5 check: full GPU suite, bench x3, N>1 path at 1 rank x3 (calibration),
# 4 and 8 ranks on one GPU, word2vec one GPU / N>1 / per-pair
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s22; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/bench_$r.json 2>$O/bench_$r.err || exit $?
  SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/x1_$r.json 2>$O/x1_$r.err || exit $?
done
for w in 4 8; do
  timeout -k 10 400 python tools/prof_world.py --world $w --no-prof --out $O/w$w --timeout 300 -- --transport xgmi > $O/w$w.log 2>&1 || exit $?
done
for r in 1 2; do
  timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/w2v_$r.json 2>$O/w2v.err || exit $?
  SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/w2vx_$r.json 2>$O/w2vx.err || exit $?
done
timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set neg_mode=per_pair > $O/w2v_pp.json 2>$O/w2v_pp.err || exit $?
