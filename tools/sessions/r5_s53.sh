# N>1 server sub-bucket count from the sources' actual bucket size: word2vec config 3 at 4 ranks (auto = 1 vs the old 2 vs 6), FM 4 ranks, tests
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s53; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gpu_eval_sharded.py tests/test_gpu_multiproc.py tests/test_gpu_xgmi_tiers.py -m gpu > $O/pytest.log 2>&1 || { grep -E "Error|error|FAILED|^E " $O/pytest.log | head -40; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for m in auto 2 6; do
    if [ $m = auto ]; then unset SS_SRV_SUB; else export SS_SRV_SUB=$m; fi
    timeout -k 10 400 python tools/prof_world.py --world 4 --no-prof --launch --out $O/w2v4_${m}_$r --timeout 300 -- --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/w2v4_${m}_$r.log 2>&1 || { tail -20 $O/w2v4_${m}_$r.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/w2v4_${m}_$r/rank0.log') if l.startswith('{')][-1]); print('w2v world4 sub=$m', d['ms_per_step'], d.get('loss'))"
  done
  unset SS_SRV_SUB
done
