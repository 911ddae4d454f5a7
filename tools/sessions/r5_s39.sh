# word2vec: 3-stage pair kernel vs the reference (tests with SS_W2V_PP_STAGES=3 and 4); oreduce update prefetch A/B (per-pair and window)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s39; mkdir -p $O
for x in 3 4; do
SS_W2V_PP_STAGES=$x timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_models.py -k "per_pair or word2vec or w2v" -m gpu > $O/pytest_$x.log 2>&1 || { grep -E "Error|error|FAILED|^E " $O/pytest_$x.log | head -30; exit 1; }
tail -1 $O/pytest_$x.log
done
for r in 1 2; do
  for x in 1 0; do
    SS_W2V_PREFETCH=$x timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set neg_mode=per_pair > $O/pp_${x}_$r.json 2>$O/pp_${x}_$r.err || exit $?
    python -c "import json; d=json.loads([l for l in open('$O/pp_${x}_$r.json') if l.startswith('{')][-1]); print('per-pair prefetch=$x', d['ms_per_step'], d['samples_per_s']/1e6, d['loss'])"
    SS_W2V_PREFETCH=$x timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/w_${x}_$r.json 2>$O/w_${x}_$r.err || exit $?
    python -c "import json; d=json.loads([l for l in open('$O/w_${x}_$r.json') if l.startswith('{')][-1]); print('window prefetch=$x', d['ms_per_step'], d['samples_per_s']/1e6, d['loss'])"
  done
done
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pp_ser -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 --set neg_mode=per_pair --set graph=0 > $O/pp_ser.log 2>&1 || exit $?
