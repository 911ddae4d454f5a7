# word2vec per-pair: staged pair kernel (SS_W2V_PP_STAGES 4 / 3 / 2 = previous kernel); tests first
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s38; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_models.py -k "per_pair or word2vec_modes" -m gpu > $O/pytest.log 2>&1 || { grep -E "Error|error|FAILED|^E " $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for x in 4 3 2; do
    SS_W2V_PP_STAGES=$x timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set neg_mode=per_pair > $O/pp_${x}_$r.json 2>$O/pp_${x}_$r.err || exit $?
    python -c "import json; d=json.loads([l for l in open('$O/pp_${x}_$r.json') if l.startswith('{')][-1]); print('stages=$x', d['ms_per_step'], d['samples_per_s']/1e6, d['loss'])"
  done
done
cd /tmp; export PYTHONPATH=$R
SS_W2V_PP_STAGES=4 HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pp4_ser -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 --set neg_mode=per_pair --set graph=0 > $O/pp4_ser.log 2>&1 || exit $?
SS_W2V_PP_STAGES=3 HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pp3_ser -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 --set neg_mode=per_pair --set graph=0 > $O/pp3_ser.log 2>&1 || exit $?
