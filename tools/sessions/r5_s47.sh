# word2vec per-pair reduce: two items per half-wave (SS_W2V_PP_ITEMS 2, QF 2 / 4) vs one (1); tests first
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s47; mkdir -p $O
for it in 2 1; do
SS_W2V_PP_ITEMS=$it timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gpu_models.py -k "fused_update or per_pair or planted" -m gpu > $O/pytest_$it.log 2>&1 || { grep -E "Error|error|FAILED|^E " $O/pytest_$it.log | head -40; tail -5 $O/pytest_$it.log; exit 1; }
tail -1 $O/pytest_$it.log
done
for r in 1 2; do
 for v in "2 2" "2 4" "1 2"; do
  set -- $v
  SS_W2V_PP_ITEMS=$1 SS_W2V_PP_QF=$2 timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set neg_mode=per_pair > $O/pp_$1_$2_$r.json 2>$O/pp_$1_$2_$r.err || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/pp_$1_$2_$r.json') if l.startswith('{')][-1]); print('per-pair items=$1 qf=$2', d['ms_per_step'], d['samples_per_s']/1e6, d['loss'])"
 done
done
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pp_ser -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 --set neg_mode=per_pair --set graph=0 > $O/pp_ser.log 2>&1 || exit $?
