# word2vec occurrence reduce: the fused update's slot index loaded beside the first gathers (SS_W2V_EARLY_SLOT 1 vs 0, one box)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s45; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gpu_models.py -k "fused_update or per_pair or planted" -m gpu > $O/pytest.log 2>&1 || { grep -E "Error|error|FAILED|^E " $O/pytest.log | head -40; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
 for x in 1 0; do
  SS_W2V_EARLY_SLOT=$x timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set neg_mode=per_pair > $O/pp_${x}_$r.json 2>$O/pp_${x}_$r.err || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/pp_${x}_$r.json') if l.startswith('{')][-1]); print('per-pair early=$x', d['ms_per_step'], d['samples_per_s']/1e6)"
  SS_W2V_EARLY_SLOT=$x timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/w_${x}_$r.json 2>$O/w_${x}_$r.err || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/w_${x}_$r.json') if l.startswith('{')][-1]); print('window early=$x', d['ms_per_step'], d['samples_per_s']/1e6)"
 done
done
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pp_ser -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 --set neg_mode=per_pair --set graph=0 > $O/pp_ser.log 2>&1 || exit $?
