# word2vec: planted-cluster quality on fp32 and bf16 rows; per-pair and window throughput on bf16 rows
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s43; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gpu_models.py -k "planted_clusters" -m gpu > $O/pytest.log 2>&1 || { grep -E "Error|error|FAILED|^E " $O/pytest.log | head -40; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for rows in bf16 fp32; do
    timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set neg_mode=per_pair --set row_dtype=$rows > $O/pp_${rows}_$r.json 2>$O/pp_${rows}_$r.err || { tail -20 $O/pp_${rows}_$r.err; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/pp_${rows}_$r.json') if l.startswith('{')][-1]); print('per-pair rows=$rows', d['ms_per_step'], d['samples_per_s']/1e6, d['loss'])"
    timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set row_dtype=$rows > $O/w_${rows}_$r.json 2>$O/w_${rows}_$r.err || { tail -20 $O/w_${rows}_$r.err; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/w_${rows}_$r.json') if l.startswith('{')][-1]); print('window rows=$rows', d['ms_per_step'], d['samples_per_s']/1e6, d['loss'])"
  done
done
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pp16_ser -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 --set neg_mode=per_pair --set graph=0 --set row_dtype=bf16 > $O/pp16_ser.log 2>&1 || exit $?
