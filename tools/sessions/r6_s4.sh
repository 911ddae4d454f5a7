# changed GPU tests; FM fused (prefetched rows) A/B; marker-attributed serial stats; long run
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s4; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_oracle.py tests/test_gpu_claim.py "tests/test_gpu_models.py" -k "oracle or claim or region or fm or w2v or word2vec or teardown" -q -rf --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -8 $O/pytest.log
[ $rc -gt 1 ] && exit $rc
for r in 1 2; do
  for f in 1 0; do
    SS_FM_FUSE=$f timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/fm_10b.conf --steps 40 --warmup 10 --set num_features=1000000000 > $O/fm_${f}_$r.json 2>$O/fm_${f}_$r.err || { tail -20 $O/fm_${f}_$r.err; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/fm_${f}_$r.json') if l.startswith('{')][-1]); print('fm fuse=$f', round(d['ms_per_step'],4), round(d['samples_per_s']/1e6,1), d['loss'])"
  done
done
timeout -k 10 300 python tools/long_run.py --steps 2000 --window 100 > $O/long.json 2> $O/long.err || { tail -20 $O/long.err; exit 1; }
python -c "import json; d=json.loads(open('$O/long.json').read().splitlines()[-1]); print('long', d['ms_min'], d['ms_max'], d['drift_last_vs_first'], d['regions'])"
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/fast_ser -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/fast_ser.log 2>&1 || exit $?
echo done
