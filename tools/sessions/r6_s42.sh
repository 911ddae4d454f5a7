# after removing the experiment knobs: dedup / kernel / oracle / bench tests, bench x2
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s42; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dedup_variants.py tests/test_gpu_oracle.py tests/test_gpu_xgmi_tiers.py tests/test_gpu_models.py -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python bench.py > $O/fast_$r.json 2>$O/fast_$r.err || { tail -20 $O/fast_$r.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('fast', d['ms_per_step'], round(d['value']/1e6,1))" $O/fast_$r.json
done
echo done
