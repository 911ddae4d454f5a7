# grouped records after the run-bound fix: the sharded-eval oracle with 3 forced sub-buckets first (stop on any failure), then the 2 / 4 / 8-rank A/B
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s46; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest "tests/test_gpu_eval_sharded.py" -k "env5" -x -q -rf --timeout 200 --timeout-method thread > $O/pytest1.log 2>&1; rc=$?
tail -3 $O/pytest1.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_eval_sharded.py tests/test_gpu_xgmi_tiers.py -x -q -rf --timeout 300 --timeout-method thread > $O/pytest2.log 2>&1; rc=$?
tail -3 $O/pytest2.log
[ $rc -ne 0 ] && exit $rc
bash tools/sessions/r6_s43.sh
