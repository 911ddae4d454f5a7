# the crashing order with the per-test gc teardown (SS_TEST_GC=1, default) and without
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s29; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_claim.py tests/test_gpu_models.py -m gpu > $O/gc1.log 2>&1; rc=$?
echo "gc1 rc=$rc"; grep -E "PASSED|FAILED" $O/gc1.log | tail -1; tail -1 $O/gc1.log
