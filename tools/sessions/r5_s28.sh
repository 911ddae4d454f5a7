# the crashing sequence with per-test GPU memory logged
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s28; mkdir -p $O
SS_TEST_MEMLOG=$O/mem.txt timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_claim.py tests/test_gpu_models.py -m gpu > $O/pytest.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "PASSED|FAILED" $O/pytest.log | tail -1; tail -4 $O/mem.txt
