# the s23 test set again, verbose (which test segfaults), 16K-key scatter tiles
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s25; mkdir -p $O
SS_BD_SKT=${SKT:-16} timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_claim.py tests/test_gpu_models.py -m gpu > $O/pytest.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -3; tail -2 $O/pytest.log
