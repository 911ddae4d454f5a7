# which earlier tests make test_hipgraph_pull_ahead_trains[w2v] segfault
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s26; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_models.py -m gpu > $O/models.log 2>&1; rc=$?
echo "models only rc=$rc"; grep -E "PASSED|FAILED|ERROR" $O/models.log | tail -2
