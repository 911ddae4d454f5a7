# bisect the graph-replay segfault: which earlier file's tests trigger it
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s27; mkdir -p $O
run() {
  name=$1; shift
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider "$@" -m gpu > $O/$name.log 2>&1; rc=$?
  echo "$name rc=$rc $(grep -cE 'PASSED' $O/$name.log) passed; last: $(grep -E 'PASSED|FAILED' $O/$name.log | tail -1)"
  [ $rc -eq 139 ] || [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
run claim tests/test_gpu_claim.py "tests/test_gpu_models.py::test_hipgraph_pull_ahead_trains"
run kernels tests/test_gpu_kernels.py "tests/test_gpu_models.py::test_hipgraph_pull_ahead_trains"
