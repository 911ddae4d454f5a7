set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s5; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread "tests/test_gpu_eval_sharded.py::test_sharded_eval_matches_world1[2-staleness1-env1-0.01]" tests/test_gpu_models.py::test_graph_capture_after_mode_switch_xgmi > $O/pytest_a.log 2>&1
rc=$?; grep -E "Error|assert|PASS|FAIL" $O/pytest_a.log | head -30; [ $rc -le 1 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -25 $O/pytest_gpu.log; exit $rc
