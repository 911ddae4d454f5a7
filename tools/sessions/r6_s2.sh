# GPU tests without the new teardown test, then the graph + server-stream capture experiment
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s2; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread --deselect tests/test_gpu_models.py::test_graph_teardown_then_replay_same_process > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
[ $rc -gt 1 ] && exit $rc
for m in none normal prio; do
  timeout -k 10 120 python tools/exp/graph_server_stream.py $m > $O/exp_$m.log 2>&1; r=$?
  echo "exp $m rc=$r"; tail -3 $O/exp_$m.log
  [ $r -ne 0 ] && break
done
exit 0
