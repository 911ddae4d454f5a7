# graph replay segfault: the graph tests with the 8K-key then the 16K-key scatter tile
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s24; mkdir -p $O
SS_BD_SKT=8 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_models.py -m gpu -k "hipgraph_pull_ahead" > $O/skt8.log 2>&1; echo "skt8 rc=$?"; grep -E "PASSED|FAILED|passed|failed" $O/skt8.log | tail -5
SS_BD_SKT=16 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_models.py -m gpu -k "hipgraph_pull_ahead" > $O/skt16.log 2>&1; echo "skt16 rc=$?"; grep -E "PASSED|FAILED|passed|failed" $O/skt16.log | tail -5
