# full GPU suite after the exchange changes
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s23; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rfs --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
exit $rc
