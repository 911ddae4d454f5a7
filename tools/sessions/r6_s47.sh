# after grouped records went default-off: the whole GPU suite, smoke(), the 1-GPU bench twice and the one-rank N>1 path (auto exchange)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s47; mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/suite.log 2>&1; rc=$?
tail -4 $O/suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 200 python bench.py > $O/bench_$r.json 2>$O/bench_$r.err || { tail -20 $O/bench_$r.err; exit 1; }
  tail -1 $O/bench_$r.json
done
SS_ENGINE_GENERAL=xgmi timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/x1.json 2>$O/x1.err || { tail -20 $O/x1.err; exit 1; }
tail -1 $O/x1.json
echo done
