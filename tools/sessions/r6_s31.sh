# end-of-session check: smoke, full GPU suite, bench (fast path x2, N>1 auto one rank), word2vec / FM quick numbers
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s31; mkdir -p $O
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rfs --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -8 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d.get('config',{}); print(sys.argv[2], d['ms_per_step'], round(d.get('value',0)/1e6,1), c.get('exchange'), c.get('loss_last'))" "$@"; }
for r in 1 2; do
  timeout -k 10 200 python bench.py > $O/fast_$r.json 2>$O/fast_$r.err || { tail -20 $O/fast_$r.err; exit 1; }
  j $O/fast_$r.json "fast_$r (bench.py defaults)"
  SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py > $O/xauto_$r.json 2>$O/xauto_$r.err || { tail -20 $O/xauto_$r.err; exit 1; }
  j $O/xauto_$r.json "xauto_$r"
done
echo done
