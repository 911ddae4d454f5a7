# Round-6 entry: smoke, GPU tests, bench (fast path and N>1 path, two reps each)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s1; mkdir -p $O
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/fast_$r.json 2>$O/fast_$r.err || { tail -20 $O/fast_$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/fast_$r.json').read().splitlines()[-1]); print('fast', d['ms_per_step'], d['value']/1e6)"
  SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/x_$r.json 2>$O/x_$r.err || { tail -20 $O/x_$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/x_$r.json').read().splitlines()[-1]); print('xgmi1', d['ms_per_step'], d['value']/1e6)"
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log; exit $rc
