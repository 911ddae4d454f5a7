# full GPU suite; fast bench x3; N>1 1-rank serial profile by roctx phase; 4 / 8 ranks on one GPU
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s5; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -8 $O/pytest.log
[ $rc -gt 1 ] && exit $rc
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/fast_$r.json 2>$O/fast_$r.err || { tail -20 $O/fast_$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/fast_$r.json').read().splitlines()[-1]); print('fast', d['ms_per_step'], round(d['value']/1e6,1))"
done
for w in 4 8; do
  timeout -k 10 500 python tools/prof_world.py --world $w --no-prof --out $O/w$w --timeout 400 -- --transport xgmi --steps 30 --warmup 10 > $O/w$w.log 2>&1 || { tail -20 $O/w$w.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/w$w/rank0.log') if l.startswith('{')][-1]); print('world$w', d['ms_per_step'], round(d['value']/1e6,1), d['config']['layout'], d['config'].get('calibration',{}).get('pull_ahead'))"
done
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 SS_ENGINE_GENERAL=xgmi timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/x_ser -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/x_ser.log 2>&1 || exit $?
echo done
