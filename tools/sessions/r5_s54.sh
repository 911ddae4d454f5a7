# final end-of-session check: smoke, full GPU suite, bench x3, N>1 path (unique / records), word2vec configs
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s54; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
for r in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/b_$r.json 2>$O/b_$r.err || exit $?
  python -c "import json; d=json.loads(open('$O/b_$r.json').read().splitlines()[-1]); print('bench', d['ms_per_step'], d['value']/1e6, d['config']['init'])"
done
for x in unique records; do
  SS_XCHG=$x SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py > $O/x_$x.json 2>$O/x_$x.err || exit $?
  python -c "import json; d=json.loads(open('$O/x_$x.json').read().splitlines()[-1]); print('xgmi1 $x', d['ms_per_step'], d['value']/1e6, d['config'].get('calibration'))"
done
timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/w.json 2>$O/w.err || exit $?
SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/wx.json 2>$O/wx.err || exit $?
timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set neg_mode=per_pair > $O/wp.json 2>$O/wp.err || exit $?
for f in w wx wp; do python -c "import json; d=json.loads([l for l in open('$O/$f.json') if l.startswith('{')][-1]); print('$f', d['ms_per_step'], d['samples_per_s']/1e6)"; done
for w in 8 4; do
  timeout -k 10 400 python tools/prof_world.py --world $w --no-prof --out $O/w$w --timeout 300 -- --transport xgmi > $O/w$w.log 2>&1 || { tail -20 $O/w$w.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/w$w/rank0.log') if l.startswith('{')][-1]); print('world$w on one GPU', d['ms_per_step'], d['value']/1e6, d['config'].get('calibration', {}).get('pull_ahead'))"
done
