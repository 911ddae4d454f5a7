# N>1 unique layout default 3072 occurrences per source bucket: full GPU suite, then 3072 vs 4096 at 4 / 8 ranks, bench
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s50; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
case $rc in 0) ;; 1) grep -E "FAILED|^E " $O/pytest.log | head -20; exit 1;; *) echo "pytest rc=$rc"; exit $rc;; esac
for w in 8 4; do
  for t in 4096 3072; do
    SS_BD_TARGET_DIST=$t timeout -k 10 400 python tools/prof_world.py --world $w --no-prof --out $O/w${w}_$t --timeout 300 -- --transport xgmi --cal-steps 0 > $O/w${w}_$t.log 2>&1 || { tail -20 $O/w${w}_$t.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/w${w}_$t/rank0.log') if l.startswith('{')][-1]); print('world$w target=$t', d['ms_per_step'], d['config']['loss_last'], d['config']['server_unique_keys_per_step'])"
  done
done
timeout -k 10 200 python bench.py > $O/b.json 2>$O/b.err || exit $?
python -c "import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); print('bench', d['ms_per_step'], d['value']/1e6)"
