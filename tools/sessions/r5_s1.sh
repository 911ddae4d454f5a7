set -u
export TMPDIR=/tmp
O=gpurun_out/s1; mkdir -p $O
for r in 1 2 3; do
  for v in zero uniform; do
    timeout -k 10 200 python bench.py --steps 50 --warmup 10 --init $v > $O/${v}_$r.json 2> $O/${v}_$r.err || exit $?
    python -c "import json,sys; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['value']/1e6)"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_u -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --init uniform > $GRAFT_REPO_ROOT/$O/prof_u.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_z -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --init zero > $GRAFT_REPO_ROOT/$O/prof_z.log 2>&1
