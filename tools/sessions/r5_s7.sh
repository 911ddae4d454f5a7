set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s7; mkdir -p $O
for r in 1 2; do
  for c in 1 0; do
    SS_CLAIM=$c timeout -k 10 400 python tools/prof_world.py --world 4 --no-prof --out $O/w4_c${c}_$r --timeout 300 -- --transport xgmi --steps 30 --warmup 6 > /dev/null 2>&1 || exit $?
    grep -h '"metric"' $O/w4_c${c}_$r/rank0.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('world4 claim$c', d['ms_per_step'], round(d['value']/1e6,1), c.get('staleness'), c.get('server_unique_keys_per_step'))"
  done
done
timeout -k 10 400 python tools/prof_world.py --world 8 --no-prof --out $O/w8 --timeout 300 -- --transport xgmi --steps 30 --warmup 6 > /dev/null 2>&1 || exit $?
grep -h '"metric"' $O/w8/rank0.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('world8', d['ms_per_step'], round(d['value']/1e6,1), c.get('staleness'), c.get('calibration'))"
timeout -k 10 400 python tools/prof_world.py --world 4 --no-prof --out $O/lk4 --timeout 300 --script tools/lookup_bench.py -- --keys 2500000 --steps 6 > /dev/null 2>&1 || exit $?
grep -h '"ms_device"' $O/lk4/rank0.log
