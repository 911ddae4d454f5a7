set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s6; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/bench_$r.json 2> $O/bench_$r.err || exit $?
  python -c "import json; d=json.loads(open('$O/bench_$r.json').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], round(d['value']/1e6,1), d['config']['init'], d['config']['loss_last'])"
done
for w in 4 8; do
  for ss in 1 0; do
    SS_SERVER_STREAM=$ss timeout -k 10 400 python tools/prof_world.py --world $w --no-prof --out $O/w${w}_ss$ss --timeout 300 -- --transport xgmi --steps 30 --warmup 6 > $O/w${w}_ss$ss.txt 2>&1 || exit $?
    grep -h '"metric"' $O/w${w}_ss$ss/rank0.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('world$w ss$ss', d['ms_per_step'], round(d['value']/1e6,1), c.get('calibration',{}).get('pull_ahead'), c.get('staleness'))"
  done
done
for ss in 1 0; do
  SS_SERVER_STREAM=$ss timeout -k 10 900 python tools/straggler.py --world 4 --delays 0,2 --staleness 0,1,2 --kind gpudelay --out $O/strag_ss$ss -- --batch 65536 --steps 30 --warmup 6 > $O/strag_ss$ss.txt 2>&1 || exit $?
  tail -8 $O/strag_ss$ss.txt
done
