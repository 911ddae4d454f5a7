# SS_XCHG=auto at 8 ranks on one GPU after the room check (expect: unique only, no hang); 4 ranks auto (both fit)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s26; mkdir -p $O
cd $R
for w in 8 4; do
  timeout -k 10 400 python tools/prof_world.py --world $w --no-prof --out $O/w${w}_auto --timeout 300 -- --transport xgmi --steps 30 --warmup 10 > $O/w${w}_auto.log 2>&1 || { tail -30 $O/w${w}_auto.log; grep -h "bench.py:" $O/w${w}_auto/*.log | sort | uniq -c; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['config']; print('world$w auto', d['ms_per_step'], round(d['value']/1e6,1), c.get('exchange'), c.get('calibration',{}).get('exchange'))" $O/w${w}_auto/rank0.log
  grep -h "bench.py:" $O/w${w}_auto/*.log | sort | uniq -c
done
echo done
