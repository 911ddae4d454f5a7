# SS_XCHG=auto at 8 ranks on one GPU (start-up with both engines' arenas, calibration, teardown) 
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s24; mkdir -p $O
cd $R
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['config']; print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), c['loss_last'], c.get('exchange'), c.get('calibration',{}).get('exchange'))" "$@"; }
timeout -k 10 600 python tools/prof_world.py --world 8 --no-prof --out $O/w8_auto --timeout 500 -- --transport xgmi --steps 30 --warmup 10 > $O/w8_auto.log 2>&1 || { tail -30 $O/w8_auto.log; exit 1; }
j $O/w8_auto/rank0.log "world8 auto"
grep -h "VmHWM\|peak" $O/w8_auto/*.log | head -3
echo done
