# long runs of the exchange the calibration picks: one rank through the N>1 path (records) 600 steps, 2 ranks on one GPU (records) 300 steps; table checks at the end
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s33; mkdir -p $O
cd $R
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['config']; print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), c.get('exchange'), 'loss', c['loss_first'], '->', c['loss_last'], 'keys', c['table_keys'])" "$@"; }
SS_ENGINE_GENERAL=xgmi timeout -k 10 300 python bench.py --steps 600 --warmup 10 > $O/x1_600.json 2>$O/x1_600.err || { tail -20 $O/x1_600.err; exit 1; }
j $O/x1_600.json "one rank auto 600 steps"
timeout -k 10 400 python tools/prof_world.py --world 2 --no-prof --out $O/w2 --timeout 300 -- --transport xgmi --steps 300 --warmup 10 > $O/w2.log 2>&1 || { tail -30 $O/w2.log; exit 1; }
j $O/w2/rank0.log "world2 auto 300 steps"
echo done
