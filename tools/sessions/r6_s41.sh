# experiment: the next route waits for this round's pull (SS_ROUTE_AFTER_PULL=1) vs the default pipelining, interleaved; kernel trace of the variant
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s41; mkdir -p $O
cd $R
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), d['config']['loss_last'])" "$@"; }
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/$n.json 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  j $O/$n.json "$n"
}
for r in 1 2 3; do
  run def_$r SS_X=0
  run rap_$r SS_ROUTE_AFTER_PULL=1
done
cd /tmp; export PYTHONPATH=$R
SS_ROUTE_AFTER_PULL=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/pipe -o run -- python3 $R/bench.py --steps 24 --warmup 8 > $O/pipe.log 2>&1 || { tail $O/pipe.log; exit 1; }
python3 $R/tools/kstats.py --range timed $O/pipe > $O/pipe_stats.txt 2>&1; head -14 $O/pipe_stats.txt
echo done
