# record path at one rank: k_rec_grad hand-off grid fix check (serial), A/B vs fast; PMC FETCH/WRITE passes (longer limit: the start-up litmus runs under the counters too)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s29; mkdir -p $O
cd $R
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['config']; print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), c.get('exchange'))" "$@"; }
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/$n.json 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  j $O/$n.json "$n"
}
for r in 1 2; do
  run fast_$r SS_X=0
  run xauto_$r SS_ENGINE_GENERAL=xgmi
done
cd /tmp; export PYTHONPATH=$R
export SS_ENGINE_GENERAL=xgmi SS_XCHG=records
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/ser -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/ser.log 2>&1 || { tail $O/ser.log; exit 1; }
python3 $R/tools/kstats.py --range timed $O/ser > $O/ser_stats.txt 2>&1; grep -E "rec_grad|per-step" $O/ser_stats.txt
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 280 rocprofv3 --kernel-trace --stats --pmc $set --output-format csv -d $O/pmc/p$i -o run -- python3 $R/bench.py --steps 4 --warmup 2 --cal-steps 0 > $O/pmc_p$i.log 2>&1 || { echo "pmc pass $i rc=$?"; tail -3 $O/pmc_p$i.log; exit 1; }
  echo "pmc pass $i ok"
done
python3 $R/tools/pmc_summary.py $O/pmc --by-grid > $O/pmc_summary.md 2>&1; cat $O/pmc_summary.md
echo done
