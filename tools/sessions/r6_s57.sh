# generator: the per-key 64-bit sample multiply replaced by one add per sample group (bit-exact): numpy-generator test, oracle, serialised kernel time, bench
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s57; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gen_ctr or sparse_lr_trains" tests/test_gpu_oracle.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/fser -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/fser.log 2>&1 || { tail $O/fser.log; exit 1; }
python3 $R/tools/kstats.py --range timed --steps 20 $O/fser > $O/fser_stats.txt 2>&1; head -12 $O/fser_stats.txt
cd $R
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 64 --warmup 16 > $O/b_$r.json 2>$O/b_$r.err || { tail $O/b_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), d['config']['loss_last'])" $O/b_$r.json b_$r
done
echo done
