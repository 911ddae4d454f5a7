# 8 sample groups per workgroup for the generator (SS_GEN_R) and the LR forward (SS_LR_FWD_R) vs 4: numerics tests, A/B, serial stats
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s32; mkdir -p $O
cd $R
SS_GEN_R=8 SS_LR_FWD_R=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_oracle.py -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['config']; print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), c['loss_last'])" "$@"; }
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/$n.json 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  j $O/$n.json "$n"
}
for r in 1 2 3; do
  run d44_$r SS_GEN_R=4 SS_LR_FWD_R=4
  run d84_$r SS_GEN_R=8 SS_LR_FWD_R=4
  run d48_$r SS_GEN_R=4 SS_LR_FWD_R=8
done
cd /tmp; export PYTHONPATH=$R
SS_GEN_R=8 SS_LR_FWD_R=8 HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/ser8 -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/ser8.log 2>&1 || { tail $O/ser8.log; exit 1; }
python3 $R/tools/kstats.py --range timed $O/ser8 > $O/ser8_stats.txt 2>&1; grep -E "gen_ctr|lr_fwd" $O/ser8_stats.txt | head -4
echo done
