# LR forward sample groups per workgroup (SS_LR_FWD_R 4 / 2 / 1) and reduce workgroup shapes (SS_BD_RT / SS_BD_ROCC): tests, A/B, serial stats
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s10; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_oracle.py tests/test_gpu_claim.py -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log
[ $rc -gt 1 ] && exit $rc
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1))" "$@"; }
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/$n.json 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  j $O/$n.json "$n"
}
for r in 1 2 3; do
  run def_$r SS_LR_FWD_R=4
  run fwd1_$r SS_LR_FWD_R=1
  run fwd2_$r SS_LR_FWD_R=2
  run rt512o8_$r SS_BD_RT=512 SS_BD_ROCC=8
  run rt512o4_$r SS_BD_RT=512 SS_BD_ROCC=4
done
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/ser_def -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/ser_def.log 2>&1 || exit $?
SS_BD_RT=512 SS_BD_ROCC=8 HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/ser_rt512 -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/ser_rt512.log 2>&1 || exit $?
echo done
