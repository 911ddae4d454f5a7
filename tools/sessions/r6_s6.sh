# k_bd_reduce occurrences in flight (SS_BD_ROCC 4 vs 2): changed-kernel tests, fast and N>1 1-rank A/B pairs, 4 ranks on one GPU
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s6; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_oracle.py tests/test_gpu_claim.py tests/test_gpu_kernels.py -q -rf --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -gt 1 ] && exit $rc
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1))" "$@"; }
for r in 1 2 3; do
  for v in 4 2; do
    SS_BD_ROCC=$v timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/fast_${v}_$r.json 2>$O/fast_${v}_$r.err || { tail -20 $O/fast_${v}_$r.err; exit 1; }
    j $O/fast_${v}_$r.json "fast rocc=$v"
  done
done
for r in 1 2; do
  for v in 4 2; do
    SS_BD_ROCC=$v SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/x_${v}_$r.json 2>$O/x_${v}_$r.err || { tail -20 $O/x_${v}_$r.err; exit 1; }
    j $O/x_${v}_$r.json "xgmi1 rocc=$v"
  done
done
for v in 4 2; do
  SS_BD_ROCC=$v timeout -k 10 500 python tools/prof_world.py --world 4 --no-prof --out $O/w4_$v --timeout 400 -- --transport xgmi --steps 30 --warmup 10 > $O/w4_$v.log 2>&1 || { tail -20 $O/w4_$v.log; exit 1; }
  j $O/w4_$v/rank0.log "world4 rocc=$v"
done
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/fast_ser -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/fast_ser.log 2>&1 || exit $?
HIP_LAUNCH_BLOCKING=1 SS_ENGINE_GENERAL=xgmi timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/x_ser -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/x_ser.log 2>&1 || exit $?
echo done
