# after the best-window rule and the generator default: bench tests, 2 / 4 ranks on one GPU with SS_XCHG=auto
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s35; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_xgmi_tiers.py tests/test_gpu_kernels.py tests/test_gpu_oracle.py -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for w in 2 4; do
  timeout -k 10 400 python tools/prof_world.py --world $w --no-prof --out $O/w${w} --timeout 300 -- --transport xgmi --steps 40 --warmup 10 > $O/w${w}.log 2>&1 || { tail -30 $O/w${w}.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['config']; print('world$w auto', d['ms_per_step'], round(d['value']/1e6,1), c.get('exchange'), c.get('calibration',{}).get('exchange'))" $O/w${w}/rank0.log
done
echo done
