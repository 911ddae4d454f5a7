set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > $OUT/t_kern.log 2>&1 || { tail -30 $OUT/t_kern.log; exit 1; }
tail -1 $OUT/t_kern.log
for v in "SS_X=0" "SS_BD_CT=256" "SS_BD_CT=512" "SS_ENGINE_GENERAL=1" "SS_ENGINE_GENERAL=1 SS_BD_CT=256"; do
  env $v timeout -k 10 120 python bench.py --steps 50 --warmup 10 > $OUT/b_x.log 2>&1 || { tail -20 $OUT/b_x.log; exit 2; }
  echo "$v: $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_x.log) $(grep -o '"unique_keys_per_step_per_gpu": [0-9]*' $OUT/b_x.log)"
done
SS_ENGINE_GENERAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_gen -o run -- python3 bench.py --steps 10 --warmup 3 > $OUT/prof_gen.log 2>&1
echo rc=$?
