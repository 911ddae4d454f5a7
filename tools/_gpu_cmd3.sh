set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "dedup or bd" > $OUT/t_dedup.log 2>&1 || exit 1
for nch in 4096 512 256; do
  SS_BD_NCH=$nch timeout -k 10 120 python bench.py --steps 50 --warmup 10 > $OUT/b_nch$nch.log 2>&1 || exit 2
  grep -o '"value": [0-9.]*, "unit[^,]*, "n_gpus[^,]*, "steps[^,]*, "warmup[^,]*, "ms_per_step": [0-9.]*' $OUT/b_nch$nch.log
done
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_serial -o run -- python3 bench.py --steps 5 --warmup 3 > $OUT/prof_serial.log 2>&1
echo rc=$?
