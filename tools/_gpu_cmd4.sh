set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
for v in "SS_ENGINE_GENERAL=1" "SS_ENGINE_GENERAL=1 SS_PULL_AHEAD=0" ; do
  env $v timeout -k 10 120 python bench.py --steps 50 --warmup 10 > $OUT/b_gen.log 2>&1 || { tail -20 $OUT/b_gen.log; exit 2; }
  echo "$v: $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_gen.log)"
done
SS_ENGINE_GENERAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_gen -o run -- python3 bench.py --steps 10 --warmup 3 > $OUT/prof_gen.log 2>&1
echo rc=$?
