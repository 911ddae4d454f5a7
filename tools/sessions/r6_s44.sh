# grouped records debug: world 2 / 4 at the bench shape and at batch 65536, the server error decoded
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s44; mkdir -p $O
cd $R
for w in 2 4; do
  for b in 65536 262144; do
    SS_XCHG=records SS_REC_GROUP=1 timeout -k 10 300 python tools/prof_world.py --world $w --no-prof --out $O/w${w}_$b --timeout 200 -- --transport xgmi --steps 10 --warmup 4 --batch $b --cal-steps 0 > $O/w${w}_$b.log 2>&1
    echo "world $w batch $b rc=$?"
    grep -h "DedupOverflow\|ms_per_step" $O/w${w}_$b/rank0.log | cut -c1-400 | tail -2
  done
done
echo done
