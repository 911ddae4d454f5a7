# PMC passes of rank 0 with 4 and 8 bench ranks on one GPU (N>1 xGMI path, unique-key exchange):
# the server kernels read peers' keys / gradients from the uncached mailboxes (VERDICT r4 Next #1a)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s41; mkdir -p $O
for w in 4 8; do
  i=0
  for set in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "SQ_WAVES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 200 python tools/prof_world.py --world $w --prof-ranks 0 --pmc "$set" --out $O/w$w/p$i --timeout 170 -- --transport xgmi --steps 4 --warmup 2 --cal-steps 0 > $O/w${w}_p$i.log 2>&1; rc=$?
    echo "world $w pass $i ($set) rc=$rc"; tail -2 $O/w${w}_p$i.log
    case $rc in 0) ;; *) exit $rc;; esac
  done
  python tools/pmc_summary.py $O/w$w > $O/w${w}_pmc.md
done
