# grouped records at 2 ranks on one GPU: rank 0's kernel stats (what makes the step 10 ms)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s45; mkdir -p $O
cd $R
SS_XCHG=records SS_REC_GROUP=1 timeout -k 10 300 python tools/prof_world.py --world 2 --prof-ranks 0 --out $O/w2 --timeout 200 -- --transport xgmi --steps 10 --warmup 4 --cal-steps 0 > $O/w2.log 2>&1; echo "rc=$?"
python - "$O/w2/rank0/run_kernel_trace.csv" <<'PY'
import csv, collections, sys
rows=list(csv.DictReader(open(sys.argv[1])))
tot=collections.Counter(); cnt=collections.Counter(); mx=collections.Counter()
for r in rows:
    n=r["Kernel_Name"].split("(")[0].replace("void ","")[:44]
    d=(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3
    tot[n]+=d; cnt[n]+=1; mx[n]=max(mx[n],d)
for n,t in tot.most_common(16):
    print(f"{n:46s} calls {cnt[n]:5d} avg {t/cnt[n]:9.1f} max {mx[n]:9.1f} us")
PY
echo done
