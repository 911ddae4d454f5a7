# long runs of the N>1 path (N bench ranks on one GPU, xGMI mailboxes, SS_XCHG=auto): a short and a long run per world on one box — drift of the per-round time while the shards fill, engine.check() after thousands of mailbox rounds
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s53; mkdir -p $O
cd $R
j() { python3 -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['config']
print(sys.argv[2], d['steps'], d['ms_per_step'], round(d['value']/1e6,1), c.get('exchange'), c.get('table_keys'), c.get('loss_first'), c.get('loss_last'))" "$@"; }
run() {  # name world steps warmup
  timeout -k 10 500 python3 tools/prof_world.py --world $2 --no-prof --timeout 480 --out $O/$1 -- --transport xgmi --steps $3 --warmup $4 > $O/$1.out 2>&1 || { echo "$1 failed"; tail -5 $O/$1.out; tail -20 $O/$1/rank0.log; exit 1; }
  grep '^{' $O/$1.out > $O/$1.json; j $O/$1.json $1
}
run w2_short 2 200 10
run w2_long 2 3000 10
run w4_short 4 200 10
run w4_long 4 2000 10
run w8_short 8 100 10
run w8_long 8 1000 10
echo done
