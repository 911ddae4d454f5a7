# final tree: the other configurations on one GPU (launcher), 2 runs each: word2vec window (graph), word2vec per-pair, FM 1B, sparse LR 10M, sparse LR batch 65536
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s55; mkdir -p $O
cd $R
j() { python3 -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d['ms_per_step'],4), round(d['samples_per_s']/1e6,1), d.get('hipgraph'), d.get('loss'))" "$@"; }
run() {  # name args...
  local n=$1; shift
  timeout -k 10 300 python3 -m swiftsnails_amd.launch "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -20 $O/$n.log; exit 1; }
  j $O/$n.log $n
}
for r in 1 2; do
  run w2v_window_$r --config configs/word2vec_1m_4x4.conf --steps 200 --warmup 20
  run w2v_pp_$r --config configs/word2vec_1m_4x4.conf --steps 100 --warmup 10 --set neg_mode=per_pair --set graph=0
  run fm1b_$r --config configs/fm_10b.conf --steps 100 --warmup 10 --set num_features=1000000000
  run lr10m_$r --config configs/sparse_lr_10m.conf --steps 100 --warmup 10
done
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --batch 65536 --steps 100 --warmup 10 > $O/b64k_$r.json 2>$O/b64k_$r.err || { tail $O/b64k_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1))" $O/b64k_$r.json b64k_$r
done
echo done
