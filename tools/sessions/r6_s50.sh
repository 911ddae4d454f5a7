# after the >4-ranks-per-GPU graph guard: config 3 split 4+4 and colocated 8 with graph: 1 now run eager rounds
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s50; mkdir -p $O
cd $R
export GLOO_SOCKET_IFNAME=lo SS_DEVICE=0 PYTHONPATH=$R SS_XGMI_TIMEOUT=60
run() {  # name nproc graph extra-set...
  local n=$1 np=$2 g=$3; shift 3
  local sets=(); for kv in "$@"; do sets+=(--set "$kv"); done
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) \
    -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 200 --warmup 20 \
    --set transport=xgmi --set graph=$g --set round_timeout=120 "${sets[@]}" > $O/$n.log 2>&1 || { echo "$n failed rc=$?"; tail -30 $O/$n.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['world'], d['servers'], d['workers'], d['hipgraph'], round(d['ms_per_step'],4), round(d['samples_per_s']/1e6,1))" $O/$n.log $n
}
run split44_graph 8 1 server_ranks=0,1,2,3 worker_ranks=4,5,6,7
run coloc8_graph 8 1
run coloc4_graph 4 1
echo done
