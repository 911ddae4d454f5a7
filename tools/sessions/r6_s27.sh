# what the uncached mailbox costs its local readers at one rank: SS_XGMI_CACHED=1 vs 0 (LR unique / records, word2vec config 3 N>1 path)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s27; mkdir -p $O
cd $R
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d.get('value',0)/1e6,1))" "$@"; }
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/$n.json 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  j $O/$n.json "$n"
}
w2v() {
  local n=$1; shift
  env "$@" SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/$n.json 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  j $O/$n.json "$n"
}
for r in 1 2; do
  run u0_$r SS_ENGINE_GENERAL=xgmi SS_XCHG=unique SS_XGMI_CACHED=0
  run u1_$r SS_ENGINE_GENERAL=xgmi SS_XCHG=unique SS_XGMI_CACHED=1
  run r0_$r SS_ENGINE_GENERAL=xgmi SS_XCHG=records SS_XGMI_CACHED=0
  run r1_$r SS_ENGINE_GENERAL=xgmi SS_XCHG=records SS_XGMI_CACHED=1
  w2v w0_$r SS_XGMI_CACHED=0
  w2v w1_$r SS_XGMI_CACHED=1
done
echo done
