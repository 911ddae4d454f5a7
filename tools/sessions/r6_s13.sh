# word2vec (per-pair and config 3, 1 GPU): count / column-scan workgroup sizes (SS_BD_CNT / SS_BD_CS 256 vs 1024) — the pipelined per-pair trace shows k_bd_count at 233 us (8 standalone) waiting for CU slots
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s13; mkdir -p $O
cd $R
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['ms_per_step'],4), round(d.get('words_per_s', d.get('samples_per_s', 0))/1e6,1))" "$@"; }
run() {  # name extra-args env...
  local n=$1 x=$2; shift 2
  env "$@" timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 $x > $O/$n.json 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  j $O/$n.json "$n"
}
for r in 1 2 3; do
  run pp_def_$r "--set neg_mode=per_pair" SS_BD_CNT=1024
  run pp_c256_$r "--set neg_mode=per_pair" SS_BD_CNT=256
  run pp_cs256_$r "--set neg_mode=per_pair" SS_BD_CNT=256 SS_BD_CS=256
done
for r in 1 2; do
  run w_def_$r "" SS_BD_CNT=1024
  run w_cs256_$r "" SS_BD_CNT=256 SS_BD_CS=256
done
for r in 1 2; do
  for v in 1024 256; do
    SS_BD_CNT=$v SS_BD_CS=$v timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/lr_${v}_$r.json 2>$O/lr_${v}_$r.err || { tail -20 $O/lr_${v}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/lr_${v}_$r.json').read().splitlines()[-1]); print('lr cnt/cs=$v', d['ms_per_step'])"
  done
done
echo done
