# N>1 path at ONE rank: source bucket target 2048 / 3072 / 4096; word2vec per-pair + config-3 N>1 baselines and a per-pair serial stage profile
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s11; mkdir -p $O
cd $R
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['ms_per_step'],4), round(d.get('value', d.get('samples_per_s', d.get('words_per_s', 0)))/1e6,1))" "$@"; }
for r in 1 2 3; do
  for t in 3072 2048 4096; do
    SS_BD_TARGET_DIST=$t SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/x_${t}_$r.json 2>$O/x_${t}_$r.err || { tail -20 $O/x_${t}_$r.err; exit 1; }
    j $O/x_${t}_$r.json "xgmi1 target=$t"
  done
done
for r in 1 2; do
  timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set neg_mode=per_pair > $O/pp_$r.json 2>$O/pp_$r.err || { tail -20 $O/pp_$r.err; exit 1; }
  j $O/pp_$r.json "w2v per-pair"
  SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/w2vx_$r.json 2>$O/w2vx_$r.err || { tail -20 $O/w2vx_$r.err; exit 1; }
  j $O/w2vx_$r.json "w2v config3 N>1 path"
done
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/pp_ser -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 --set neg_mode=per_pair --set graph=0 > $O/pp_ser.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/pp_pipe -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 --set neg_mode=per_pair --set graph=0 > $O/pp_pipe.log 2>&1 || exit $?
echo done
