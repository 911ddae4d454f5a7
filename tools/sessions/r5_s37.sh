# word2vec per-pair + config-3 N>1 path: serial kernel stats (current tree)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s37; mkdir -p $O
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pp_ser -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 --set neg_mode=per_pair --set graph=0 > $O/pp_ser.log 2>&1 || exit $?
SS_ENGINE_GENERAL=xgmi HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x_ser -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 --set graph=0 > $O/x_ser.log 2>&1 || exit $?
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/w1_ser -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 --set graph=0 > $O/w1_ser.log 2>&1 || exit $?
cd $R
for r in 1 2; do
timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set neg_mode=per_pair > $O/pp_$r.json 2>$O/pp_$r.err || exit $?
SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/x_$r.json 2>$O/x_$r.err || exit $?
done
for f in $O/pp_*.json $O/x_*.json; do python -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['ms_per_step'], d['samples_per_s']/1e6)"; done
