# word2vec config 3 shape: one-GPU fast path vs the N>1 path at one rank, serialised kernel stats (graph replay off for the trace)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s30; mkdir -p $O
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/fast -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 --set graph=0 > $O/fast.log 2>&1 || { tail $O/fast.log; exit 1; }
python3 $R/tools/kstats.py $O/fast 32 > $O/fast_stats.txt 2>&1; head -30 $O/fast_stats.txt
SS_ENGINE_GENERAL=xgmi HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/x1 -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 --set graph=0 > $O/x1.log 2>&1 || { tail $O/x1.log; exit 1; }
python3 $R/tools/kstats.py $O/x1 32 > $O/x1_stats.txt 2>&1; head -40 $O/x1_stats.txt
echo done
