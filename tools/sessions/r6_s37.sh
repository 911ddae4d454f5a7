# word2vec config 3 shape, graph replay (as measured): kernel traces of the one-GPU path and the N>1 path at one rank, for the per-stream timeline
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s37; mkdir -p $O
cd /tmp; export PYTHONPATH=$R
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/fast -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/fast.log 2>&1 || { tail $O/fast.log; exit 1; }
SS_ENGINE_GENERAL=xgmi timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/x1 -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 > $O/x1.log 2>&1 || { tail $O/x1.log; exit 1; }
grep -h "ms_per_step" $O/fast.log $O/x1.log | cut -c1-200
echo done
