# word2vec config-3 shape through the N>1 path at one rank (graph replay): time + kernel stats, eager for comparison
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s56; mkdir -p $O
cd $R
j() { python3 -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d['ms_per_step'],4), round(d['samples_per_s']/1e6,1), d.get('hipgraph'))" "$@"; }
SS_ENGINE_GENERAL=xgmi timeout -k 10 300 python3 -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 400 --warmup 20 > $O/g.log 2>&1 || { tail -20 $O/g.log; exit 1; }
j $O/g.log graph
SS_ENGINE_GENERAL=xgmi timeout -k 10 300 python3 -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 400 --warmup 20 --set graph=0 > $O/e.log 2>&1 || { tail -20 $O/e.log; exit 1; }
j $O/e.log eager
timeout -k 10 300 python3 -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 400 --warmup 20 > $O/f.log 2>&1 || { tail -20 $O/f.log; exit 1; }
j $O/f.log fast1
cd /tmp; export PYTHONPATH=$R SS_ENGINE_GENERAL=xgmi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/word2vec_1m_4x4.conf --steps 200 --warmup 20 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
head -30 $O/prof/run_kernel_stats.csv | cut -d, -f1-4
echo done
