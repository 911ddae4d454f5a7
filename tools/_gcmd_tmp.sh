set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1 || { tail -60 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err
cut -c1-220 gpurun_out/bench.json
VARIANTS="gen:SS_ENGINE_GENERAL=rccl" REPS=1 ARGS="--steps 60 --warmup 10" bash tools/ab_env.sh
A="--config configs/word2vec_1m_4x4.conf --steps 300 --warmup 10 --set server_ranks=all --set worker_ranks=all --set table_stats=0"
VARIANTS="w2v_win:SS_X=1" REPS=1 CMD="python -m swiftsnails_amd.launch" ARGS="$A" bash tools/ab_env.sh
VARIANTS="w2v_pairs:SS_X=1" REPS=1 CMD="python -m swiftsnails_amd.launch" ARGS="$A --set w2v_mode=pairs" bash tools/ab_env.sh
F="--config configs/fm_10b.conf --steps 60 --warmup 5 --set num_features=1000000000 --set table_stats=0"
VARIANTS="fm:SS_X=1" REPS=1 CMD="python -m swiftsnails_amd.launch" ARGS="$F" bash tools/ab_env.sh
A2="--config configs/word2vec_1m_4x4.conf --steps 20 --warmup 3 --set server_ranks=all --set worker_ranks=all --set table_stats=0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_w2v_final -o run -- python3 -m swiftsnails_amd.launch $A2 > gpurun_out/prof_w2v_final.log 2>&1
