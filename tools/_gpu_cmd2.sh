set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_default -o run -- python3 bench.py --steps 10 --warmup 3 > $OUT/prof_default.log 2>&1 && \
SS_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --transport gloo --batch 65536 > $OUT/bench_gloo2.log 2>&1
echo rc=$?
