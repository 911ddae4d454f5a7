#!/usr/bin/env bash
# One GPU-box session: smoke -> gpu tests -> bench -> rocprofv3 kernel stats.
# Stops at the first fault/abort/timeout (exit 124/134/137/139 or signal);
# an ordinary test failure (pytest exit 1) does not stop the session.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-smoke,tests,bench,prof}
BENCH_ARGS=${BENCH_ARGS:-"--steps 30 --warmup 5"}

fatal() {  # exit code -> is it a fault we must not continue after?
  case "$1" in
    0|1|2|5) return 1 ;;
    *) return 0 ;;
  esac
}

run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/session.log"
  local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a "$OUT/session.log"
  tail -n 15 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name (rc=$rc): stopping session" | tee -a "$OUT/session.log"; exit $rc; fi
  return 0
}

# steps separated by ';' (a custom step may contain spaces and commas)
if [[ "$STEPS" == *";"* ]]; then IFS=';' read -ra STEP_LIST <<< "$STEPS"
else IFS=',' read -ra STEP_LIST <<< "$STEPS"; fi
n=0
for s in "${STEP_LIST[@]}"; do
  n=$((n + 1))
  case $s in
    smoke) run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread ;;
    bench) run bench 600 python bench.py $BENCH_ARGS ;;
    general) run bench_general 600 env SS_ENGINE_GENERAL=rccl python bench.py $BENCH_ARGS ;;
    general_xgmi) run bench_general_xgmi 600 env SS_ENGINE_GENERAL=xgmi python bench.py $BENCH_ARGS ;;
    prof_general) run rocprof_general 600 env SS_ENGINE_GENERAL=rccl rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_general" -o run -- python3 bench.py --steps 10 --warmup 3 ;;
    prof_xgmi) run rocprof_xgmi 600 env SS_ENGINE_GENERAL=xgmi rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_xgmi" -o run -- python3 bench.py --steps 10 --warmup 3 ;;
    rehearse8) run rehearse8 900 python tools/rehearse_world.py --world 8 --steps 20 --warmup 4 ;;
    general3) run bench_general3 600 env SS_ENGINE_GENERAL=rccl SS_RCCL_COMMS=3 python bench.py $BENCH_ARGS ;;
    graph_lr4k) run graph_lr4k 600 env SS_ENGINE_GENERAL=xgmi python bench.py --batch 4096 --steps 64 --warmup 16 --graph on ;;
    eager_lr4k) run eager_lr4k 600 env SS_ENGINE_GENERAL=xgmi python bench.py --batch 4096 --steps 64 --warmup 16 ;;
    fast_lr4k) run fast_lr4k 600 python bench.py --batch 4096 --steps 64 --warmup 16 --graph on ;;
    graph_w2v) run graph_w2v 600 env SS_ENGINE_GENERAL=xgmi python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 ;;
    fast_w2v) run fast_w2v 600 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 ;;
    prof_w2v_x) run rocprof_w2v_x 600 env SS_ENGINE_GENERAL=xgmi rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_w2v_x" -o run -- python3 -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 ;;
    prof_lr4k_x) run rocprof_lr4k_x 600 env SS_ENGINE_GENERAL=xgmi rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_lr4k_x" -o run -- python3 bench.py --batch 4096 --steps 32 --warmup 16 --graph on ;;
    w2v_pp) run w2v_pp 600 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set neg_mode=per_pair ;;
    w2v_pairs_f32) run w2v_pairs_f32 600 env SS_W2V_MFMA=f32 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set w2v_mode=pairs ;;
    w2v_pairs_bf16) run w2v_pairs_bf16 600 python -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16 --set w2v_mode=pairs ;;
    prof_w2v_pp) run rocprof_w2v_pp 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_w2v_pp" -o run -- python3 -m swiftsnails_amd.launch --config configs/word2vec_1m_4x4.conf --steps 32 --warmup 16 --set neg_mode=per_pair ;;
    general_nopa) run bench_general_nopa 600 env SS_ENGINE_GENERAL=rccl SS_PULL_AHEAD=0 python bench.py $BENCH_ARGS ;;
    prof) run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 10 --warmup 3 ;;
    *) run custom$n 600 bash -c "$s" ;;
  esac
done
echo "session done"
