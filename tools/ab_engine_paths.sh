#!/usr/bin/env bash
# A/B of the 1-GPU fast path vs the N>1 engine path (three size-1 RCCL
# communicators) on one box, plus a kernel trace of the N>1 path.
# Stops at the first failing step.
set -eu
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/ab
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${ARGS:-"--steps 40 --warmup 8"}
b() {  # name env...
  local name=$1; shift
  echo "== $name: $*"
  env "$@" timeout -k 10 300 python bench.py $ARGS > "$OUT/$name.json" 2> "$OUT/$name.err"
  python -c "import json,sys;d=json.loads([l for l in open('$OUT/$name.json') if l.startswith('{')][-1]);print('$name', d['ms_per_step'], 'ms/step', round(d['value']/1e6,1), 'M/s')"
}
for rep in 1 2; do
  b fast_$rep SS_ENGINE_GENERAL=0
  b general_$rep SS_ENGINE_GENERAL=rccl
  b general_nopa_$rep SS_ENGINE_GENERAL=rccl SS_PULL_AHEAD=0
done
if [ "${PROF:-1}" = 1 ]; then
  SS_ENGINE_GENERAL=rccl timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_general" -o run -- python3 bench.py --steps 10 --warmup 3 > "$OUT/prof_general.log" 2>&1
fi
echo ab done
