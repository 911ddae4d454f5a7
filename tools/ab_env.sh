#!/usr/bin/env bash
# A/B of bench.py under environment variants on one box, interleaved reps.
#   VARIANTS="name1:K=V,K=V name2:K=V" REPS=2 ARGS="--steps 40 --warmup 8" tools/ab_env.sh
# CMD overrides the program (default "python bench.py"), e.g. the launcher:
#   CMD="python -m swiftsnails_amd.launch" ARGS="--config configs/word2vec_1m_4x4.conf ..."
set -eu
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/abenv
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${ARGS:-"--steps 40 --warmup 8"}
CMD=${CMD:-"python bench.py"}
REPS=${REPS:-2}
for rep in $(seq 1 "$REPS"); do
  for v in $VARIANTS; do
    name=${v%%:*}; kv=${v#*:}
    envs=()
    if [ "$kv" != "$v" ] && [ -n "$kv" ]; then IFS=, read -ra envs <<< "$kv"; fi
    env "${envs[@]}" timeout -k 10 300 $CMD $ARGS > "$OUT/${name}_$rep.json" 2> "$OUT/${name}_$rep.err"
    python - "$OUT/${name}_$rep.json" "$name" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
v = d.get("value", d.get("samples_per_s", 0.0))
loss = d.get("loss", d.get("config", {}).get("loss_last"))
print(f"{sys.argv[2]:24s} {d['ms_per_step']:.4f} ms/step {v/1e6:7.1f} M/s loss {loss}")
PY
  done
done
echo abenv done
