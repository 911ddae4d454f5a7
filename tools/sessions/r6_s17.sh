# re-entry baseline: fast path, N>1 path at one rank (unique), record exchange at one rank; interleaved
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s17; mkdir -p $O
cd $R
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1))" "$@"; }
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/$n.json 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  j $O/$n.json "$n"
}
for r in 1 2 3; do
  run fast_$r SS_X=0
  run xu_$r SS_ENGINE_GENERAL=xgmi
  run xr_$r SS_ENGINE_GENERAL=xgmi SS_XCHG=records
done
echo done
