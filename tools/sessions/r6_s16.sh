# sorted scatter tile (SS_BD_SKT 16 vs 8: 140 vs ~76 KB of LDS per 1024-thread workgroup — in the pipelined N>1 trace the scatter runs 258 us against 101 standalone, waiting for a CU with that much LDS free)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s16; mkdir -p $O
cd $R
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1))" "$@"; }
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/$n.json 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  j $O/$n.json "$n"
}
for r in 1 2 3; do
  run x16_$r SS_ENGINE_GENERAL=xgmi SS_BD_SKT=16
  run x8_$r SS_ENGINE_GENERAL=xgmi SS_BD_SKT=8
done
for r in 1 2 3; do
  run f16_$r SS_BD_SKT=16
  run f8_$r SS_BD_SKT=8
done
for v in 16 8; do
  SS_BD_SKT=$v timeout -k 10 500 python tools/prof_world.py --world 4 --no-prof --out $O/w4_$v --timeout 400 -- --transport xgmi --steps 30 --warmup 10 > $O/w4_$v.log 2>&1 || { tail -20 $O/w4_$v.log; exit 1; }
  j $O/w4_$v/rank0.log "world4 skt=$v"
done
echo done
