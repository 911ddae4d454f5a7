# fast path at the bench shape: eager (default) vs --graph on, interleaved pairs on one box
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s51; mkdir -p $O
cd $R
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), d['config']['hipgraph'], d['config']['loss_last'])" "$@"; }
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 64 --warmup 16 > $O/e_$r.json 2>$O/e_$r.err || { tail -20 $O/e_$r.err; exit 1; }
  j $O/e_$r.json "eager_$r"
  timeout -k 10 200 python bench.py --steps 64 --warmup 16 --graph on > $O/g_$r.json 2>$O/g_$r.err || { tail -20 $O/g_$r.err; exit 1; }
  j $O/g_$r.json "graph_$r"
done
echo done
