# round 6 HEAD against the round-5 tree (_ab/r5 = commit 1b2e775, built in-tree) on ONE box: bench.py defaults interleaved x4, the N>1 path at one rank x2; then long runs of the calibrated exchange
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s34; mkdir -p $O
cd $R
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['config']; print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), c.get('exchange'), c.get('loss_last'))" "$@"; }
for r in 1 2 3 4; do
  for v in r6 r5; do
    D=$R; [ $v = r5 ] && D=$R/_ab/r5
    (cd $D && timeout -k 10 200 python bench.py > $O/fast_${v}_$r.json 2>$O/fast_${v}_$r.err) || { tail -20 $O/fast_${v}_$r.err; exit 1; }
    j $O/fast_${v}_$r.json "fast $v"
  done
done
for r in 1 2; do
  for v in r6 r5; do
    D=$R; [ $v = r5 ] && D=$R/_ab/r5
    (cd $D && SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py > $O/x_${v}_$r.json 2>$O/x_${v}_$r.err) || { tail -20 $O/x_${v}_$r.err; exit 1; }
    j $O/x_${v}_$r.json "xgmi1 $v"
  done
done
bash tools/sessions/r6_s33.sh
echo done
