# k_srv_count with batched source loads and ~256 sub-buckets per workgroup: server tests, then A/B vs the previous commit (_ab/base) at 4 and 8 ranks on one GPU (unique exchange) and one rank
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s40; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_multiproc.py tests/test_gpu_eval_sharded.py tests/test_gpu_oracle.py -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -gt 1 ] && exit $rc
j() { python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1))" "$@"; }
for r in 1 2; do
  for v in new base; do
    D=$R; [ $v = base ] && D=$R/_ab/base
    for w in 8 4; do
      (cd $D && SS_XCHG=unique timeout -k 10 400 python tools/prof_world.py --world $w --no-prof --out $O/w${w}_${v}_$r --timeout 300 -- --transport xgmi --steps 30 --warmup 10 > $O/w${w}_${v}_$r.log 2>&1) || { tail -30 $O/w${w}_${v}_$r.log; exit 1; }
      j $O/w${w}_${v}_$r/rank0.log "world$w $v"
    done
  done
done
echo done
