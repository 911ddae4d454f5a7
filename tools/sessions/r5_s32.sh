# k_bd_reduce with 4 occurrences per thread in flight vs the committed tree (_ab/base)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s32; mkdir -p $O
for r in 1 2 3; do
  for v in new base; do
    d=$R; [ $v = base ] && d=$R/_ab/base
    (cd $d && timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b_${v}_$r.json 2>$O/b_${v}_$r.err) || exit $?
    (cd $d && SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/x_${v}_$r.json 2>$O/x_${v}_$r.err) || exit $?
    python -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().splitlines()[-1]); x=json.loads(open('$O/x_${v}_$r.json').read().splitlines()[-1]); print('$v', d['ms_per_step'], 'xgmi', x['ms_per_step'], x['config']['loss_last'])"
  done
done
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ser -o run -- python3 $R/bench.py --steps 25 --warmup 2 > $O/ser.log 2>&1 || exit $?
SS_ENGINE_GENERAL=xgmi HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serx -o run -- python3 $R/bench.py --steps 25 --warmup 2 --cal-steps 0 > $O/serx.log 2>&1 || exit $?
