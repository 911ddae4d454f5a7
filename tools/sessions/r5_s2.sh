set -u
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/s2; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_claim.py tests/test_gpu_xgmi_tiers.py::test_failed_tier_error_bits_do_not_fail_next_tier tests/test_gpu_multiproc.py::test_split_roles_calibration_world3 tests/test_gpu_multiproc.py::test_bench_script_world2_xgmi_one_gpu tests/test_gpu_eval_sharded.py > $O/pytest_claim.log 2>&1
rc=$?; tail -5 $O/pytest_claim.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for v in "c1u:SS_CLAIM=1:uniform" "c0u:SS_CLAIM=0:uniform" "c1z:SS_CLAIM=1:zero" "x1u:SS_CLAIM=1,SS_ENGINE_GENERAL=xgmi:uniform" "x0u:SS_CLAIM=0,SS_ENGINE_GENERAL=xgmi:uniform"; do
    IFS=: read name env init <<< "$v"
    env ${env//,/ } timeout -k 10 200 python bench.py --steps 50 --warmup 10 --init $init > $O/${name}_$r.json 2> $O/${name}_$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/${name}_$r.json').read().strip().splitlines()[-1]); print('$name', d['ms_per_step'], round(d['value']/1e6,1), d['config']['loss_first'], d['config']['loss_last'], d['config']['table_keys'])"
  done
done
cd /tmp && HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_serial -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $O/prof_serial.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pipe -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $O/prof_pipe.log 2>&1
cd $GRAFT_REPO_ROOT && timeout -k 10 180 ./tools/mb_slots 32 5300000 12 > $O/mb_slots.txt 2>&1; cat $O/mb_slots.txt
