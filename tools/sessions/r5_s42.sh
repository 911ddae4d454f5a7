# record layout as a per-deduper bit: record / xgmi GPU tests, 1-rank and 4-rank record runs
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s42; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py::test_server_bucket_past_parking_area "tests/test_gpu_models.py::test_record_exchange_world1_matches_unique" tests/test_gpu_eval_sharded.py tests/test_gpu_xgmi_tiers.py tests/test_gpu_claim.py -m gpu > $O/pytest.log 2>&1 || { grep -E "Error|error|FAILED|^E " $O/pytest.log | head -40; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for x in records unique; do
  SS_XCHG=$x SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cal-steps 0 > $O/x_$x.json 2>$O/x_$x.err || { tail -20 $O/x_$x.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/x_$x.json').read().splitlines()[-1]); print('$x xgmi1', d['ms_per_step'], d['config']['loss_last'])"
  SS_XCHG=$x timeout -k 10 400 python tools/prof_world.py --world 4 --no-prof --out $O/w4_$x --timeout 300 -- --transport xgmi --cal-steps 0 > $O/w4_$x.log 2>&1 || { tail -20 $O/w4_$x.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/w4_$x/rank0.log') if l.startswith('{')][-1]); print('$x world4', d['ms_per_step'], d['config']['loss_last'])"
done
