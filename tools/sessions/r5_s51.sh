# one source needs no server sub-buckets (srv_sub_buckets(1) = 1 again): N>1 path tests at world 1 and 2-4, the 1-rank N>1 bench
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s51; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gpu_xgmi_tiers.py tests/test_gpu_claim.py tests/test_gpu_eval_sharded.py "tests/test_gpu_models.py::test_record_exchange_world1_matches_unique" "tests/test_gpu_models.py::test_graph_capture_after_mode_switch_xgmi" -m gpu > $O/pytest.log 2>&1 || { grep -E "Error|error|FAILED|^E " $O/pytest.log | head -40; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for x in unique records; do
    SS_XCHG=$x SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cal-steps 0 > $O/x_${x}_$r.json 2>$O/x_${x}_$r.err || { tail -20 $O/x_${x}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/x_${x}_$r.json').read().splitlines()[-1]); print('$x xgmi1', d['ms_per_step'], d['config']['loss_last'])"
  done
done
