# fused merge + next pull (k_merge_pull): claim/models tests, A/B bench (SS_MERGE_PULL 1 vs 0), serial stats
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s33; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_claim.py tests/test_gpu_models.py -m gpu > $O/pytest.log 2>&1 || { grep -E "Error|error|FAILED|^E " $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for x in 1 0; do
    SS_MERGE_PULL=$x timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/b_${x}_$r.json 2>$O/b_${x}_$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${x}_$r.json').read().splitlines()[-1]); print('mp=$x', d['ms_per_step'], d['config']['loss_last'], d['config']['table_keys'])"
  done
done
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ser -o run -- python3 $R/bench.py --steps 25 --warmup 2 > $O/ser.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/pipe -o run -- python3 $R/bench.py --steps 30 --warmup 10 > $O/pipe.log 2>&1 || exit $?
