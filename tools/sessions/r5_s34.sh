# N>1 servers: response fill fused into the claimed pull (SS_SRV_FILL_FUSED 1 vs 0)
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s34; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_claim.py tests/test_gpu_eval_sharded.py -m gpu > $O/pytest.log 2>&1 || { grep -E "Error|error|FAILED|^E " $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for x in 1 0; do
    SS_SRV_FILL_FUSED=$x SS_ENGINE_GENERAL=xgmi timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cal-steps 0 > $O/x_${x}_$r.json 2>$O/x_${x}_$r.err || exit $?
    python -c "import json; d=json.loads(open('$O/x_${x}_$r.json').read().splitlines()[-1]); print('fused=$x xgmi1', d['ms_per_step'], d['config']['loss_last'])"
  done
done
for x in 1 0; do
  SS_SRV_FILL_FUSED=$x timeout -k 10 400 python tools/prof_world.py --world 4 --no-prof --out $O/w4_$x --timeout 300 -- --transport xgmi --cal-steps 0 > $O/w4_$x.log 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/w4_$x/rank0.log') if l.startswith('{')][-1]); print('fused=$x world4', d['ms_per_step'], d['config']['loss_last'])"
done
