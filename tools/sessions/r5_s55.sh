# FM one GPU: serialised kernel stats and pipelined runs
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s55; mkdir -p $O
timeout -k 10 200 python -m swiftsnails_amd.launch --config configs/fm_10b.conf --steps 40 --warmup 10 --set num_features=1000000000 > $O/fm.json 2>$O/fm.err || { tail -20 $O/fm.err; exit 1; }
python -c "import json; d=json.loads([l for l in open('$O/fm.json') if l.startswith('{')][-1]); print('fm', d['ms_per_step'], d['samples_per_s']/1e6)"
cd /tmp; export PYTHONPATH=$R
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fm_ser -o run -- python3 -m swiftsnails_amd.launch --config $R/configs/fm_10b.conf --steps 20 --warmup 5 --set num_features=1000000000 > $O/fm_ser.log 2>&1 || exit $?
