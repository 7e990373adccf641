# config 5 (512^3): plain timing without event timers, then a kernel trace for the launch gaps
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
A="--shape 512 512 512 --batch 1 --morph3d --steps 2 --warmup 1 --no-cpu-baseline --no-h2h"
timeout -k 10 300 python3 bench.py $A --no-profile > gpurun_out/r3t_c5np.json 2> gpurun_out/r3t_c5np.err || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/r3t_c5np.json').read());print('noprof', d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3t_c5tr -o run -- python3 bench.py $A --no-profile > gpurun_out/r3t_c5tr.log 2>&1
echo "rocprof rc=$?"
ls gpurun_out/r3t_c5tr
exit 0
