# multi-tensor weight path: GPU tests + C4 bench + rocprof (experiment script)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_calib.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_multi.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/t_multi.log; exit 1; }
tail -2 gpurun_out/t_multi.log
timeout -k 10 300 python3 -u bench.py --workload c4 --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/b_c4.log 2>&1 || { echo "bench rc=$?"; tail gpurun_out/b_c4.log; exit 1; }
tail -1 gpurun_out/b_c4.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4m -o run --output-format csv -- python3 -u bench.py --workload c4 --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/p_c4.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo done
