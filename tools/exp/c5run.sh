set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_calib.py tests/test_abi_cpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_calib.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_calib.log; exit 1; }
tail -2 gpurun_out/t_calib.log
timeout -k 10 300 python3 -u bench.py --workload c5 --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/b_c5.log 2>&1 || { echo "bench rc=$?"; tail gpurun_out/b_c5.log; exit 1; }
tail -1 gpurun_out/b_c5.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5p -o run --output-format csv -- python3 -u bench.py --workload c5 --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/p_c5.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo done
