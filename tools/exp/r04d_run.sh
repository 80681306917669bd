# round 4: K2o at G=2 (block-size variants), the fold, C5 leg + kernel trace + PMC
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_silu.py tests/test_gpu_c5_calib.py tests/test_gpu_calib.py tests/test_gpu_dist_calib.py -x -q --timeout 120 --timeout-method thread -k "parts_out or c5 or calib or defer or fold" > gpurun_out/t_r04d.log 2>&1 || { echo "tests rc=$?"; tail -60 gpurun_out/t_r04d.log; exit 1; }
tail -2 gpurun_out/t_r04d.log
timeout -k 10 300 python -u tools/exp/k2o_bench.py 20 > gpurun_out/k2o_bench2.log 2>&1 || { echo "k2o bench rc=$?"; tail gpurun_out/k2o_bench2.log; exit 1; }
cat gpurun_out/k2o_bench2.log
timeout -k 10 300 python3 -u bench.py --workload c5 --steps 32 --warmup 4 > gpurun_out/b_c5.log 2>&1 || { echo "bench c5 rc=$?"; tail gpurun_out/b_c5.log; exit 1; }
tail -1 gpurun_out/b_c5.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 -u bench.py --workload c5 --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1 || { echo "prof rc=$?"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C -d gpurun_out/pmc_c5b_$C -o run --output-format csv -- python3 -u bench.py --workload c5 --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_c5b_$C.log 2>&1 || { echo "pmc $C rc=$?"; exit 1; }
done
echo done
