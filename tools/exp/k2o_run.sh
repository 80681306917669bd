set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_silu.py -x -q --timeout 120 --timeout-method thread -k "parts_out" > gpurun_out/t_k2o.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/t_k2o.log; exit 1; }
tail -2 gpurun_out/t_k2o.log
timeout -k 10 300 python -u tools/exp/k2o_bench.py 20 > gpurun_out/k2o_bench.log 2>&1 || { echo "bench rc=$?"; tail gpurun_out/k2o_bench.log; exit 1; }
cat gpurun_out/k2o_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k2o -o run --output-format csv -- python3 -u tools/exp/k2o_bench.py 5 > gpurun_out/p_k2o.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo done
