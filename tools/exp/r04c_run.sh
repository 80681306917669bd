# round 4: K2o bench + kernel trace, the C5 leg, then the r04b items
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u tools/exp/k2o_bench.py 20 > gpurun_out/k2o_bench.log 2>&1 || { echo "k2o bench rc=$?"; tail gpurun_out/k2o_bench.log; exit 1; }
cat gpurun_out/k2o_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k2o -o run --output-format csv -- python3 -u tools/exp/k2o_bench.py 5 > gpurun_out/p_k2o.log 2>&1 || { echo "prof rc=$?"; exit 1; }
timeout -k 10 300 python3 -u bench.py --workload c5 --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/b_c5.log 2>&1 || { echo "bench c5 rc=$?"; tail gpurun_out/b_c5.log; exit 1; }
tail -1 gpurun_out/b_c5.log
bash tools/exp/r04b_run.sh
