set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_default3.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_default3.log; exit 1; }
grep "bench summary" gpurun_out/bench_default3.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default3 -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline > gpurun_out/prof_default3.log 2>&1 || { echo "prof rc=$?"; exit 1; }
grep "bench summary" gpurun_out/prof_default3.log
echo done
