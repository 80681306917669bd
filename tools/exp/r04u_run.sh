# Round-4 tree check: full GPU suite, smoke, default bench, and the default bench under
# rocprofv3 --kernel-trace --stats.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_r04u.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/t_r04u.log; exit 1; }
tail -2 gpurun_out/t_r04u.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke_r04u.log 2>&1 || { echo "smoke rc=$?"; tail gpurun_out/smoke_r04u.log; exit 1; }
tail -1 gpurun_out/smoke_r04u.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_r04u.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_r04u.log; exit 1; }
grep "bench summary" gpurun_out/bench_r04u.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04u -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline > gpurun_out/prof_r04u.log 2>&1 || { echo "prof rc=$?"; exit 1; }
grep "bench summary" gpurun_out/prof_r04u.log
echo done
