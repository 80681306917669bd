# round 4: the whole GPU suite, then the default bench line
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_capture.py tests/test_gpu_dist_calib.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_cap.log 2>&1 || { echo "capture tests rc=$?"; tail -40 gpurun_out/t_cap.log; exit 1; }
tail -2 gpurun_out/t_cap.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_full.log 2>&1 || { echo "tests rc=$?"; tail -60 gpurun_out/t_full.log; exit 1; }
tail -3 gpurun_out/t_full.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_default2.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_default2.log; exit 1; }
grep "bench summary" gpurun_out/bench_default2.log
echo done
