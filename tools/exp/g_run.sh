set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest rc=$?; grep -E "Error|error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 -u tools/exp/graph_bench.py > gpurun_out/graph.log 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/graph.log; exit 1; }
grep "layers" gpurun_out/graph.log
