set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest rc=$?; grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
