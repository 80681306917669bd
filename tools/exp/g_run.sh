set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest rc=$?; grep -E "Error|assert|FAILED|mismatch" gpurun_out/pytest_gpu.log | head -30; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
