set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest rc=$?; grep -E "Error|error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for T in "" "11=0" "" "11=0"; do
TUNE="$T" timeout -k 10 300 python3 -u tools/exp/pcm_bench.py > gpurun_out/pcm.log 2>&1 || { echo "rc=$?"; tail gpurun_out/pcm.log; exit 1; }
echo "TUNE=$T"; grep "axis 0" gpurun_out/pcm.log
done
