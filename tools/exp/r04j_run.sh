set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
PROFILE=1 timeout -k 10 300 python3 -u tools/exp/api_host.py > gpurun_out/api_host.log 2>&1 || { echo "rc=$?"; tail gpurun_out/api_host.log; exit 1; }
cat gpurun_out/api_host.log
