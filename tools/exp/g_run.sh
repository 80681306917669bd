set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/exp/codes_bench.py > gpurun_out/codes.log 2>&1 || { echo "rc=$?"; tail gpurun_out/codes.log; exit 1; }
grep -v amdgpu.ids gpurun_out/codes.log
