set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/exp/pcm_bench.py > gpurun_out/pcm.log 2>&1 || { echo "rc=$?"; tail gpurun_out/pcm.log; exit 1; }
grep -v amdgpu gpurun_out/pcm.log
