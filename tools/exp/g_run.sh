set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2 3; do
timeout -k 10 300 python3 -u tools/exp/host_overhead.py > gpurun_out/host_ovh.log 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/host_ovh.log; exit 1; }
grep -E "learnable fwd\+bwd|trivial" gpurun_out/host_ovh.log
done
