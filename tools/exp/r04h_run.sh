set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/exp/c4_floor.py > gpurun_out/c4_floor_h.log 2>&1 || { echo "c4 rc=$?"; tail -5 gpurun_out/c4_floor_h.log; exit 1; }
cat gpurun_out/c4_floor_h.log
echo done
