set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for T in "" "11=0" "10=0" "" "11=0" "10=0"; do
TUNE="$T" timeout -k 10 300 python3 -u tools/exp/pcm_bench.py > gpurun_out/pcm.log 2>&1 || { echo "rc=$?"; tail gpurun_out/pcm.log; exit 1; }
echo "TUNE=$T"; grep "axis 0" gpurun_out/pcm.log
done
