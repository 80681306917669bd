set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
SHAPES="4096x256x3x3 2048x1024x3x3 2048x512x3x3 3072x512x3x3 1024x1024x3x3 512x1024x3x3 1024x2048x1x1 4096x512x1x1" FS="0 -1" ROUNDS=5 timeout -k 10 400 python3 -u tools/exp/gate_bench.py > gpurun_out/gate_shapes.log 2>&1 || { echo "rc=$?"; tail gpurun_out/gate_shapes.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gate_shapes.log
