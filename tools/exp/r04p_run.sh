set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_torch_ext.py tests/test_gpu_model_launch.py > gpurun_out/t_r04p.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_r04p.log; exit 1; }
tail -2 gpurun_out/t_r04p.log
