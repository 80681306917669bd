set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_lsq_module.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_pcm.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_pcm.log; exit 1; }
tail -1 gpurun_out/t_pcm.log
timeout -k 10 300 python3 -u tools/exp/pcm_bench.py > gpurun_out/pcm.log 2>&1 || { echo "pcm rc=$?"; tail gpurun_out/pcm.log; exit 1; }
grep -v amdgpu.ids gpurun_out/pcm.log
