# Public-API step host cost after the bound op's checks / allocation moved to C++; the
# tests that cover observe_quantize.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_torch_ext.py tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_calib.py tests/test_gpu_fuzz.py > gpurun_out/t_r04k.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_r04k.log; exit 1; }
tail -2 gpurun_out/t_r04k.log
timeout -k 10 300 python3 -u tools/exp/api_host.py > gpurun_out/api_host_k.log 2>&1 || { echo "rc=$?"; tail gpurun_out/api_host_k.log; exit 1; }
cat gpurun_out/api_host_k.log
timeout -k 10 300 python3 -u tools/exp/api_timings.py > gpurun_out/api_timings_k.log 2>&1 || { echo "rc=$?"; tail gpurun_out/api_timings_k.log; exit 1; }
cat gpurun_out/api_timings_k.log
