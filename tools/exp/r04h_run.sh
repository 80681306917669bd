# K4d element math with selects instead of exec branches (valid lanes, in-range m) vs
# round 3 branches, at C4 sizes and scale; then the K4d parity tests.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
echo "== product (branch-free selects)"
timeout -k 10 300 python3 -u tools/exp/c4_floor.py > gpurun_out/c4_sel.log 2>&1 || { echo "c4 rc=$?"; tail -5 gpurun_out/c4_sel.log; exit 1; }
cat gpurun_out/c4_sel.log
timeout -k 10 400 python3 tools/exp/build_variant.py /tmp/vsiq_sel0.so -DVSIQ_EXP_K4_SEL=0 > /tmp/bv.log 2>&1 || { echo "build failed"; tail /tmp/bv.log; exit 1; }
echo "== -DVSIQ_EXP_K4_SEL=0"
VSIQ_LIBRARY=/tmp/vsiq_sel0.so timeout -k 10 300 python3 -u tools/exp/c4_floor.py || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deferred_grads.py tests/test_gpu_model_launch.py tests/test_gpu_multi.py tests/test_gpu_parity.py tests/test_gpu_lsq_module.py > gpurun_out/t_k4d.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_k4d.log; exit 1; }
tail -3 gpurun_out/t_k4d.log
echo done
