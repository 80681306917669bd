# r04s: as r04r after the lean element masks g for tail lanes (one select instead of two f64
# selects) and reuses g*s for the STE quotient; K4d at C4 sizes and the C3 leg, product vs
# -DVSIQ_EXP_K4_LEAN=0, twice; then the K4-family parity tests.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python3 tools/exp/build_variant.py /tmp/vsiq_lean0.so -DVSIQ_EXP_K4_LEAN=0 > /tmp/bv.log 2>&1 || { echo "build failed"; tail /tmp/bv.log; exit 1; }
for rep in 1 2; do
  echo "== product (lean STEQ element) $rep"
  timeout -k 10 300 python3 -u tools/exp/c4_floor.py 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 300 python3 -u bench.py --workload c3 --steps 40 --warmup 5 --no-cpu-baseline --no-api 2>&1 | grep "bench summary" || exit 1
  echo "== -DVSIQ_EXP_K4_LEAN=0 $rep"
  VSIQ_LIBRARY=/tmp/vsiq_lean0.so timeout -k 10 300 python3 -u tools/exp/c4_floor.py 2>&1 | grep -v amdgpu.ids || exit 1
  VSIQ_LIBRARY=/tmp/vsiq_lean0.so timeout -k 10 300 python3 -u bench.py --workload c3 --steps 40 --warmup 5 --no-cpu-baseline --no-api 2>&1 | grep "bench summary" || exit 1
done
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deferred_grads.py tests/test_gpu_model_launch.py tests/test_gpu_multi.py tests/test_gpu_parity.py tests/test_gpu_lsq_module.py tests/test_gpu_c4.py tests/test_gpu_silu.py > gpurun_out/t_r04s.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_r04s.log; exit 1; }
tail -2 gpurun_out/t_r04s.log
echo done
