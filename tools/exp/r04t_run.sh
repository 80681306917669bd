# r04t: the group fast-path test with u's range implied by x's (VSIQ_EXP_K4_GRPCHK 2, product) vs
# u tested in the tree (1); K4d at C4 sizes and the C3 leg, twice; then the K4-family parity tests.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python3 tools/exp/build_variant.py /tmp/vsiq_gc1.so -DVSIQ_EXP_K4_GRPCHK=1 > /tmp/bv.log 2>&1 || { echo "build failed"; tail /tmp/bv.log; exit 1; }
for rep in 1 2; do
  echo "== product (group test with u implied by x) $rep"
  timeout -k 10 300 python3 -u tools/exp/c4_floor.py 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 300 python3 -u bench.py --workload c3 --steps 40 --warmup 5 --no-cpu-baseline --no-api 2>&1 | grep "bench summary" || exit 1
  echo "== -DVSIQ_EXP_K4_GRPCHK=1 $rep"
  VSIQ_LIBRARY=/tmp/vsiq_gc1.so timeout -k 10 300 python3 -u tools/exp/c4_floor.py 2>&1 | grep -v amdgpu.ids || exit 1
  VSIQ_LIBRARY=/tmp/vsiq_gc1.so timeout -k 10 300 python3 -u bench.py --workload c3 --steps 40 --warmup 5 --no-cpu-baseline --no-api 2>&1 | grep "bench summary" || exit 1
done
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deferred_grads.py tests/test_gpu_model_launch.py tests/test_gpu_multi.py tests/test_gpu_parity.py tests/test_gpu_lsq_module.py tests/test_gpu_c4.py tests/test_gpu_silu.py > gpurun_out/t_r04t.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_r04t.log; exit 1; }
tail -2 gpurun_out/t_r04t.log
echo done
