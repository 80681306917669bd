set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 -u bench.py --workload c1 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/b_c1.log 2>&1 || { echo "c1 rc=$?"; tail gpurun_out/b_c1.log; exit 1; }
grep '^{' gpurun_out/b_c1.log | cut -c1-150
grep -o '"kernels".*' gpurun_out/b_c1.log
timeout -k 10 200 python3 -u tools/exp/fold_bench.py > gpurun_out/fold_new.log 2>&1 || { echo "bench rc=$?"; exit 1; }
grep -v amdgpu.ids gpurun_out/fold_new.log
