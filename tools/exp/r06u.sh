#!/bin/bash
# round 6 session u (and v): K11 -- u: the std pass folded by its last workgroup (one launch fewer per
# call; slower: arrivals on one counter serialize, reverted), v: the one-lane final without
# the empty multi-row cascade: tests/test_gpu_mean.py, the mean reference's cost per C5 calibration batch twice
# (tools/exp/k11_calib_cost.py), then the same under a kernel trace, by kernel and grid.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mean.py \
    tests/test_gpu_parity.py > gpurun_out/r06u_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06u_tests.log; exit 1; }
tail -1 gpurun_out/r06u_tests.log
for rep in 1 2; do
  timeout -k 10 300 python -u tools/exp/k11_calib_cost.py 20 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06u_tr -o run --output-format csv \
    -- python3 -u tools/exp/k11_calib_cost.py 20 > gpurun_out/r06u_cost_traced.log 2>&1 || { echo "trace failed"; exit 1; }
python3 tools/exp/trace_by_grid.py gpurun_out/r06u_tr k_mean k_std k_observe_part_out > gpurun_out/r06u_k11_by_grid.txt || exit 1
rm -rf gpurun_out/r06u_tr
exit 0
