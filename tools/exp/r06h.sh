#!/bin/bash
# round 6 session h: K11 tests + kernel trace, then the per-workload profile round (bench
# line saving its gate table, frozen-table kernel trace with timed-region markers, PMC).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_mean.py \
    > gpurun_out/r06h_mean_tests.log 2>&1 || { tail -20 gpurun_out/r06h_mean_tests.log; exit 1; }
tail -1 gpurun_out/r06h_mean_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06h_k11tr -o run --output-format csv \
    -- python3 -u tools/exp/k11_bench.py > gpurun_out/r06h_k11.log 2>&1 || exit 1
cat gpurun_out/r06h_k11.log | grep "^n="
python3 tools/exp/trace_by_grid.py gpurun_out/r06h_k11tr k_mean > gpurun_out/r06h_k11_by_grid.txt || exit 1
rm -rf gpurun_out/r06h_k11tr
TAG=r06h WORKLOADS="${WORKLOADS:-c2 c3 c5}" bash tools/profile_round.sh || exit $?
exit 0
