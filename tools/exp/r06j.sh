#!/bin/bash
# round 6 session j: K6 with ISSUE 3 hard-coded (its GPU tests + the C2 bench legs), then
# the C2-shape gate sweep of K3 / STE / learnable forward (with and without mask) / K6 /
# a plain gated copy (tools/exp/c2_floor.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lsq_module.py \
    > gpurun_out/r06j_lsq_module.log 2>&1 || { echo "lsq module tests failed"; tail -5 gpurun_out/r06j_lsq_module.log; exit 1; }
tail -1 gpurun_out/r06j_lsq_module.log
timeout -k 10 300 python -u bench.py --workload c2 --extras none --no-cpu-baseline --no-api \
    > gpurun_out/r06j_c2.log 2>&1 || { echo "bench failed"; exit 1; }
grep 'bench summary' gpurun_out/r06j_c2.log | cut -c1-260
timeout -k 10 400 python -u tools/exp/c2_floor.py 200 > gpurun_out/r06j_c2_floor.txt 2>&1 || { echo "floor failed"; tail -5 gpurun_out/r06j_c2_floor.txt; exit 1; }
cat gpurun_out/r06j_c2_floor.txt
exit 0
