#!/bin/bash
# round 6 session w: the final tree -- smoke, full GPU suite, default line
# (tools/gpu_round.sh), then the mean reference's cost per C5 calibration batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_round.sh || exit $?
tail -1 gpurun_out/pytest_gpu.log
grep "bench summary" gpurun_out/bench.log | cut -c1-900
timeout -k 10 300 python -u tools/exp/k11_calib_cost.py 20 2>&1 | grep -v amdgpu.ids || exit 1
exit 0
