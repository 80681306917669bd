#!/bin/bash
# round 6 session ab: the shipped build of the last commit -- smoke, full GPU suite and the
# default line (tools/gpu_round.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_round.sh || exit $?
tail -1 gpurun_out/pytest_gpu.log
grep "bench summary" gpurun_out/bench.log | cut -c1-900
exit 0
