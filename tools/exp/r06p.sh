#!/bin/bash
# round 6 session p: the final tree after the K6 column change -- smoke, full GPU suite,
# default line (tools/gpu_round.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_round.sh || exit $?
tail -1 gpurun_out/pytest_gpu.log
grep "bench summary" gpurun_out/bench.log | cut -c1-900
exit 0
