#!/bin/bash
# round 6 session m: the final tree -- smoke, full GPU suite and the default line
# (tools/gpu_round.sh), then the profile round for every workload (TAG=r06m).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_round.sh || exit $?
tail -1 gpurun_out/pytest_gpu.log
grep "bench summary" gpurun_out/bench.log | cut -c1-900
TAG=r06m WORKLOADS="${WORKLOADS:-c2 c3 c4 c5 c1}" bash tools/profile_round.sh || exit $?
for w in c2 c3 c4 c5 c1; do grep "bench summary" gpurun_out/bench_$w.log | cut -c1-300; done
exit 0
