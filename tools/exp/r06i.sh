#!/bin/bash
# round 6 session i: K6 axis-0 second-half load issue point (VSIQ_EXP_PCR_ISSUE 2 / 3 / 5, a temporary switch of
# k_lsq.hip removed after this session: ISSUE 3 is hard-coded),
# C2 bench learnable legs, twice each, then the remaining profile-round workloads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for rep in 1 2; do
  for P in 5 3 2; do
    VSIQ_EXP_PCR_ISSUE=$P timeout -k 10 300 python -u bench.py --workload c2 --extras none --no-cpu-baseline --no-api \
        > gpurun_out/r06i_c2_issue${P}_$rep.log 2>&1 || { echo "issue $P failed"; exit 1; }
    echo "issue $P rep $rep: $(grep 'bench summary' gpurun_out/r06i_c2_issue${P}_$rep.log | grep -o 'pc_learn[^]]*')"
  done
done
TAG=r06h WORKLOADS="${WORKLOADS:-c4 c1}" bash tools/profile_round.sh || exit $?
exit 0
