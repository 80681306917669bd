#!/bin/bash
# round 6 session aa: K6 axis 0's second-half issue point again, now that the row's
# qparams are scalar loads issued after the first half (VSIQ_EXP_PCR_ISSUE 2 / 3 / 4, a
# temporary switch; 3 is the product), C2 bench learnable legs three times each.
# (Record of a session: the switch was removed after it.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for rep in 1 2 3; do
  for P in 3 2 4; do
    VSIQ_EXP_PCR_ISSUE=$P timeout -k 10 300 python -u bench.py --workload c2 --extras none --no-cpu-baseline --no-api \
        > gpurun_out/r06aa_c2_issue${P}_$rep.log 2>&1 || { echo "issue $P failed"; exit 1; }
    echo "issue $P rep $rep: $(grep 'bench summary' gpurun_out/r06aa_c2_issue${P}_$rep.log | grep -o 'pc_learn[^]]*')"
  done
done
exit 0
