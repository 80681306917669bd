#!/bin/bash
# round 6 session x: C3's K4 (G = 8, multi-round) with its qparams as scalar loads after the
# first loads (VSIQ_EXP_K4_LATE=1, a temporary switch: 98 VGPRs, 4 waves / SIMD) against the
# product order (qparams first, 96 VGPRs, 5 waves), C3 bench line three times each way.
# (Record of a session: the switch was removed after it.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for rep in 1 2 3; do
  for L in 0 1; do
    VSIQ_EXP_K4_LATE=$L timeout -k 10 300 python -u bench.py --workload c3 --extras none --no-cpu-baseline --no-api \
        > gpurun_out/r06x_c3_late${L}_$rep.log 2>&1 || { echo "bench $L failed"; exit 1; }
    echo "late $L rep $rep: $(grep 'bench summary' gpurun_out/r06x_c3_late${L}_$rep.log | grep -o '\[fq_fwd[^]]*\]')"
  done
done
exit 0
