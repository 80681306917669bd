#!/bin/bash
# round 6 session f: K6 axis-0 staging A/B (0 registers / 1 LDS / 3 LDS + split loads), K11
# v2 timing, the gate / mean / LSQ-module GPU tests, and a tuned vs frozen-table C2 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r06f}
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_gate.py \
    tests/test_gpu_mean.py tests/test_gpu_lsq_module.py tests/test_gpu_parity.py > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for S in 0 1 3; do
  VSIQ_EXP_PCR_STAGE=$S timeout -k 10 300 python -u bench.py --workload c2 --extras none --no-cpu-baseline --no-api \
      > gpurun_out/${T}_c2_stage$S.log 2>&1 || { echo "stage $S failed"; exit 1; }
  echo "stage $S: $(grep 'bench summary' gpurun_out/${T}_c2_stage$S.log)"
done
timeout -k 10 300 python -u bench.py --workload c2 --extras none --no-cpu-baseline --no-api \
    --save-gate-table gpurun_out/${T}_gates.txt > gpurun_out/${T}_c2_tuned.log 2>&1 || exit 1
echo "tuned : $(grep 'bench summary' gpurun_out/${T}_c2_tuned.log)"
timeout -k 10 300 python -u bench.py --workload c2 --extras none --no-cpu-baseline --no-api \
    --gate-table gpurun_out/${T}_gates.txt > gpurun_out/${T}_c2_frozen.log 2>&1 || exit 1
echo "frozen: $(grep 'bench summary' gpurun_out/${T}_c2_frozen.log)"
timeout -k 10 300 python3 -u tools/exp/k11_bench.py > gpurun_out/${T}_k11.log 2>&1 || exit 1
cat gpurun_out/${T}_k11.log
exit 0
