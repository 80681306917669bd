#!/bin/bash
# round 6 session c: full GPU suite, C2 line saving the gate table, C2 rocprof kernel trace
# of the timed regions with that table frozen (bench.py --markers, tools/timed_region_stats.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r06c}
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/${T}_steps.log
  return $rc
}
run ${T}_tests 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run ${T}_bench_c2 300 python -u bench.py --workload c2 --extras none --no-cpu-baseline --no-api \
    --save-gate-table gpurun_out/${T}_gates.txt || exit $?
run ${T}_prof_c2 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof_c2 -o run --output-format csv \
    -- python3 -u bench.py --workload c2 --extras none --no-cpu-baseline --no-api \
    --gate-table gpurun_out/${T}_gates.txt --markers || exit $?
python3 tools/timed_region_stats.py gpurun_out/${T}_prof_c2 gpurun_out/${T}_c2_timed_region.csv
find gpurun_out/${T}_prof_c2 -type f -name '*kernel_trace.csv' -size +20M -delete
exit 0
