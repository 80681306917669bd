#!/bin/bash
# round 6 session a: RCCL capture probe (event recycling), K11 + chain tests, gate-table
# bench, timed-region rocprof of C2 with a frozen table.  Every GPU step has its own limit;
# a failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/r06a_steps.log
  return $rc
}
run r06a_probe 280 python -u tools/exp/rccl_capture_probe.py recycle recycle_twin recycle:nocache recycle_twin:nocache
run r06a_tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mean.py \
    tests/test_gpu_parity.py tests/test_gpu_fused_golden.py tests/test_gpu_gate.py || exit $?
run r06a_bench_c2 300 python -u bench.py --workload c2 --extras none --no-cpu-baseline --no-api \
    --save-gate-table gpurun_out/r06a_gates.txt || exit $?
run r06a_prof_c2 300 rocprofv3 --kernel-trace -d gpurun_out/r06a_prof_c2 -o run --output-format csv \
    -- python3 -u bench.py --workload c2 --extras none --no-cpu-baseline --no-api \
    --gate-table gpurun_out/r06a_gates.txt --markers || exit $?
python3 tools/timed_region_stats.py gpurun_out/r06a_prof_c2 gpurun_out/r06a_c2_timed_region.csv
find gpurun_out/r06a_prof_c2 -type f -name '*kernel_trace.csv' -size +20M -delete
exit 0
