#!/bin/bash
# One GPU-box session: smoke -> pytest -m gpu -> bench.  Every GPU step has its own
# time limit; a crash / abort / timeout ends the script (no further GPU work).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log
  return $rc
}
run smoke 600 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
run pytest_gpu "${PYTEST_TIMEOUT:-900}" python -u -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-}
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run bench 600 python -u bench.py ${BENCH_ARGS:-} || exit $?
exit 0
