#!/bin/bash
# Parametrised GPU-box runner for experiments (replaces round 4's per-experiment
# r04*_run.sh scripts).  Usage, inside a gpurun call:
#   bash tools/exp/run.sh TAG SECONDS:NAME:COMMAND [SECONDS:NAME:COMMAND ...]
# Every step runs under its own `timeout -k 10 SECONDS`, its output goes to
# gpurun_out/TAG_NAME.log and its last lines are echoed; the first failing step (non-zero
# exit, abort, timeout) ends the run, so nothing more touches the GPU after a fault.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=$1
shift
for spec in "$@"; do
  secs=${spec%%:*}
  rest=${spec#*:}
  name=${rest%%:*}
  cmd=${rest#*:}
  log="gpurun_out/${tag}_${name}.log"
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$log" 2>&1
  rc=$?
  grep -v "amdgpu.ids" "$log" | tail -n "${TAIL_LINES:-6}"
  if [ $rc -ne 0 ]; then
    echo "== $name failed rc=$rc"
    exit $rc
  fi
done
echo "== done"
