#!/bin/bash
# Per workload: a bench line (saving its store-gate table), a rocprofv3 kernel-trace +
# stats of the same workload with that table frozen and trace markers around the timed
# regions (-> <TAG>_<W>_timed_region.csv: the timed launches alone), then separate PMC
# passes for FETCH_SIZE and WRITE_SIZE (never combined with other trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r01}
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log
  return $rc
}
export TMPDIR=/tmp
for W in ${WORKLOADS:-c1 c2 c3 c4 c5}; do
  case $W in
    c4) S=20; WU=4; SP=8; WP=2 ;;
    c5) S=16; WU=2; SP=16; WP=2 ;;
    *)  S=200; WU=20; SP=40; WP=5 ;;
  esac
  run bench_$W 600 python3 -u bench.py --workload $W --steps $S --warmup $WU ${BENCH_EXTRA:-} \
      --save-gate-table gpurun_out/gates_${TAG}_$W.txt || exit $?
  # the trace with the gate table the bench run above saved (frozen: no tuner launches) and
  # trace markers around the timed regions (tools/timed_region_stats.py cuts them out)
  run prof_$W 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$W -o run --output-format csv \
      -- python3 -u bench.py --workload $W --steps $S --warmup $WU --no-cpu-baseline \
      --gate-table gpurun_out/gates_${TAG}_$W.txt --markers || exit $?
  python3 tools/timed_region_stats.py gpurun_out/prof_${TAG}_$W gpurun_out/${TAG}_${W}_timed_region.csv || exit $?
  for C in FETCH_SIZE WRITE_SIZE; do
    run pmc_${W}_$C 600 rocprofv3 --pmc $C -d gpurun_out/pmc_${TAG}_${W}_$C -o run --output-format csv \
        -- python3 -u bench.py --workload $W --steps $SP --warmup $WP --no-cpu-baseline || exit $?
  done
  # reduce on the box (gpurun copies back at most 64 MiB): the PMC passes -> HBM bytes per
  # launch, then keep only the kernel-stats summaries of the traces
  python3 tools/pmc_to_traffic.py gpurun_out/pmc_traffic_${TAG}.json \
      $W=gpurun_out/pmc_${TAG}_${W}_FETCH_SIZE,gpurun_out/pmc_${TAG}_${W}_WRITE_SIZE > /dev/null || exit $?
  find gpurun_out/prof_${TAG}_$W gpurun_out/pmc_${TAG}_${W}_* -type f ! -name '*kernel_stats.csv' -delete
done
exit 0
