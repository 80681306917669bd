# Per-dispatch K4d durations in the C4 leg at 2 (default) / 4 / 8 / 16 groups per lane
# (VSIQ_TUNE_LSQ_GROUPS), from rocprofv3 kernel traces reduced on the box
# (tools/exp/trace_by_grid.py).  Run inside gpurun: bash tools/exp/r05p_k4d_groups.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for G in ${GROUPS_LIST:-0 4 8 16}; do
  T=""; [ "$G" -ne 0 ] && T="--tune ${TUNE_KEY:-9}=$G"
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr_g$G -o run --output-format csv -- python3 -u bench.py --workload ${WORKLOAD:-c4} --steps 30 --warmup 4 --no-cpu-baseline --no-api $T > gpurun_out/tr_g$G.log 2>&1 || { echo "G=$G failed"; tail -5 gpurun_out/tr_g$G.log; exit 1; }
  echo "== G=$G $(grep 'bench summary' gpurun_out/tr_g$G.log | cut -c1-110)"
  python3 tools/exp/trace_by_grid.py gpurun_out/tr_g$G ${KERNELS:-k_lsq_bwd} || exit 1
  rm -rf gpurun_out/tr_g$G
done
