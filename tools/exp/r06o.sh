#!/bin/bash
# round 6 session o: K6 on axis-1 short rows -- channel tiles (VSIQ_TUNE_PC_PACKED 3, new;
# 8 or 4 images per workgroup, VSIQ_EXP_PCT_NB, a temporary switch) against the channel
# columns (1, default) at 10x10 and 20x20, kernel-trace medians by grid, twice; the K6
# module tests first (they cover the tile form).
# (Record of a session: the tile form and VSIQ_TUNE_PC_PACKED 3 were removed after it; the
# script fails on the knob now.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lsq_module.py \
    > gpurun_out/r06o_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06o_tests.log; exit 1; }
tail -1 gpurun_out/r06o_tests.log
K="k_pcc_lsq k_pct_lsq k_pcm_lsq_fold"
for rep in 1 2; do
  for S in 256x256x10x10 256x128x20x20; do
    for V in "1 8" "3 8" "3 4"; do
      set -- $V
      VSIQ_EXP_PCT_NB=$2 TUNE="10=$1" SHAPE=$S ROUNDS=3 timeout -k 10 300 rocprofv3 --kernel-trace \
          -d gpurun_out/r06o_tr -o run --output-format csv -- python3 -u tools/exp/pcm_bench.py \
          > gpurun_out/r06o_tr_${S}_$1_$2_$rep.log 2>&1 || { echo "trace $S $V failed"; exit 1; }
      echo "== $S packed $1 nb $2 rep $rep"
      python3 tools/exp/trace_by_grid.py gpurun_out/r06o_tr $K || exit 1
      rm -rf gpurun_out/r06o_tr
    done
  done
done
exit 0
