#!/bin/bash
# round 6 session n: the K6 column form with 4 against 8 groups per lane (VSIQ_EXP_PCC_CG,
# a temporary switch: 8 = 81 images of 10x10 per workgroup, 4 waves / SIMD, one round at
# 256x256x10x10) at the three YOLOv8n axis-1 shapes, kernel-trace medians by grid, twice;
# then the K6 module tests under CG 8.
# (Record of a session: VSIQ_EXP_PCC_CG was removed after it -- 8 groups per lane is now
# the only form.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
K="k_pcc_lsq k_pcm_lsq_fold"
for rep in 1 2; do
  for S in 256x256x10x10 256x128x20x20 256x64x40x40; do
    for CG in 4 8; do
      VSIQ_EXP_PCC_CG=$CG SHAPE=$S ROUNDS=3 timeout -k 10 300 rocprofv3 --kernel-trace \
          -d gpurun_out/r06n_tr -o run --output-format csv -- python3 -u tools/exp/pcm_bench.py \
          > gpurun_out/r06n_tr_${S}_${CG}_$rep.log 2>&1 || { echo "trace $S $CG failed"; exit 1; }
      echo "== $S groups $CG rep $rep"
      python3 tools/exp/trace_by_grid.py gpurun_out/r06n_tr $K || exit 1
      rm -rf gpurun_out/r06n_tr
    done
  done
done
VSIQ_EXP_PCC_CG=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_lsq_module.py > gpurun_out/r06n_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06n_tests.log; exit 1; }
tail -1 gpurun_out/r06n_tests.log
exit 0
