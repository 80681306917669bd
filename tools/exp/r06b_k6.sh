#!/bin/bash
# round 6 session b: K6 / per-channel learnable forward kernel times (rocprofv3 kernel
# trace of tools/exp/pcm_bench.py, reduced by grid) and HBM bytes (separate FETCH_SIZE /
# WRITE_SIZE passes) at the verdict's shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r06b}
K="k_pcr_lsq k_pcc_lsq k_pcp_lsq k_pcm_lsq k_pc_fq k_pcp_fq k_lsq_bwd k_pcm_lsq_fold"
for S in ${SHAPES:-1024x1024x3x3 256x256x10x10 256x128x20x20}; do
  SHAPE=$S ROUNDS=3 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_tr_$S -o run --output-format csv \
      -- python3 -u tools/exp/pcm_bench.py > gpurun_out/${TAG}_tr_$S.log 2>&1 || { echo "trace $S failed"; exit 1; }
  echo "== $S trace"; cat gpurun_out/${TAG}_tr_$S.log | grep axis
  python3 tools/exp/trace_by_grid.py gpurun_out/${TAG}_tr_$S $K || exit 1
  rm -rf gpurun_out/${TAG}_tr_$S
  if [ "${PMC:-1}" = 1 ]; then
    for C in FETCH_SIZE WRITE_SIZE; do
      SHAPE=$S ROUNDS=1 timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/${TAG}_pmc_${S}_$C -o run --output-format csv \
          -- python3 -u tools/exp/pcm_bench.py > gpurun_out/${TAG}_pmc_${S}_$C.log 2>&1 || { echo "pmc $S $C failed"; exit 1; }
      python3 tools/exp/pmc_by_grid.py gpurun_out/${TAG}_pmc_${S}_$C $C $K || exit 1
      rm -rf gpurun_out/${TAG}_pmc_${S}_$C
    done
  fi
done
exit 0
