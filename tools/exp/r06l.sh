#!/bin/bash
# round 6 session l: the stats / calibration GPU tests after the fp32 stats records, then
# the K6 column form at 256x256x10x10 under three workgroup orders (VSIQ_TUNE_XCD_ORDER
# 0 hardware, 1 XCD-contiguous, 2 channel ranges per XCD with image blocks outermost),
# twice each, kernel trace medians by grid.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fused_golden.py tests/test_gpu_mean.py tests/test_gpu_calib.py tests/test_gpu_calib_reads.py \
    tests/test_gpu_c5_calib.py tests/test_gpu_lsq_module.py > gpurun_out/r06l_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/r06l_tests.log; exit 1; }
tail -1 gpurun_out/r06l_tests.log
K="k_pcc_lsq k_pcm_lsq_fold"
for rep in 1 2; do
  for XO in 1 2 0; do
    TUNE="13=$XO" SHAPE=256x256x10x10 ROUNDS=3 timeout -k 10 300 rocprofv3 --kernel-trace \
        -d gpurun_out/r06l_tr_$XO -o run --output-format csv -- python3 -u tools/exp/pcm_bench.py \
        > gpurun_out/r06l_tr_${XO}_$rep.log 2>&1 || { echo "trace $XO failed"; exit 1; }
    echo "== xcd order $XO rep $rep"
    python3 tools/exp/trace_by_grid.py gpurun_out/r06l_tr_$XO $K || exit 1
    rm -rf gpurun_out/r06l_tr_$XO
  done
done
exit 0
