#!/bin/bash
# round 6 session k: qparams as scalar loads issued after the streaming loads (K1, K4 at
# G <= 2, K7, the learnable per-channel forward, K6) and the tuner's per-launch event
# pairs: smoke, the full GPU suite and the default line (tools/gpu_round.sh), the C2-shape
# gate sweep (tools/exp/c2_floor.py), then the K6 column form (axis 1, 256x256x10x10)
# with grad_x in registers against LDS staging at 7 waves (VSIQ_EXP_PCC_STAGE, a
# temporary switch) under a kernel trace.
# (Record of a session: its VSIQ_EXP_PCC_STAGE variant was removed after it; the script
# no longer selects it.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_round.sh || exit $?
tail -1 gpurun_out/pytest_gpu.log
grep "bench summary" gpurun_out/bench.log | cut -c1-700
timeout -k 10 400 python -u tools/exp/c2_floor.py 200 > gpurun_out/r06k_c2_floor.txt 2>&1 || { echo "floor failed"; tail -5 gpurun_out/r06k_c2_floor.txt; exit 1; }
tail -7 gpurun_out/r06k_c2_floor.txt
K="k_pcc_lsq k_pcp_fq k_pcm_lsq_fold"
for rep in 1 2; do
  for ST in 0 1; do
    VSIQ_EXP_PCC_STAGE=$ST SHAPE=256x256x10x10 ROUNDS=3 timeout -k 10 300 rocprofv3 --kernel-trace \
        -d gpurun_out/r06k_tr_$ST -o run --output-format csv -- python3 -u tools/exp/pcm_bench.py \
        > gpurun_out/r06k_tr_${ST}_$rep.log 2>&1 || { echo "trace $ST failed"; exit 1; }
    echo "== stage $ST rep $rep"; grep axis gpurun_out/r06k_tr_${ST}_$rep.log
    python3 tools/exp/trace_by_grid.py gpurun_out/r06k_tr_$ST $K || exit 1
    rm -rf gpurun_out/r06k_tr_$ST
  done
done
exit 0
