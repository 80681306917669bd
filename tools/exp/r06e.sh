#!/bin/bash
# round 6 session e: K6 axis-0 output staging (VSIQ_EXP_PCR_STAGE 0 registers / 1 LDS /
# 2 no gate) in the C2 bench's learnable legs, their kernel trace, and C1's PMC bytes per
# kernel (with the trace marker as the empty-kernel baseline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r06e}
for S in 0 1 2; do
  VSIQ_EXP_PCR_STAGE=$S timeout -k 10 300 python -u bench.py --workload c2 --extras none --no-cpu-baseline --no-api \
      > gpurun_out/${T}_c2_stage$S.log 2>&1 || { echo "stage $S failed"; exit 1; }
  echo "stage $S: $(grep 'bench summary' gpurun_out/${T}_c2_stage$S.log)"
done
VSIQ_EXP_PCR_STAGE=${TRACE_STAGE:-1} timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_tr -o run --output-format csv \
    -- python3 -u bench.py --workload c2 --extras none --no-cpu-baseline --no-api > gpurun_out/${T}_tr.log 2>&1 || exit 1
python3 tools/exp/trace_by_grid.py gpurun_out/${T}_tr k_pcr_lsq k_pc_fq k_pc_observe k_ste || exit 1
rm -rf gpurun_out/${T}_tr
for W7 in 0 1; do
  VSIQ_EXP_PCC_W7=$W7 SHAPE=256x256x10x10 ROUNDS=3 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_pcc$W7 -o run \
      --output-format csv -- python3 -u tools/exp/pcm_bench.py > gpurun_out/${T}_pcc$W7.log 2>&1 || exit 1
  echo "== 10x10 W7=$W7"; grep axis gpurun_out/${T}_pcc$W7.log
  python3 tools/exp/trace_by_grid.py gpurun_out/${T}_pcc$W7 k_pcc_lsq k_pcp_fq || exit 1
  rm -rf gpurun_out/${T}_pcc$W7
done
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/${T}_pmc_c1_$C -o run --output-format csv \
      -- python3 -u bench.py --workload c1 --extras none --no-cpu-baseline --no-api --steps 200 --warmup 20 --markers \
      > gpurun_out/${T}_pmc_c1_$C.log 2>&1 || { echo "pmc c1 $C failed"; exit 1; }
  python3 tools/exp/pmc_by_grid.py gpurun_out/${T}_pmc_c1_$C $C || exit 1
  rm -rf gpurun_out/${T}_pmc_c1_$C
done
timeout -k 10 300 python3 -u tools/exp/k11_bench.py > gpurun_out/${T}_k11.log 2>&1 || exit 1
cat gpurun_out/${T}_k11.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_k11tr -o run --output-format csv \
    -- python3 -u tools/exp/k11_bench.py > /dev/null 2>&1 || exit 1
python3 tools/exp/trace_by_grid.py gpurun_out/${T}_k11tr k_mean || exit 1
rm -rf gpurun_out/${T}_k11tr
exit 0
