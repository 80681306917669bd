#!/bin/bash
# round 6 session q: K6 axis 0 with g by LDS-DMA (VSIQ_EXP_PCR_GLDS=1, a temporary switch)
# against the split-load form: the K6 module tests under the LDS-DMA form, the C2 bench's
# learnable legs twice each way, then the C2 gate sweep's K6 column each way.
# (Record of a session: the LDS-DMA variant and VSIQ_EXP_PCR_GLDS were removed after it.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
VSIQ_EXP_PCR_GLDS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_lsq_module.py > gpurun_out/r06q_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06q_tests.log; exit 1; }
tail -1 gpurun_out/r06q_tests.log
for rep in 1 2; do
  for GL in 0 1; do
    VSIQ_EXP_PCR_GLDS=$GL timeout -k 10 300 python -u bench.py --workload c2 --extras none --no-cpu-baseline --no-api \
        > gpurun_out/r06q_c2_gl${GL}_$rep.log 2>&1 || { echo "bench $GL failed"; exit 1; }
    echo "glds $GL rep $rep: $(grep 'bench summary' gpurun_out/r06q_c2_gl${GL}_$rep.log | grep -o 'pc_learn[^]]*')"
  done
done
for GL in 0 1; do
  VSIQ_EXP_PCR_GLDS=$GL timeout -k 10 400 python -u tools/exp/c2_floor.py 200 > gpurun_out/r06q_floor_gl$GL.txt 2>&1 \
      || { echo "floor $GL failed"; tail -5 gpurun_out/r06q_floor_gl$GL.txt; exit 1; }
  echo "== floor glds $GL"; grep "best K6" gpurun_out/r06q_floor_gl$GL.txt
done
exit 0
