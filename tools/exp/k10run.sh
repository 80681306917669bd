#!/bin/bash
# C1 with K10 (one launch, grid barrier), its timing-only variants (build them first:
# python tools/exp/build_variant.py tools/exp/so/k10_nobar.so -DVSIQ_EXP_K10=1, and
# ... k10_nobar_nofold.so -DVSIQ_EXP_K10=3) and K9 (the default), two rounds interleaved.
set -e
mkdir -p gpurun_out
for r in 1 2; do
for v in k10 nobar nofold k9; do
  case $v in
    k10) E="C1_K10=1";; nobar) E="C1_K10=1 VSIQ_LIBRARY=tools/exp/so/k10_nobar.so";;
    nofold) E="C1_K10=1 VSIQ_LIBRARY=tools/exp/so/k10_nobar_nofold.so";; k9) E="C1_K10=0";;
  esac
  env $E timeout -k 10 120 python -u bench.py --workload c1 --steps 400 --no-cpu-baseline > gpurun_out/c1_${v}_$r.log 2>&1
done
done
