set -e
mkdir -p gpurun_out
for r in 1 2; do
for v in k10 nobar nofold k9; do
  case $v in
    k10) E="";; nobar) E="VSIQ_LIBRARY=tools/exp/so/k10_nobar.so";; nofold) E="VSIQ_LIBRARY=tools/exp/so/k10_nobar_nofold.so";; k9) E="C1_K9=1";;
  esac
  env $E timeout -k 10 120 python -u bench.py --workload c1 --steps 400 --no-cpu-baseline > gpurun_out/c1_${v}_$r.log 2>&1
done
done
