set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for L in default tools/exp/_k1u1.so tools/exp/_k1u4.so tools/exp/_k1u8.so default; do
  if [ $L = default ]; then E=""; else E="VSIQ_LIBRARY=$L"; fi
  env $E timeout -k 10 200 python3 -u tools/exp/k1_bench.py > gpurun_out/k1.log 2>&1 || { echo "$L rc=$?"; tail gpurun_out/k1.log; exit 1; }
  grep "n=" gpurun_out/k1.log
done
