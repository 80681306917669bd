set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
i=0
for L in default tools/exp/_flat256.so tools/exp/_flat512.so; do
  i=$((i+1))
  if [ $L = default ]; then E=""; else E="VSIQ_LIBRARY=$L"; fi
  env $E timeout -k 10 200 python3 -u tools/exp/fold_bench.py > gpurun_out/flat_$i.log 2>&1 || { echo "$L rc=$?"; exit 1; }
  grep -v amdgpu.ids gpurun_out/flat_$i.log
done
