set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for L in default tools/exp/_k4gate.so default tools/exp/_k4gate.so; do
  if [ $L = default ]; then E=""; else E="VSIQ_LIBRARY=$L"; fi
  env $E SIZES="2097152 3276800 6553600 9437184 13107200" timeout -k 10 200 python3 -u tools/exp/fold_bench.py > gpurun_out/k4g.log 2>&1 || { echo "$L rc=$?"; tail gpurun_out/k4g.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/k4g.log
done
