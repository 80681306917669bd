set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
for v in 0 1 2 3; do
  if [ $v = 0 ]; then unset VSIQ_LIBRARY; else export VSIQ_LIBRARY=$PWD/tools/exp/lib_k4_$v.so; fi
  timeout -k 10 200 python3 -u bench.py --workload c3 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/k4v_$v.log 2>&1 || exit 1
done
