set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/t_fold.log 2>&1 || { echo tests failed; exit 1; }
for G in 0 2 4 16; do
  timeout -k 10 200 python3 -u bench.py --workload c3 --steps 100 --warmup 10 --no-cpu-baseline --tune 9=$G > gpurun_out/k4g_c3_$G.log 2>&1 || exit 1
  timeout -k 10 200 python3 -u bench.py --workload c4 --steps 20 --warmup 4 --no-cpu-baseline --tune 9=$G > gpurun_out/k4g_c4_$G.log 2>&1 || exit 1
done
timeout -k 10 200 python3 -u bench.py --workload c5 --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/k4g_c5.log 2>&1
