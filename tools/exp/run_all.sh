# GPU tests + the four bench workloads (one line each) -> gpurun_out/
set -o pipefail
R=${GRAFT_REPO_ROOT:-.}
cd $R
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/t_all.log 2>&1 || { echo "tests rc=$?"; exit 1; }
for W in c2 c3 c4 c5; do
  case $W in c4) S=20; WU=4;; c5) S=16; WU=2;; *) S=200; WU=20;; esac
  timeout -k 10 300 python3 -u bench.py --workload $W --steps $S --warmup $WU --no-cpu-baseline > gpurun_out/b_$W.log 2>&1 || { echo "bench $W rc=$?"; exit 1; }
done
