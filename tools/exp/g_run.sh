set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_parity.py tests/test_gpu_act.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest rc=$?; grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for G in 0 -1 0 -1; do
  timeout -k 10 200 python3 -u bench.py --workload c4 --steps 20 --warmup 4 --no-cpu-baseline --tune 11=$G > gpurun_out/c4g.log 2>&1 || { echo "$G rc=$?"; tail gpurun_out/c4g.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/c4g.log').read().strip().splitlines()[-1]); k=d['kernels']
print('gate $G', round(d['value']), {a:(round(b['avg_us'],1), round(b['frac'],3)) for a,b in k.items()})"
done
