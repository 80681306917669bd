set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest rc=$?; grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for i in 1; do
timeout -k 10 300 python -u bench.py --workload c5 --steps 16 --warmup 2 > gpurun_out/b_c5.log 2>&1 || { echo bench rc=$?; tail gpurun_out/b_c5.log; exit 1; }
python3 -c "
import json,sys; d=json.loads(open('gpurun_out/b_c5.log').read().strip().splitlines()[-1]); k=d['kernels']
print('c5', round(d['value']), {a:(round(b['avg_us'],1), round(b['frac'],3)) for a,b in k.items()}, d['config']['self_check'])"
done
