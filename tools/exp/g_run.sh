set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest rc=$?; grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_c2.log 2>&1 || { echo bench rc=$?; tail gpurun_out/b_c2.log; exit 1; }
python3 -c "
import json,sys; d=json.loads(open('gpurun_out/b_c2.log').read().strip().splitlines()[-1]); k=d['kernels']
print('c2', round(d['value']), 'fwd %.2f bwd %.2f frac %.3f' % (k['pc_observe_fq_fwd']['avg_us'], k['ste_bwd']['avg_us'], d['roofline']['frac']), d['config']['self_check'])"
done
