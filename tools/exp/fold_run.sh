# K4 fold experiments: LSQ tests, per-size K4/K2 timing, C3/C4 bench lines
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_parity.py tests/test_gpu_act.py tests/test_gpu_lsq_module.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_k4.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_k4.log; exit 1; }
tail -1 gpurun_out/t_k4.log
timeout -k 10 200 python3 -u tools/exp/fold_bench.py > gpurun_out/fold_new.log 2>&1 || { echo "bench rc=$?"; exit 1; }
grep -v amdgpu.ids gpurun_out/fold_new.log
timeout -k 10 300 python3 -u bench.py --workload c4 --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/b_c4.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
timeout -k 10 300 python3 -u bench.py --workload c3 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b_c3.log 2>&1 || { echo "c3 rc=$?"; exit 1; }
grep -h '^{' gpurun_out/b_c4.log gpurun_out/b_c3.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['workload'][:30], round(d['ms_per_step'], 4), {k: (round(v['avg_us'], 1), round(v['frac'], 3)) for k, v in d['kernels'].items()})"
