set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --workload c1 --steps 200 --warmup 20 > gpurun_out/b_c1.log 2>&1 || { echo "c1 rc=$?"; tail gpurun_out/b_c1.log; exit 1; }
grep '^{' gpurun_out/b_c1.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1 -o run --output-format csv -- python3 -u bench.py --workload c1 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/p_c1.log 2>&1 || { echo "prof rc=$?"; exit 1; }
timeout -k 10 300 python3 -u tools/exp/pcm_bench.py > gpurun_out/pcm.log 2>&1 || { echo "pcm rc=$?"; tail gpurun_out/pcm.log; exit 1; }
grep -v amdgpu.ids gpurun_out/pcm.log
