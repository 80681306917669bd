set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 4 --bits-w 8 --bits-a 8 > gpurun_out/b_c4_w8a8.log 2>&1 || { echo bench rc=$?; tail gpurun_out/b_c4_w8a8.log; exit 1; }
tail -1 gpurun_out/b_c4_w8a8.log
