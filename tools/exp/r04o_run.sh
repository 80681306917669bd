# N > 1 rehearsal of the round-4 bench path: two ranks on one MI355X over gloo (the driver's
# N = 2..8 runs use RCCL, one GPU per rank), every leg self-checked; then --dry-run at N = 2.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
VSIQ_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_n2_gloo.log 2>&1 || { echo "n2 rc=$?"; tail -30 gpurun_out/bench_n2_gloo.log; exit 1; }
grep -E "bench summary|ranks_joined" gpurun_out/bench_n2_gloo.log | cut -c1-1500
echo done
