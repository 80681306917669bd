#!/bin/bash
# round 6 session y: rehearsal of bench.py's N > 1 path on the final tree -- two ranks
# sharing the box's one MI355X over gloo (VSIQ_BENCH_BACKEND=gloo), every leg run and
# self-checked (the driver's 8-GPU node runs the RCCL form).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp VSIQ_BENCH_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r06y_bench_n2_gloo.log 2>&1 \
    || { echo "n2 gloo failed"; tail -30 gpurun_out/r06y_bench_n2_gloo.log; exit 1; }
grep '"metric"' gpurun_out/r06y_bench_n2_gloo.log | cut -c1-300
grep "bench summary" gpurun_out/r06y_bench_n2_gloo.log | cut -c1-600
exit 0
