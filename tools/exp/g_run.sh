set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for W in c2 c5; do
VSIQ_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 4 --workload $W > gpurun_out/dist2_$W.log 2>&1 || { echo "$W rc=$?"; tail -30 gpurun_out/dist2_$W.log; exit 1; }
grep '^{' gpurun_out/dist2_$W.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], round(d['value']), d['config']['self_check'])"
done
