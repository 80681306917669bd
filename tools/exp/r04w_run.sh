# C3 K4 (in-kernel fold) groups per lane after the round-4 element work: 2 / 4 / 8 / 16 (default 8 at its size)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for rep in 1 2; do
  for G in 8 4 2 16; do
    echo -n "G=$G rep $rep: "
    timeout -k 10 300 python3 -u bench.py --workload c3 --steps 60 --warmup 5 --no-cpu-baseline --no-api --tune 9=$G 2>&1 | grep "bench summary" || exit 1
  done
done
