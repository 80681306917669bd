set -e
mkdir -p gpurun_out
o=gpurun_out/r02p_c1_sweep.txt
: > $o
run() { echo "== $*" >> $o; timeout -k 10 120 python -u bench.py --workload c1 --no-cpu-baseline --steps 400 "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), 'us/step', {k: round(v['avg_us'],2) for k,v in d['kernels'].items()})" >> $o; }
run
run --tune 7=1
for g in 1 2 4 16 32 64; do run --tune 7=2 --tune 8=$g; done
