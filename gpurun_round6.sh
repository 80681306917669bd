cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "$n rc=$rc" | tee -a gpurun_out/steps.log; return $rc; }
run pytest6 900 python3 -u -m pytest tests -m gpu -x -q; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run pmc6b 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU -d gpurun_out/pmc6b -o run --output-format csv -- python3 -u bench.py --workload c3 --steps 4 --warmup 1 --no-cpu-baseline || exit $?
run bench6 600 python3 -u bench.py || exit $?
run bench6c3 600 python3 -u bench.py --workload c3 || exit $?
