cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "$n rc=$rc" | tee -a gpurun_out/steps.log; return $rc; }
run smoke2 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
run pytest2 900 python3 -u -m pytest tests -m gpu -x -q; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run tune 600 python3 -u tools/exp/tune.py || exit $?
run bench2 600 python3 -u bench.py || exit $?
