set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u $R/bench.py --no-cpu-baseline > $R/gpurun_out/bd1.log 2>&1
timeout -k 10 200 python3 -u $R/tools/exp/order_bench.py > $R/gpurun_out/order2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_defer -o run --output-format csv -- python3 -u $R/bench.py --no-cpu-baseline > $R/gpurun_out/bd2.log 2>&1
