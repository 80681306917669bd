#!/bin/bash
# round 6 session g: smoke, full GPU suite, the default bench line (tools/gpu_round.sh),
# then the K11 kernel trace by grid.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_round.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06g_k11tr -o run --output-format csv \
    -- python3 -u tools/exp/k11_bench.py > gpurun_out/r06g_k11.log 2>&1 || exit 1
python3 tools/exp/trace_by_grid.py gpurun_out/r06g_k11tr k_mean > gpurun_out/r06g_k11_by_grid.txt || exit 1
rm -rf gpurun_out/r06g_k11tr
exit 0
