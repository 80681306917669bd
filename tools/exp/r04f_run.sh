set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_r04f.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/t_r04f.log; exit 1; }
tail -2 gpurun_out/t_r04f.log
timeout -k 10 300 python3 -u tools/exp/api_timings.py > gpurun_out/api_timings.log 2>&1 || { echo "api rc=$?"; tail gpurun_out/api_timings.log; exit 1; }
cat gpurun_out/api_timings.log
bash tools/exp/k4_variants_box.sh > gpurun_out/k4_variants.log 2>&1 || { echo "k4 variants rc=$?"; tail -20 gpurun_out/k4_variants.log; exit 1; }
cat gpurun_out/k4_variants.log
echo done
