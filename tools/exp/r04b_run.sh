# round 4: public-API host trace (ours vs torch's trivial step), the default bench line,
# its kernel trace, and the C5 PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
MODE=api timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/trace_api -o run -- python3 -u tools/exp/api_trace.py > gpurun_out/trace_api.log 2>&1 || { echo "trace api rc=$?"; tail gpurun_out/trace_api.log; exit 1; }
MODE=torch timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/trace_torch -o run -- python3 -u tools/exp/api_trace.py > gpurun_out/trace_torch.log 2>&1 || { echo "trace torch rc=$?"; tail gpurun_out/trace_torch.log; exit 1; }
grep "us/step" gpurun_out/trace_api.log gpurun_out/trace_torch.log
python3 tools/exp/hip_api_summary.py gpurun_out/trace_api 700 > gpurun_out/hip_api_api.txt && python3 tools/exp/hip_api_summary.py gpurun_out/trace_torch 700 > gpurun_out/hip_api_torch.txt && cat gpurun_out/hip_api_api.txt gpurun_out/hip_api_torch.txt
MODE=api timeout -k 10 120 python3 -u tools/exp/api_trace.py > gpurun_out/free_api.log 2>&1 && MODE=torch timeout -k 10 120 python3 -u tools/exp/api_trace.py > gpurun_out/free_torch.log 2>&1 && cat gpurun_out/free_api.log gpurun_out/free_torch.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_default.log; exit 1; }
python3 tools/summarize_bench.py gpurun_out/bench_default.log > gpurun_out/bench_summary.txt 2>&1; cat gpurun_out/bench_summary.txt | head -40
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline --no-api > gpurun_out/prof_default.log 2>&1 || { echo "prof rc=$?"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C -d gpurun_out/pmc_c5_$C -o run --output-format csv -- python3 -u bench.py --workload c5 --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_c5_$C.log 2>&1 || { echo "pmc $C rc=$?"; exit 1; }
done
for B in 32 64 128; do
  BATCH=$B timeout -k 10 300 python3 -u tools/exp/model_step.py > gpurun_out/model_step_$B.log 2>&1 || { echo "model_step $B rc=$?"; tail gpurun_out/model_step_$B.log; exit 1; }
  cat gpurun_out/model_step_$B.log
done
echo done
