cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU -d gpurun_out/pmc_sq_c3 -o run --output-format csv -- python3 -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_sq_c3.log 2>&1
echo rc=$? >> gpurun_out/pmc_sq_c3.log
timeout -k 10 400 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_grbm_c3 -o run --output-format csv -- python3 -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_grbm_c3.log 2>&1
echo rc=$? >> gpurun_out/pmc_grbm_c3.log
