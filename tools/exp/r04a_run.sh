set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_silu.py tests/test_gpu_parity.py tests/test_gpu_model_launch.py tests/test_gpu_deferred_grads.py tests/test_gpu_multi.py tests/test_gpu_ddp_step.py tests/test_gpu_graph.py tests/test_gpu_bnfold_ckpt.py tests/test_gpu_c5_calib.py tests/test_gpu_bench_capture.py -x -q --timeout 120 --timeout-method thread -k "capture or c5 or silu_layout or parts_out or sym_tensor_zp or per_channel_learnable or model_launch or deferred or multi or ddp or graph or ckpt or state_dict or golden_per_channel" > gpurun_out/t_r04a.log 2>&1 || { echo "tests rc=$?"; tail -60 gpurun_out/t_r04a.log; exit 1; }
tail -3 gpurun_out/t_r04a.log
timeout -k 10 300 python -u tools/exp/act_mall.py > gpurun_out/act_mall.log 2>&1 && cat gpurun_out/act_mall.log && timeout -k 10 300 python -u tools/exp/c4_floor.py > gpurun_out/c4_floor.log 2>&1 && cat gpurun_out/c4_floor.log && timeout -k 10 300 python -u tools/exp/k2o_bench.py 20 > gpurun_out/k2o_bench.log 2>&1 || { echo "bench rc=$?"; tail gpurun_out/k2o_bench.log; exit 1; }
cat gpurun_out/k2o_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k2o -o run --output-format csv -- python3 -u tools/exp/k2o_bench.py 5 > gpurun_out/p_k2o.log 2>&1 || { echo "prof rc=$?"; exit 1; }
timeout -k 10 300 python3 -u bench.py --workload c5 --steps 32 --warmup 4 --no-cpu-baseline > gpurun_out/b_c5.log 2>&1 || { echo "bench c5 rc=$?"; tail gpurun_out/b_c5.log; exit 1; }
tail -1 gpurun_out/b_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['value'], d['ms_per_step'], d['roofline']['frac'], {k: (round(v['avg_us'],1), round(v['frac'],3)) for k,v in d['kernels'].items()}, d['config']['self_check'])"
echo done
