#!/bin/bash
# Store cache-policy variants (VSIQ_ST_POLICY builds in expvar/) on the C2 headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in base ${VARIANTS:-st1 st2 st3 st4}; do
    if [ $v = base ]; then unset VSIQ_LIBRARY; else export VSIQ_LIBRARY=$PWD/expvar/$v.so; fi
    timeout -k 10 120 python3 -u bench.py --extras none --no-cpu-baseline --no-api ${BENCH_ARGS:-} > gpurun_out/st_$v.$rep.json 2> gpurun_out/st_$v.$rep.err || exit $?
    python3 -c "import json,sys;d=json.load(open('gpurun_out/st_$v.$rep.json'));k=d['kernels'];print('$v',$rep,round(d['ms_per_step']*1e3,2),{n:round(v['avg_us'],2) for n,v in k.items()},d['config']['self_check'])" | tee -a gpurun_out/st_policy.txt
  done
done
