# On the GPU box: build K4 element-math variants of the product library (VSIQ_EXP_K4_STEQ=0:
# grad_x by the general fast division as in round 3; VSIQ_EXP_K4 bits: 1 = no f64
# gradient accumulation, 2 = no fast-division range check) into /tmp and time
# K4d at the C4 sizes with each (tools/exp/c4_floor.py, VSIQ_LIBRARY).  Experiment only.
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
echo "== product library (grad_x by the one-step STE quotient)"
timeout -k 10 300 python3 -u tools/exp/c4_floor.py || exit 1
for V in "-DVSIQ_EXP_K4_STEQ=0" "-DVSIQ_EXP_K4=1" "-DVSIQ_EXP_K4=3"; do
  N=$(echo $V | tr -cd '0-9A-Z_' | tail -c 12)
  timeout -k 10 400 python3 tools/exp/build_variant.py /tmp/vsiq_k4_$N.so $V > /tmp/bv_$N.log 2>&1 || { echo "build $V failed"; tail /tmp/bv_$N.log; exit 1; }
  echo "== $V"
  VSIQ_LIBRARY=/tmp/vsiq_k4_$N.so timeout -k 10 300 python3 -u tools/exp/c4_floor.py || exit 1
done
