# On the GPU box: build K4 element-math variants of the product library (VSIQ_EXP_K4 bits:
# 1 = no f64 gradient accumulation, 2 = no fast-division range check) into /tmp and time
# K4d at the C4 sizes with each (tools/exp/c4_floor.py, VSIQ_LIBRARY).  Experiment only.
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for V in 1 2 3; do
  timeout -k 10 400 python3 tools/exp/build_variant.py /tmp/vsiq_k4_$V.so -DVSIQ_EXP_K4=$V > /tmp/bv_$V.log 2>&1 || { echo "build $V failed"; tail /tmp/bv_$V.log; exit 1; }
done
for V in 1 2 3; do
  echo "== VSIQ_EXP_K4=$V"
  VSIQ_LIBRARY=/tmp/vsiq_k4_$V.so timeout -k 10 300 python3 -u tools/exp/c4_floor.py || exit 1
done
