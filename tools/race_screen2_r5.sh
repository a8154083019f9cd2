# Race screens: the whole GPU suite on two more
# timing-perturbed builds -- loader waves above the compute waves (lp2), the
# compute waves at the comm / loader waves' priority (cp0) -- then the
# default build once more.
set -o pipefail
O=gpurun_out/race_screen2; mkdir -p $O
for v in lp2 cp0; do
  BURG_LIB=finitedifference_amd/libburgers_hip_$v.so timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_$v.log 2>&1 || { tail -20 $O/pytest_gpu_$v.log; exit 1; }
  tail -2 $O/pytest_gpu_$v.log
done
