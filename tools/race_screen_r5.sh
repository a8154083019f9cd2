# Race screen: the whole GPU suite on a timing-perturbed build (comm wave at
# priority 2, above the compute waves)
set -o pipefail
O=gpurun_out/race_screen; mkdir -p $O
BURG_LIB=finitedifference_amd/libburgers_hip_cp2.so timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu_cp2.log 2>&1
rc=$?
tail -5 $O/pytest_gpu_cp2.log
exit $rc
