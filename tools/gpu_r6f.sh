#!/bin/bash
# DMA read-back off by default: race screens of the wide kernels and the halo
# paths with the loader (lp2) and the comm wave (cp2) above the compute
# waves, then the whole suite, smoke and the bench line on the default build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6f; mkdir -p $O
K="4096 or 8192 or wide or retained or slab or fine750 or test_gpu_job or reserve or trajectory"
for v in lp2 cp2; do
  BURG_LIB=$PWD/finitedifference_amd/libburgers_hip_$v.so timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
SKIP_BENCH= TAG=r6f bash tools/gpu_r6.sh || exit 1
