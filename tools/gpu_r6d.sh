#!/bin/bash
# the store-wave build as the default: the whole suite; the narrow tests on
# the store wave at priority 2 (race screen); the read-back ceiling with the
# range check off; then the final build's profiles
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6d; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
BURG_LIB=$PWD/finitedifference_amd/libburgers_hip_swp2.so timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "pipe_1024 or pipe_bitwise_sequential or sweep_each or retained or slab_halo_two or run_fom or direct_npy or fine750" > $O/pytest_swp2.log 2>&1 || { tail -30 $O/pytest_swp2.log; exit 1; }
tail -1 $O/pytest_swp2.log
TAG=ab_skip2 bash tools/readback_ab_r6.sh || exit 1
