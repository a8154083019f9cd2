#!/bin/bash
# Race screen, round 6: the halo-store paths -- the
# multi-process slab tests, the multi-GPU drop-in and the paired slab test --
# once on the timing-perturbed build (comm wave at priority 2, above the
# compute waves: the build that exposed the store-VGPR hazard in round 5;
# make VARIANT=cp2 KNOBS=-DBURG_COMM_PRIO=2), then the whole suite on the
# default build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-screen_r6}; mkdir -p $O
BURG_LIB=$PWD/finitedifference_amd/libburgers_hip_cp2.so timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "slab_halo or fine750 or test_gpu_job or paired_slab or slab_wide" > $O/pytest_cp2_slabs.log 2>&1 || { tail -40 $O/pytest_cp2_slabs.log; exit 1; }
tail -2 $O/pytest_cp2_slabs.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
