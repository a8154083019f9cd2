#!/bin/bash
# Race screen of the store waves (round 6): the
# narrow-tile tests (paired and one-cell, sweeps, retained windows, slabs) on
# the build with the store wave above the compute waves (priority 2:
# make VARIANT=swp2 KNOBS=-DBURG_STOREWAVE_PRIO=2), then the whole suite on
# the default build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-screen_sw}; mkdir -p $O
BURG_LIB=$PWD/finitedifference_amd/libburgers_hip_swp2.so timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "pair or sweep or pipe_1024 or pipe_bitwise_sequential or retained or slab_halo or run_fom_main or direct_npy" > $O/pytest_swp2.log 2>&1 || { tail -40 $O/pytest_swp2.log; exit 1; }
tail -2 $O/pytest_swp2.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
