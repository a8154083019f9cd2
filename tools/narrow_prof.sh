#!/bin/bash
# Where the 1024^2 9-mu sweep's compute waves spend their clocks (a
# -DBURG_PIPE_PROF build, BURG_LIB): loop, store waits, readiness waits, and
# the blocks that waited by missing kind.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
X="--nx 1024 --sweep 9 --dt 0.05 --steps 2 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e"
BURG_STREAM_DEBUG=8 BURG_LIB=$R/finitedifference_amd/libburgers_hip_prof.so timeout -k 10 200 python bench.py $X 2>&1 | grep -E "\[pipe\]|value" | cut -c1-200 | tail -8
BURG_STREAM_DEBUG=8 timeout -k 10 200 python bench.py $X --nx 4096 --sweep 1 --dt 0.0125 2>&1 | grep -E "\[pipe\]" | tail -2
