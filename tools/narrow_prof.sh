#!/bin/bash
# Where the pipe kernel's compute waves spend their clocks (a
# -DBURG_PIPE_PROF build, BURG_LIB): loop, store waits, readiness waits (by
# compute wave: a wave that waits less than its neighbours paces them), and
# the blocks that waited by missing kind -- for the 1024^2 9-mu sweep, one
# 1024^2 trajectory and the 4096^2 trajectory.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
X="--steps 2 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check"
for A in "--nx 1024 --sweep 9 --dt 0.05" "--nx 1024 --dt 0.05" "--nx 4096 --dt 0.0125"; do
  echo "== $A"
  BURG_STREAM_DEBUG=8 BURG_LIB=$R/finitedifference_amd/libburgers_hip_prof.so timeout -k 10 200 python bench.py $X $A 2>&1 | grep -E "\[pipe\]" | tail -3
done
