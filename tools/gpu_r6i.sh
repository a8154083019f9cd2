#!/bin/bash
# Round-6 closing evidence of the final sources (the whole GPU suite ran on
# this build in tools/pair_traj_ab_r6.sh): smoke, rocprofv3 kernel stats of
# the default bench command and the 1024^2 sweep's HBM passes (tools/prof_r3.sh NAMES=b1), the default bench
# line and the N = 2 rehearsal (tools/gpu_r6.sh)
set -o pipefail
export TMPDIR=/tmp
TAG=prof_r6i NAMES="b1" bash tools/prof_r3.sh || exit 1
SKIP_SUITE=1 TAG=r6i bash tools/gpu_r6.sh || exit 1
