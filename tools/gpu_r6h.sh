#!/bin/bash
# Round-6 evidence of the paired store wave build: rocprofv3 kernel stats of
# the default bench command and the HBM / clock passes of the 1024^2 9-mu
# sweep (b1) and one 1024^2 trajectory (bs) (tools/prof_r3.sh), then smoke,
# the default bench line and the N = 2 rehearsal (tools/gpu_r6.sh; the whole
# GPU suite ran on this build in tools/sw_cheap_ab_r6.sh)
set -o pipefail
export TMPDIR=/tmp
TAG=prof_r6h NAMES="b1 bs" bash tools/prof_r3.sh || exit 1
SKIP_SUITE=1 TAG=r6h bash tools/gpu_r6.sh || exit 1
