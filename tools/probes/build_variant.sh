#!/bin/bash
# A library variant for A/B runs and race screens: every object rebuilt with
# extra defines in its own object directory (Makefile VARIANT / KNOBS);
# burg_build_flags() of the variant names the knobs.
#   tools/probes/build_variant.sh NAME "-DBURG_X=1 ..."  ->  finitedifference_amd/libburgers_hip_NAME.so
set -e
cd "$(dirname "$0")/../../finitedifference_amd/csrc"
make -s -j8 VARIANT="$1" KNOBS="$2"
echo built ../libburgers_hip_$1.so
