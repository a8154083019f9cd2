#!/bin/bash
# Round-6 knob builds (rebuild after every source change: the GPU tests
# refuse a library whose build id differs from the sources)
set -e
cd "$(dirname "$0")/.."
make -s -j8 -C finitedifference_amd/csrc
tools/probes/build_variant.sh cp2 "-DBURG_COMM_PRIO=2"
tools/probes/build_variant.sh nochk "-DBURG_AB_NOCHECK"
for n in 32 64 128; do tools/probes/build_variant.sh nochk_skip$n "-DBURG_AB_NOCHECK -DBURG_AB_SKIP=$n"; done
tools/probes/build_variant.sh nosw "-DBURG_STORE_WAVE=0"
tools/probes/build_variant.sh swp2 "-DBURG_STOREWAVE_PRIO=2"
