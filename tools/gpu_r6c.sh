#!/bin/bash
# race screen (cp2 on the halo-store tests, then the whole suite), the
# store-wave A/B and the read-back ceiling A/B, one call
set -o pipefail
TAG=screen_r6 bash tools/race_screen_r6.sh || exit 1
echo SCREEN_OK
TAG=ab_sw bash tools/narrow_sw_ab_r6.sh || exit 1
TAG=ab_skip bash tools/readback_ab_r6.sh || exit 1
