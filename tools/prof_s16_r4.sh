#!/bin/bash
# the N = 8 per-GPU slab (16384 x 2048, W = 512) of the round-4 build: kernel
# stats and the HBM / clock PMC passes (tools/prof_r3.sh NAMES=s16)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
NAMES="s16" NO_STATS=1 TAG=prof_r4c bash tools/prof_r3.sh || exit 1
echo NEXTOK
