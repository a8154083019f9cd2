#!/bin/bash
# profiles of the final round-4 build: rocprofv3 kernel stats of the default
# bench command and of the POD probe (tools/prof_r3.sh, NAMES=pod)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
NAMES="pod" TAG=prof_r4b bash tools/prof_r3.sh || exit 1
echo NEXTOK
