#!/bin/bash
# final round-4 check of the committed build: the full GPU suite, then smoke,
# the default bench line and the N = 2 rehearsals (tools/gpu_round4.sh)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r4zz
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_full.log 2>&1 || { tail -40 $O/pytest_gpu_full.log; exit 1; }
tail -2 $O/pytest_gpu_full.log
TAG=r4zz_round NO_MALL=1 bash tools/gpu_round4.sh || exit 1
echo NEXTOK
